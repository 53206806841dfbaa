#!/bin/bash
# timing experiment: every build/libzmqg_curve_<variant>.so through tools/kbench.py
# (outputs checked: "ok" in each line).  Stops at the first fault/timeout.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for lib in build/libzmqg_curve_*.so; do
  ZMQG_CURVE_LIB=$PWD/$lib timeout -k 10 120 python tools/kbench.py "$@" 2>&1 | grep -v amdgpu.ids
  rc=${PIPESTATUS[0]}; [ $rc -ne 0 ] && { echo "rc=$rc at $lib"; exit $rc; }
done
exit 0
