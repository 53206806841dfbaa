#!/bin/bash
# quick k_frames_st timing: stamps of the default and register-staged builds,
# then kbench of seq, st (default library) and the libraries given.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for b in build/st_stamps build/st_stamps_reg; do
  [ -x $b ] || continue
  echo "== $b"; timeout -k 10 60 $b 2>&1 | grep -E "waves|K=3|lifetime|encode|decode|^  [ 0-9]: " || exit 1
done
for r in 1 2; do
  timeout -k 10 120 python tools/kbench.py --iters 30 --tag seq || exit 1
  ZMQG_FRAMES_G=16 timeout -k 10 120 python tools/kbench.py --iters 30 --tag st || exit 1
  for lib in "$@"; do
    ZMQG_FRAMES_G=16 ZMQG_CURVE_LIB=$PWD/$lib timeout -k 10 120 python tools/kbench.py --iters 30 --tag $lib || exit 1
  done
done
