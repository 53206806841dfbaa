#!/bin/bash
# k_frames_seq variant check: parity suites with the one-lane kernel forced on
# every batch (ZMQG_FRAMES_G=0) for each library build given, then config-2
# kernel timings of the default build and each variant (twice, interleaved).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for lib in "$@"; do
  ZMQG_CURVE_LIB=$PWD/$lib ZMQG_FRAMES_G=0 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_boundary.py tests/test_zmtp.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_seqvariant.log 2>&1 || { tail -40 gpurun_out/pytest_seqvariant.log; exit 1; }
  echo "$lib: $(tail -1 gpurun_out/pytest_seqvariant.log)"
done
for r in 1 2; do
  timeout -k 10 120 python tools/kbench.py --iters 30 --tag default || exit 1
  for lib in "$@"; do
    ZMQG_CURVE_LIB=$PWD/$lib timeout -k 10 120 python tools/kbench.py --iters 30 --tag $lib || exit 1
  done
done
