#!/bin/bash
# k_frames_lds layouts (build/libzmqg_s<sector>b<buffers>.so) at config 2 and
# 1 Mi x 256 B: parity with the kernel forced, timings, and WRITE_SIZE
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in build/libzmqg_s64b1.so build/libzmqg_s64b2.so; do
  ZMQG_FRAMES_G=8 ZMQG_CURVE_LIB=$PWD/$lib timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_boundary.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_lds.log 2>&1 || { tail -40 gpurun_out/pytest_lds.log; exit 1; }
  echo "$lib: $(tail -1 gpurun_out/pytest_lds.log)"
done
for r in 1 2; do
  timeout -k 10 120 python tools/kbench.py --iters 30 --tag seq || exit 1
  for lib in build/libzmqg_s16b2.so build/libzmqg_s64b1.so build/libzmqg_s64b2.so; do
    ZMQG_FRAMES_G=8 ZMQG_CURVE_LIB=$PWD/$lib timeout -k 10 120 python tools/kbench.py --iters 30 --tag $lib || exit 1
  done
done
for lib in build/libzmqg_s16b2.so build/libzmqg_s64b1.so; do
  ZMQG_CURVE_LIB=$PWD/$lib timeout -k 10 120 python tools/kbench.py --iters 10 --msgs 1048576 --size 256 --tag 256B-$lib || exit 1
done
O=gpurun_out/pmct_s64
ZMQG_FRAMES_G=8 ZMQG_CURVE_LIB=$PWD/build/libzmqg_s64b1.so timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $PWD/$O/write -o pmc -- python tools/kbench.py --iters 3 > $O.log 2>&1 || exit 1
echo done
