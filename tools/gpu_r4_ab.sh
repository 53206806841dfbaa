#!/bin/bash
# Round 4: A/B of two library builds on the config-2 frame kernels (kbench,
# alternating, same box).  A = build/libzmqg_curve_r4a.so, B = the tree's.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for r in 1 2 3; do
  for lib in build/libzmqg_curve_r4a.so libzmq_amd/libzmqg_curve.so; do
    ZMQG_CURVE_LIB=$PWD/$lib timeout -k 10 120 python -u tools/kbench.py --tag $(basename $(dirname $lib))/$(basename $lib) > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
    tail -1 gpurun_out/ab.log
  done
done
timeout -k 10 300 python -u -m pytest tests/test_zmtp.py tests/test_gpu_timed_path.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1 || { tail -30 gpurun_out/pytest_ab.log; exit 1; }
tail -1 gpurun_out/pytest_ab.log
timeout -k 10 180 python -u tools/zmtp_bench.py 2>&1 | grep decode_zmtp
