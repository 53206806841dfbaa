#!/bin/bash
# Round 4: config 4 (16 Mi x 256 B, 1,024 sessions) frame kernels of two
# library builds alternating on one box (A = build/libzmqg_curve_r4a.so, B =
# the tree's), after the whole GPU suite on B.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && { grep -B5 -A30 "FAILED\|Error" gpurun_out/pytest_gpu.log | head -60; exit 1; }
for r in 1 2 3; do
  for lib in build/libzmqg_curve_r4a.so libzmq_amd/libzmqg_curve.so; do
    ZMQG_CURVE_LIB=$PWD/$lib timeout -k 10 180 python -u tools/kbench.py --msgs 16777216 --size 256 --sessions 1024 --iters 5 --tag $(basename $(dirname $lib)) > gpurun_out/cfg4ab.log 2>&1 || { tail -20 gpurun_out/cfg4ab.log; exit 1; }
    tail -1 gpurun_out/cfg4ab.log
  done
done
