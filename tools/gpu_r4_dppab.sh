#!/bin/bash
# Round 4: the frame kernels' prologue reductions on DPP -- the whole GPU
# suite, then the config-2 frame-kernel A/B against the build before
# (tools/gpu_r4_ab.sh).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && { grep -B5 -A30 "FAILED\|Error" gpurun_out/pytest_gpu.log | head -60; exit 1; }
bash tools/gpu_r4_ab.sh
