#!/bin/bash
# Round 4: per-message path -- its tests, the latency tool, and k_msg's kernel
# durations (rocprofv3 kernel trace).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/prof_msg
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_msg.py tests/test_host_adapter.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_msg.log 2>&1 || { tail -30 gpurun_out/pytest_msg.log; exit 1; }
tail -1 gpurun_out/pytest_msg.log
timeout -k 10 120 ./build/msg_latency > gpurun_out/msg_latency.json 2>&1 || exit 1
cat gpurun_out/msg_latency.json
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_msg -o msg --output-format csv -- ./build/msg_latency > /dev/null 2>&1 || exit 1
grep k_msg gpurun_out/prof_msg/msg_kernel_stats.csv | cut -d, -f1-4,6,7
