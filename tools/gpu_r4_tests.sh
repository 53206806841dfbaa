#!/bin/bash
# Round 4: the whole GPU suite (one process), smoke, per-message latency.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -3
[ $rc -ne 0 ] && { grep -B5 -A30 "FAILED\|Error" gpurun_out/pytest_gpu.log | head -80; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 120 ./build/msg_latency > gpurun_out/msg_latency.json 2>&1; echo "msg_latency rc=$?"; cat gpurun_out/msg_latency.json
