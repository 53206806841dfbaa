#!/bin/bash
# ZMTP parity + timings and the per-message latency probe in one call.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_zmtp.py tests/test_host_adapter.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_misc.log 2>&1 || { tail -30 gpurun_out/pytest_misc.log; exit 1; }
tail -1 gpurun_out/pytest_misc.log
timeout -k 10 200 python tools/zmtp_bench.py || exit 1
timeout -k 10 200 ./build/msg_latency || exit 1
