#!/bin/bash
# Parity of the default (max-ilp) build, then kernel timings against variants.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_sched.log 2>&1 || { tail -40 gpurun_out/pytest_sched.log; exit 1; }
tail -1 gpurun_out/pytest_sched.log
bash tools/gpu_libtime.sh "$@"
