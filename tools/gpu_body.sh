#!/bin/bash
# Body-kernel change check: the GPU parity suites that run frames above the
# frame kernel's 4.5 KiB, the config-5 frame size timing, bench configs 3-5.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu ${TESTS:-tests} > gpurun_out/body_tests.log 2>&1
rc=$?
tail -5 gpurun_out/body_tests.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/body_tests.log | head -30; exit 1; }
timeout -k 10 180 python tools/kbench.py --iters 5 --msgs 128 --size 16777216 --sessions 8 --tag body || exit 1
timeout -k 10 400 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-staged > gpurun_out/body_bench.log 2>&1 || { tail -5 gpurun_out/body_bench.log; exit 1; }
tail -1 gpurun_out/body_bench.log
