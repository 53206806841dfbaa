#!/bin/bash
# Round 4: the ZMTP receive side -- its tests and the synchronous
# decode_zmtp timing (tools/zmtp_bench.py), then a kernel trace of it.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/zprof4
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_zmtp.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_zmtp.log 2>&1 || { tail -40 gpurun_out/pytest_zmtp.log; exit 1; }
tail -3 gpurun_out/pytest_zmtp.log
for r in 1 2; do
timeout -k 10 180 python -u tools/zmtp_bench.py > gpurun_out/zmtp_bench.log 2>&1 || { cat gpurun_out/zmtp_bench.log; exit 1; }
cat gpurun_out/zmtp_bench.log
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/zprof4 -o run --output-format csv -- python -u tools/zmtp_bench.py > gpurun_out/zprof4.log 2>&1 || { tail -20 gpurun_out/zprof4.log; exit 1; }
grep -E "zmtp|k_frames_seq|k_body|k_post" gpurun_out/zprof4/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-160
