#!/bin/bash
# Round 4: the ZMTP receive side's fused middle (k_zmtp_chain) -- its tests,
# the synchronous decode_zmtp timing, and a kernel trace of the bench.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/zprof4
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_zmtp.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_zmtp.log 2>&1 || { tail -40 gpurun_out/pytest_zmtp.log; exit 1; }
tail -3 gpurun_out/pytest_zmtp.log
timeout -k 10 180 python -u tools/zmtp_bench.py > gpurun_out/zmtp_bench.log 2>&1 || { cat gpurun_out/zmtp_bench.log; exit 1; }
cat gpurun_out/zmtp_bench.log
ZMQG_ZMTP_CLK=1 timeout -k 10 120 python -u tools/zmtp_bench.py > gpurun_out/zmtp_clk.log 2>&1 || { tail -20 gpurun_out/zmtp_clk.log; exit 1; }
grep -m3 zmtp_chain gpurun_out/zmtp_clk.log; tail -2 gpurun_out/zmtp_clk.log
ZMQG_ZMTP_SPLIT=1 timeout -k 10 120 python -u tools/zmtp_bench.py > gpurun_out/zmtp_split.log 2>&1 || { tail -20 gpurun_out/zmtp_split.log; exit 1; }
ZMQG_ZMTP_SCAN1=1 timeout -k 10 120 python -u tools/zmtp_bench.py > gpurun_out/zmtp_scan1.log 2>&1 || { tail -20 gpurun_out/zmtp_scan1.log; exit 1; }
echo "scan1:"; tail -1 gpurun_out/zmtp_scan1.log
echo "split:"; tail -1 gpurun_out/zmtp_split.log
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/zprof4 -o run --output-format csv -- python -u tools/zmtp_bench.py > gpurun_out/zprof4.log 2>&1 || { tail -20 gpurun_out/zprof4.log; exit 1; }
grep -E "zmtp|k_frames_seq|k_body|k_post" gpurun_out/zprof4/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-160
