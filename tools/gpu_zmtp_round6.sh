#!/bin/bash
# Round 6, DESIGN.md section 7: the ZMTP parse's parity suite, then
# tools/zmtp_bench.py twice and once under a kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/zr; rm -rf gpurun_out/zr/prof
timeout -k 10 300 python -u -m pytest tests/test_zmtp.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/zr/pytest.log 2>&1 || { tail -30 gpurun_out/zr/pytest.log; exit 1; }
tail -1 gpurun_out/zr/pytest.log
ZMQG_ZMTP_CUB=1 timeout -k 10 300 python -u -m pytest tests/test_zmtp.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/zr/pytest_cub.log 2>&1 || { tail -30 gpurun_out/zr/pytest_cub.log; exit 1; }
echo "cub: $(tail -1 gpurun_out/zr/pytest_cub.log)"
for r in 1 2; do
  timeout -k 10 120 python tools/zmtp_bench.py > gpurun_out/zr/bench_$r.log 2>&1 || { cat gpurun_out/zr/bench_$r.log; exit 1; }
  echo "run $r: $(tail -4 gpurun_out/zr/bench_$r.log | tr '\n' ' ')"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/zr/prof -o zr -- python3 $GRAFT_REPO_ROOT/tools/zmtp_bench.py > $GRAFT_REPO_ROOT/gpurun_out/zr/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/zr/prof.log; exit 1; }
echo done
