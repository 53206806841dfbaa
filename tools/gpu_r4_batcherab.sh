#!/bin/bash
# Round 4: curve_batcher_t with the slot's longest frame passed as max_len
# (B, build/batcher_bench) against the build before (A,
# build/batcher_bench_A), after the host-adapter GPU tests.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_host_adapter.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_adapter.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_adapter.log; [ $rc -ne 0 ] && { tail -40 gpurun_out/pytest_adapter.log; exit 1; }
for r in 1 2; do
  for b in batcher_bench_A batcher_bench; do
    echo "== $b"; timeout -k 10 200 ./build/$b || exit 1
  done
done
