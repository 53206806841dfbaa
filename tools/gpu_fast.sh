#!/bin/bash
# Straight-line interior steps (ZMQG_SEQ_FAST): parity of the default build,
# then config-2 kernel timings of the default build against the given ones.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_fast.log 2>&1 || { tail -40 gpurun_out/pytest_fast.log; exit 1; }
tail -1 gpurun_out/pytest_fast.log
for r in 1 2; do
  timeout -k 10 120 python tools/kbench.py --iters 30 --tag default || exit 1
  for lib in "$@"; do
    ZMQG_CURVE_LIB=$PWD/$lib timeout -k 10 120 python tools/kbench.py --iters 30 --tag $lib || exit 1
  done
done
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-host-staged --no-configs || exit 1
