#!/bin/bash
# k_body A/B: GPU suite on the default build, then configs 3 and 5 through
# bench.py for the default build and the library given as argument, twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_body.log 2>&1 || { tail -40 gpurun_out/pytest_body.log; exit 1; }
tail -1 gpurun_out/pytest_body.log
for r in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 5 --warmup 2 --no-cpu-baseline --no-host-staged --configs 3,5 || exit 1
  ZMQG_CURVE_LIB=$PWD/$1 timeout -k 10 300 python bench.py --gpus 1 --steps 5 --warmup 2 --no-cpu-baseline --no-host-staged --configs 3,5 || exit 1
done
