#!/bin/bash
# Variant builds of the library (ZMQG_CURVE_LIB=each argument) against the
# default: parity suites with each variant, then config-2 kernel timings.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for lib in "$@"; do
  ZMQG_CURVE_LIB=$PWD/$lib timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_boundary.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_libvariant.log 2>&1 || { tail -40 gpurun_out/pytest_libvariant.log; exit 1; }
  echo "$lib: $(tail -1 gpurun_out/pytest_libvariant.log)"
done
for r in 1 2; do
  timeout -k 10 120 python tools/kbench.py --iters 30 --tag default || exit 1
  for lib in "$@"; do
    ZMQG_CURVE_LIB=$PWD/$lib timeout -k 10 120 python tools/kbench.py --iters 30 --tag $lib || exit 1
  done
done
