#!/bin/bash
# Frame-kernel variant check: smoke and the parity suites with one variant
# forced on every batch (ZMQG_FRAMES_G=$1: 0 seq, 8 lds, 16 st), then
# config-2-shaped kernel timings of the default choice and the variant at
# the batch sizes given (default 65536).  Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
G=$1; shift
export ZMQG_FRAMES_G=$G
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/variant_smoke.log 2>&1 || { tail -30 gpurun_out/variant_smoke.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_boundary.py tests/test_zmtp.py tests/test_gpu_timed_path.py tests/test_gpu_verify_first.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_variant.log 2>&1 || { tail -40 gpurun_out/pytest_variant.log; exit 1; }
echo "G=$G: $(tail -1 gpurun_out/pytest_variant.log)"
unset ZMQG_FRAMES_G
for m in ${@:-65536}; do
  for r in 1 2; do
    timeout -k 10 120 python tools/kbench.py --iters 30 --msgs $m --tag default-$m || exit 1
    ZMQG_FRAMES_G=$G timeout -k 10 120 python tools/kbench.py --iters 30 --msgs $m --tag G$G-$m || exit 1
  done
done
