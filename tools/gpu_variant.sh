#!/bin/bash
# Frame-kernel variant check on the GPU: the parity suites with the variant
# forced on every batch (ZMQG_FRAMES_G=$1), then config-2 kernel timings of
# the default choice and of the variant.  Usage: tools/gpu_variant.sh G
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
G=${1:-8}
ZMQG_FRAMES_G=$G timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_boundary.py tests/test_gpu_nonce.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_variant.log 2>&1 || { tail -40 gpurun_out/pytest_variant.log; exit 1; }
tail -2 gpurun_out/pytest_variant.log
timeout -k 10 120 python tools/kbench.py --iters 30 --tag default || exit 1
ZMQG_FRAMES_G=$G timeout -k 10 120 python tools/kbench.py --iters 30 --tag G$G || exit 1
ZMQG_FRAMES_G=$G timeout -k 10 120 python tools/kbench.py --iters 10 --msgs 1048576 --size 256 --tag G$G-256B || exit 1
timeout -k 10 120 python tools/kbench.py --iters 10 --msgs 1048576 --size 256 --tag default-256B || exit 1
