#!/bin/bash
# k_frames_st check and timing: parity suites with st forced, phase stamps,
# kernel timings of seq, st and the variant libraries given as arguments.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export ZMQG_FRAMES_G=16
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/variant_smoke.log 2>&1 || { tail -30 gpurun_out/variant_smoke.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_boundary.py tests/test_zmtp.py tests/test_gpu_timed_path.py tests/test_gpu_verify_first.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_variant.log 2>&1 || { tail -40 gpurun_out/pytest_variant.log; exit 1; }
echo "st: $(tail -1 gpurun_out/pytest_variant.log)"
unset ZMQG_FRAMES_G
if [ -x build/st_stamps ]; then timeout -k 10 60 build/st_stamps > gpurun_out/st_stamps.log 2>&1 || { cat gpurun_out/st_stamps.log; exit 1; }; cat gpurun_out/st_stamps.log; fi
for r in 1 2; do
  timeout -k 10 120 python tools/kbench.py --iters 30 --tag seq || exit 1
  ZMQG_FRAMES_G=16 timeout -k 10 120 python tools/kbench.py --iters 30 --tag st || exit 1
  for lib in "$@"; do
    ZMQG_FRAMES_G=16 ZMQG_CURVE_LIB=$PWD/$lib timeout -k 10 120 python tools/kbench.py --iters 30 --tag $lib || exit 1
  done
done
