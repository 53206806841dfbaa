#!/bin/bash
# Config 2 resident (bench.py main line) and HBM-fed (hbm_fed) decode/encode
# for several library builds (tools/bin/*.so given as arguments), alternating
# over two rounds on one box; parity suites first for the first argument.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/vt
ZMQG_CURVE_LIB=$PWD/$1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_boundary.py tests/test_gpu_verify_first.py tests/test_gpu_variant_bounds.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/vt/pytest.log 2>&1 || { tail -40 gpurun_out/vt/pytest.log; exit 1; }
echo "$1: $(tail -1 gpurun_out/vt/pytest.log)"
for r in 1 2; do
  for L in "$@"; do
    ZMQG_CURVE_LIB=$PWD/$L timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-staged --no-deployable --no-configs --hbm-sets 8 > gpurun_out/vt/bench.log 2>&1 || { tail -20 gpurun_out/vt/bench.log; exit 1; }
    tail -1 gpurun_out/vt/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); h=d['hbm_fed']; print('$L', 'main', round(d['value'],1), 'dec_us', round(d['roofline']['avg_launch_us'],1), 'hbm', round(h['value'],1), 'enc_us', round(h['encode_us'],1), 'dec_us', round(h['decode_us'],1))"
  done
done
