#!/bin/bash
# A variant build of the library (tools/bin/<lib>) against the default:
# parity suites with the variant, then config 2's decode resident (bench.py
# main line) and HBM-fed (tools/hbm_probe.py) with each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/vh
lib=$1
ZMQG_CURVE_LIB=$PWD/$lib timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_boundary.py tests/test_gpu_verify_first.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/vh/pytest.log 2>&1 || { tail -40 gpurun_out/vh/pytest.log; exit 1; }
echo "$lib: $(tail -1 gpurun_out/vh/pytest.log)"
for r in 1 2; do
  for L in default $lib; do
    if [ $L = default ]; then E=""; else E="ZMQG_CURVE_LIB=$PWD/$L"; fi
    env $E timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-staged --no-deployable --no-configs --hbm-sets 8 > gpurun_out/vh/bench_$r.log 2>&1 || { tail -20 gpurun_out/vh/bench_$r.log; exit 1; }
    tail -1 gpurun_out/vh/bench_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); h=d['hbm_fed']; print('$L', 'main', round(d['value'],1), 'dec_us', round(d['roofline']['avg_launch_us'],1), 'hbm', round(h['value'],1), 'enc_us', round(h['encode_us'],1), 'dec_us', round(h['decode_us'],1))"
  done
done
