#!/bin/bash
# ZMQG_OPT_STREAM_OUT: parity (tests/test_gpu_timed_path.py), then the
# bench's main line (MALL-resident, graph replays) with and without the
# hint on its decodes, alternating, two rounds (hbm_fed always uses it).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_timed_path.py -m gpu -x -q --timeout 120 --timeout-method thread 2>&1 | tail -1 || exit 1
for r in 1 2; do
  for so in "" "--stream-out"; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-staged --no-deployable --no-configs --hbm-sets 8 $so > gpurun_out/so.log 2>&1 || { tail -20 gpurun_out/so.log; exit 1; }
    tail -1 gpurun_out/so.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); h=d['hbm_fed']; print('main${so:+ stream-out}', round(d['value'],1), 'dec_us', round(d['roofline']['avg_launch_us'],1), 'enc_us', round(d['roofline']['encode_main_avg_us'],1), 'hbm', round(h['value'],1), 'dec_us', round(h['decode_us'],1))"
  done
done
