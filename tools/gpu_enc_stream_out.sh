#!/bin/bash
# Encode under ZMQG_OPT_STREAM_OUT: its parity tests,
# then config 2's encodes timed HBM-fed (8 sets) and cache-resident (1 set),
# with and without the hint, k_frames_seq (tools/hbm_probe.py --time-enc).
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/enc_so.log
: > $L
timeout -k 10 300 python -u -m pytest tests/test_gpu_timed_path.py -x -v --timeout 120 --timeout-method thread \
    -k "stream_out" >> $L 2>&1 || exit 1
for sets in 8 1; do
  for so in "" "--enc-stream-out"; do
    echo "== sets $sets $so" >> $L
    timeout -k 10 180 python -u tools/hbm_probe.py --variants 0 --forms bench --stream-out --time-enc --sets $sets \
        --reps 4 $so >> $L 2>&1 || exit 1
  done
done
for so in "" "--enc-stream-out"; do
  echo "== sets 8 again $so" >> $L
  timeout -k 10 180 python -u tools/hbm_probe.py --variants 0 --forms bench --stream-out --time-enc --sets 8 \
      --reps 4 $so >> $L 2>&1 || exit 1
done
