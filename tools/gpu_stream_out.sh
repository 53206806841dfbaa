#!/bin/bash
# ZMQG_OPT_STREAM_OUT against the default stores: parity (the stream-out
# cases of tests/test_gpu_timed_path.py), then tools/hbm_probe.py's warm
# (MALL-resident) and bench (HBM-fed) forms with and without the hint,
# alternating, two rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
timeout -k 10 300 python -u -m pytest tests/test_gpu_timed_path.py -m gpu -x -q --timeout 120 --timeout-method thread 2>&1 | tail -1 || exit 1
for r in 1 2; do
  echo "default:"; timeout -k 10 200 python tools/hbm_probe.py --variants 0 --reps 2 --forms warm,bench 2>&1 | grep variant || exit 1
  echo "stream-out:"; timeout -k 10 200 python tools/hbm_probe.py --variants 0 --reps 2 --forms warm,bench --stream-out 2>&1 | grep variant || exit 1
done
