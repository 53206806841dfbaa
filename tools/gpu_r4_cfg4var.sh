#!/bin/bash
# Round 4: config 4 as bench.py runs it (16 Mi x 256 B, 1,024 sessions,
# device nonces, max_len bound) with the library's variant choice against
# k_frames_seq and k_frames_lds forced, two rounds.
cd "${GRAFT_REPO_ROOT:-.}"
for r in 1 2; do
  for g in default 0 8; do
    if [ $g = default ]; then unset ZMQG_FRAMES_G; else export ZMQG_FRAMES_G=$g; fi
    timeout -k 10 300 python bench.py --steps 5 --warmup 2 --configs 4 --no-cpu-baseline --no-host-staged 2>/dev/null \
      | python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); c=d['configs']['config4']; print('G=$g', 'config4', round(c['value'],1), 'GiB/s', round(c['ms_per_step'],3), 'ms/step')" || exit 1
  done
done
