#!/bin/bash
# tools/hbm_probe.py with the address-order side prefetch at a few grid sizes.
cd "${GRAFT_REPO_ROOT:-.}"
set -o pipefail
timeout -k 10 200 python tools/hbm_probe.py --variants 0 --reps 2 || exit 1
for b in 256 1024 4096; do
  echo "stream prefetch, $b workgroups:"
  timeout -k 10 200 python tools/hbm_probe.py --variants 0 --reps 2 --stream-prefetch $b || exit 1
done
