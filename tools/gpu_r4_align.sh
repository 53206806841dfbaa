#!/bin/bash
# Round 4: config-2 frame kernels with the wire frames packed (1,057-byte
# stride) against 64-byte-aligned wire frames (1,088-byte stride), kbench,
# alternating on one box.
cd "${GRAFT_REPO_ROOT:-.}"
for r in 1 2 3; do
  for al in 1 64; do
    timeout -k 10 120 python -u tools/kbench.py --wire-align $al --tag align$al 2>&1 | tail -1 || exit 1
  done
done
