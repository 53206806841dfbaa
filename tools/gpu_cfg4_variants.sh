#!/bin/bash
# Config-4-shaped (16 Mi x 256 B, 1024 sessions) frame-kernel timings per
# variant (ZMQG_FRAMES_G) and per library build given as arguments.
cd "${GRAFT_REPO_ROOT:-.}"
K="python tools/kbench.py --iters 5 --msgs 16777216 --size 256 --sessions 1024"
timeout -k 10 180 $K --tag default || exit 1
for g in 0 16 2; do
  ZMQG_FRAMES_G=$g timeout -k 10 180 $K --tag G=$g || exit 1
done
for lib in "$@"; do
  ZMQG_FRAMES_G=0 ZMQG_CURVE_LIB=$PWD/$lib timeout -k 10 180 $K --tag "$lib G=0" || exit 1
done
