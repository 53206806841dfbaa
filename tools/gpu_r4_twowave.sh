#!/bin/bash
# Round 4: does a second wave per SIMD pay for the one-lane-per-frame kernel?
# The same 64 MiB of payload as config 2, as 65,536 x 1 KiB (one wave per
# SIMD, 17 windows a lane) and as 131,072 x 512 B (two waves per SIMD, 9
# windows a lane), each variant forced (ZMQG_FRAMES_G: 0 seq, 8 lds, 2 two
# lanes a frame), two rounds.
cd "${GRAFT_REPO_ROOT:-.}"
for r in 1 2; do
  for g in 0 8; do
    ZMQG_FRAMES_G=$g timeout -k 10 120 python tools/kbench.py --iters 30 --msgs 65536 --size 1024 --tag G$g-65536x1024 || exit 1
    ZMQG_FRAMES_G=$g timeout -k 10 120 python tools/kbench.py --iters 30 --msgs 131072 --size 512 --tag G$g-131072x512 || exit 1
    ZMQG_FRAMES_G=$g timeout -k 10 120 python tools/kbench.py --iters 30 --msgs 262144 --size 256 --tag G$g-262144x256 || exit 1
  done
  ZMQG_FRAMES_G=2 timeout -k 10 120 python tools/kbench.py --iters 30 --msgs 65536 --size 1024 --tag G2-65536x1024 || exit 1
done
