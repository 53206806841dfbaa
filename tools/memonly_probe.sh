#!/bin/bash
# memory-path-only timings (no Salsa20, no Poly1305: ZMQG_FRAMES_ABLATE=96
# builds) of the frame-kernel variants at config 2; outputs not checked
cd "${GRAFT_REPO_ROOT:-.}"
for lib in ab96_d1 ab96_d2; do
  ZMQG_CURVE_LIB=$PWD/build/libzmqg_$lib.so timeout -k 10 120 python tools/kbench.py --iters 20 --tag seq-$lib || exit 1
  ZMQG_FRAMES_G=8 ZMQG_CURVE_LIB=$PWD/build/libzmqg_$lib.so timeout -k 10 120 python tools/kbench.py --iters 20 --tag lds-$lib || exit 1
done
timeout -k 10 120 python tools/kbench.py --iters 20 --tag full-default || exit 1
ZMQG_FRAMES_G=8 timeout -k 10 120 python tools/kbench.py --iters 20 --tag full-lds || exit 1
