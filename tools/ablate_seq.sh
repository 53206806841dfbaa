#!/bin/bash
# Timing ablations of k_frames_seq (config 2): tools/bin/libzmqg_ab<V>.so built
# with -DZMQG_FRAMES_ABLATE=V (see curve_frames.hpp); outputs are not checked.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 120 python tools/kbench.py --iters 30 --tag base || exit 1
for v in 8 16 24 32 64 96 120; do
  ZMQG_CURVE_LIB=$PWD/tools/bin/libzmqg_ab$v.so timeout -k 10 120 python tools/kbench.py --iters 30 --tag ab$v || exit 1
done
