#!/bin/bash
# Instruction-cache counters of the frame kernels: config 2 (one wave per
# SIMD) and twice the frames (two waves per SIMD, k_frames_seq forced).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/icache
for m in 65536 131072; do
  ZMQG_FRAMES_G=0 timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_INSTS_VALU SQ_WAVES -d $PWD/gpurun_out/icache/m$m -o run --output-format csv -- python tools/kbench.py --iters 3 --msgs $m --tag m$m || exit 1
done
