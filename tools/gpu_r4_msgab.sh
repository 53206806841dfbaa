#!/bin/bash
# Round 4: per-call time of two per-message builds, alternating on one box
# (A = build/msgA/libzmqg_curve.so, B = the tree's).
cd "${GRAFT_REPO_ROOT:-.}"
for r in 1 2 3; do
  for D in $PWD/build/msgA $PWD/libzmq_amd; do
    LD_LIBRARY_PATH=$D:$LD_LIBRARY_PATH timeout -k 10 120 ./build/msg_kernel_bench $(basename $D) || exit 1
  done
done
