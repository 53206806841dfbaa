#!/bin/bash
# Config-2 kernel timings of the default build against variant builds given
# as arguments (tools/bin/libzmqg_*.so), twice, interleaved; outputs not checked.
cd "${GRAFT_REPO_ROOT:-.}"
for r in 1 2; do
  timeout -k 10 120 python tools/kbench.py --iters 30 --tag default || exit 1
  for lib in "$@"; do
    ZMQG_CURVE_LIB=$PWD/$lib timeout -k 10 120 python tools/kbench.py --iters 30 --tag $lib || exit 1
  done
done
