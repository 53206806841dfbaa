#!/bin/bash
# timing experiment: production build vs ablation builds (see Makefile "ablate")
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for lib in libzmq_amd/libzmqg_curve.so build/libzmqg_curve_ablate2.so build/libzmqg_curve_ablate3.so build/libzmqg_curve_ablate4.so build/libzmqg_curve_ablate5.so; do
  ZMQG_CURVE_LIB=$PWD/$lib timeout -k 10 120 python tools/kbench.py "$@" || exit $?
done
