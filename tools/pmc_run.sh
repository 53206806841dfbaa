#!/bin/bash
# PMC counter collection (own run, kernel-trace only) for the body kernels.
# usage: pmc_run.sh [lib.so] -- extra kbench args
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
LIB=${1:-libzmq_amd/libzmqg_curve.so}; shift || true
TAG=$(basename $LIB .so)
mkdir -p gpurun_out/pmc_$TAG
ZMQG_CURVE_LIB=$PWD/$LIB timeout -k 10 300 rocprofv3 -i tools/pmc_body.txt --kernel-trace --output-format csv -d $PWD/gpurun_out/pmc_$TAG -o pmc -- python tools/kbench.py --iters 3 "$@" > gpurun_out/pmc_$TAG/run.log 2>&1
rc=$?
tail -2 gpurun_out/pmc_$TAG/run.log
exit $rc
