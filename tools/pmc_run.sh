#!/bin/bash
# PMC counter collection (own run, kernel-trace only) for the body kernels.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
timeout -k 10 300 rocprofv3 -i tools/pmc_body.txt --kernel-trace --output-format csv -d $PWD/gpurun_out/pmc -o pmc -- python tools/kbench.py --iters 3 "$@" > gpurun_out/pmc/run.log 2>&1
rc=$?
tail -3 gpurun_out/pmc/run.log
ls gpurun_out/pmc | head -20
exit $rc
