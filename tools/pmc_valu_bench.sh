#!/bin/bash
# VALU instruction counts of the bench's frame kernels: one rocprofv3 --pmc
# pass (kernel-trace only) over python bench.py --eager; summarised into
# profiles/pmc_valu_config2.json by tools/pmc_valu_summary.py.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/pmcv
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-trace --output-format csv -d $PWD/$O -o pmc -- \
    python bench.py --eager --steps 3 --warmup 1 --no-cpu-baseline --no-host-staged --no-configs > $O/run.log 2>&1 || { echo "valu pass failed"; tail -5 $O/run.log; exit 1; }
python tools/pmc_valu_summary.py $O > $O/summary.json && cat $O/summary.json
