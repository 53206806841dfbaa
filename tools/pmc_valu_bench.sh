#!/bin/bash
# VALU instruction counts of the bench's frame kernels and where their wave
# cycles go: two rocprofv3 --pmc passes (kernel-trace only) over python bench.py --eager; summarised into
# profiles/pmc_valu_config2.json by tools/pmc_valu_summary.py.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/pmcv
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-trace --output-format csv -d $PWD/$O -o pmc -- \
    python bench.py --eager --steps 3 --warmup 1 --settle-ms 0 --no-cpu-baseline --no-host-staged --no-configs --no-deployable --hbm-sets 0 > $O/run.log 2>&1 || { echo "valu pass failed"; tail -5 $O/run.log; exit 1; }
python tools/pmc_valu_summary.py $O > $O/summary.json && cat $O/summary.json
# where the waves' cycles go: issuing, waiting at s_waitcnt, stalled at issue
# (disjoint: ACTIVE_INST_ANY + WAIT_ANY + WAIT_INST_ANY ~ WAVE_CYCLES)
S=gpurun_out/pmcs
mkdir -p $S
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY --kernel-trace --output-format csv -d $PWD/$S -o pmc -- \
    python bench.py --eager --steps 3 --warmup 1 --settle-ms 0 --no-cpu-baseline --no-host-staged --no-configs --no-deployable --hbm-sets 0 > $S/run.log 2>&1 || { echo "stall pass failed"; tail -5 $S/run.log; exit 1; }
python tools/pmc_valu_summary.py $S > $S/summary.json && cat $S/summary.json
