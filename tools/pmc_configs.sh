#!/bin/bash
# PMC pass (instruction mix, wave-cycle shares) and HBM bytes (FETCH_SIZE /
# WRITE_SIZE, passes of their own) over bench.py's BASELINE configs 3, 4, 5,
# one bench run per config and pass; tools/pmc_configs.py summarises the
# k_body / k_frames_* launches into gpurun_out/pmc_configs.json.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
A="SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM"
for c in ${CFGS:-3 4 5}; do
  p=0
  for C in "$A" "FETCH_SIZE" "WRITE_SIZE"; do
    p=$((p + 1))
    O=gpurun_out/pmcc/c$c/p$p
    mkdir -p $O
    timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $PWD/$O -o pmc -- \
        python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-host-staged --configs $c > $O/run.log 2>&1 \
        || { echo "pmc config $c pass $p failed"; tail -5 $O/run.log; exit 1; }
  done
done
python tools/pmc_configs.py gpurun_out/pmcc
