#!/bin/bash
# PMC passes over k_body at the config-5 frame size (tools/kbench.py, 128 x
# 16 MiB, 8 sessions): instruction mix and wave-cycle shares (pass A), LDS and
# memory instruction detail (pass B), HBM bytes (FETCH_SIZE, WRITE_SIZE in
# passes of their own).  Summary: tools/pmc_body.py -> gpurun_out/pmc_body.json
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
SHAPE="--msgs ${MSGS:-128} --size ${SIZE:-16777216} --sessions ${SESS:-8}"
A="SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM"
B="SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVES"
i=0
for C in "$A" "$B" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i + 1))
  O=gpurun_out/pmcb/p$i
  mkdir -p $O
  timeout -s KILL 150 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $PWD/$O -o pmc -- \
      python tools/kbench.py --iters 2 $SHAPE --tag pmc$i > $O/run.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $O/run.log; exit 1; }
done
python tools/pmc_body.py gpurun_out/pmcb
