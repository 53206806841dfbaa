#!/bin/bash
# PMC passes (one rocprofv3 run per counter group) over a prototype binary.
# usage: tools/pmc_proto.sh OUTDIR -- cmd args...
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=$1; shift; shift
mkdir -p $OUT
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $PWD/$OUT/p$i -o pmc -- "$@" > $OUT/p$i.log 2>&1 || { echo "pass $i failed rc=$?"; tail -3 $OUT/p$i.log; exit 1; }
done
echo done
