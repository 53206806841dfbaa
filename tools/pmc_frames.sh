#!/bin/bash
# PMC passes over the library's frame kernels (config 2 via tools/kbench.py),
# one rocprofv3 run per counter group (MI355X_MICROARCH.md: separate passes).
# Usage: tools/pmc_frames.sh OUTDIR [kbench args]
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
out=$1; shift
mkdir -p $out
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $PWD/$out/p$i -o pmc -- python3 tools/kbench.py "$@" > $out/p$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pmc pass $i failed rc=$rc"; tail -5 $out/p$i.log; exit 1; fi
done
echo pmc done
