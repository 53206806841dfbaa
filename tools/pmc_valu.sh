#!/bin/bash
# SQ_INSTS_VALU / SQ_WAVE_CYCLES / GRBM_GUI_ACTIVE per kernel for each given binary (one pass each)
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
for b in "$@"; do
  n=$(basename $b)
  FB_ENC2_ONLY=1 timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $PWD/gpurun_out/pv/$n -o pmc -- $b > gpurun_out/pv_$n.log 2>&1
  rc=$?  # (ablation builds compute wrong bytes and exit 2: fine; a kill or crash is not)
  if [ $rc -ge 124 ]; then echo "$n failed rc=$rc"; exit 1; fi
done
echo done
