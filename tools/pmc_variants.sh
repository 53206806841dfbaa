#!/bin/bash
# VALU instruction counts and busy cycles of the frame kernels for every
# build/libzmqg_curve_*.so (one rocprofv3 --pmc pass per build, kbench workload).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
for lib in build/libzmqg_curve_*.so; do
  tag=$(basename $lib .so)
  export ZMQG_CURVE_LIB=$PWD/$lib
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $PWD/gpurun_out/pv/$tag -o pmc -- python tools/kbench.py --iters 3 > gpurun_out/pv_$tag.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "$tag failed rc=$rc"; tail -5 gpurun_out/pv_$tag.log; exit 1; fi
done
echo done
