#!/bin/bash
# Config 4's frame kernels under PMC (one rocprofv3 pass per counter group,
# kernel-trace only): instruction mix and issue stalls, then HBM bytes
# (FETCH_SIZE, WRITE_SIZE passes of their own).  Output gpurun_out/pmc4/p*/;
# tools/pmc4_summary.py turns it into per-launch figures stamped with the
# library's source id.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
A="SQ_WAVE_CYCLES SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS"
p=0
for C in "$A" "FETCH_SIZE" "WRITE_SIZE"; do
  p=$((p + 1))
  O=gpurun_out/pmc4/p$p
  mkdir -p $O
  timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $PWD/$O -o pmc -- \
      python bench.py --steps 1 --warmup 1 --settle-ms 0 --no-cpu-baseline --no-host-staged --no-deployable \
      --hbm-sets 0 --configs 4 > $O/run.log 2>&1 || { echo "pmc pass $p failed"; tail -5 $O/run.log; exit 1; }
done
python tools/pmc_summary.py gpurun_out/pmc4 16777216 256 gpurun_out/pmc4/summary.json "config 4: 16 Mi x 256 B, 1024 sessions, k_frames_lds"
