#!/bin/bash
# HBM traffic of the bench's kernels (MI355X_MICROARCH.md HBM section): one
# rocprofv3 pass per counter (FETCH_SIZE, WRITE_SIZE), kernel-trace only,
# plus the same counters over tools/framecopy (known byte counts, lane-strided
# dwordx4 pattern) to calibrate the gfx950 FETCH_SIZE scale for this access
# shape.  Output: gpurun_out/pmct/{fetch,write}[_cal]/...
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/pmct
mkdir -p $O
for c in FETCH_SIZE WRITE_SIZE; do
  t=$(echo $c | tr A-Z a-z | cut -d_ -f1)
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $PWD/$O/$t -o pmc -- \
      python bench.py --eager --steps 3 --warmup 1 --settle-ms 0 --no-cpu-baseline --no-host-staged --no-configs > $O/$t.log 2>&1 || { echo "bench pass $c failed"; exit 1; }
  timeout -s KILL 60 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $PWD/$O/${t}_cal -o pmc -- \
      ./tools/bin/framecopy > $O/${t}_cal.log 2>&1 || { echo "calibration pass $c failed"; exit 1; }
done
echo done
