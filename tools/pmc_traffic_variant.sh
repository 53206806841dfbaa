#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of the frame kernels under ZMQG_FRAMES_G=$1 (kbench, config 2)
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/pmct_g$1
mkdir -p $O
for c in FETCH_SIZE WRITE_SIZE; do
  t=$(echo $c | tr A-Z a-z | cut -d_ -f1)
  ZMQG_FRAMES_G=$1 timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $PWD/$O/$t -o pmc -- \
      python tools/kbench.py --iters 3 > $O/$t.log 2>&1 || { echo "pass $c failed"; exit 1; }
done
echo done
