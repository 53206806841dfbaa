#!/bin/bash
# VALU instructions per tile and wave-cycle shares of k_body for the default
# build and each timing ablation (tools/bin/libzmqg_body_ab<V>.so, -DZMQG_ABLATE=V:
# 2 no keystream/MAC, 3 no edge stores, 4 no finish, 5 no interior stores,
# 6 no DMA; outputs garbage), config-5 frame size.  The VALU difference to the
# default build is what that piece issues.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
SHAPE="--msgs ${MSGS:-128} --size ${SIZE:-16777216} --sessions ${SESS:-8}"
C="SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU"
for v in default ${ABL:-2 3 4 5 6}; do
  O=gpurun_out/abpmc/$v
  mkdir -p $O
  if [ $v = default ]; then LIB=""; else LIB=$PWD/tools/bin/libzmqg_body_ab$v.so; [ -f $LIB ] || continue; fi
  ZMQG_CURVE_LIB=$LIB timeout -s KILL 150 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $PWD/$O -o pmc -- \
      python tools/kbench.py --iters 2 $SHAPE --tag ab$v > $O/run.log 2>&1 || { echo "pmc $v failed"; tail -5 $O/run.log; exit 1; }
  grep '"tag"' $O/run.log | cut -c1-400
  python tools/pmc_body.py $O | sed "s/^/$v /"
done
