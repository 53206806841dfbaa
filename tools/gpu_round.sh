#!/bin/bash
# GPU-box runner: parity tests, smoke, bench, rocprof summary.  Stops at the
# first step that faults, aborts or times out (exit 124/134/137/139).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; esac; [ "$1" -ge 128 ] && return 0; return 1; }
step() {  # step NAME TIMEOUT CMD...
  local name=$1 to=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 "$to" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $OUT/steps.log
  tail -5 $OUT/$name.log
  if fatal $rc; then echo "fatal rc=$rc in $name; stopping"; exit $rc; fi
  return $rc
}
MODE=${1:-all}
if [[ $MODE == all || $MODE == test ]]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [[ $MODE == all || $MODE == bench ]]; then
  step bench 600 python bench.py --gpus 1 --steps 20 --warmup 5
fi
if [[ $MODE == all || $MODE == prof ]]; then
  step rocprof 600 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/prof -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-staged --no-configs
fi
exit 0
