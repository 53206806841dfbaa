#!/bin/bash
# The bench as the driver runs it (python bench.py --gpus 1 --steps 20
# --warmup 5, everything on), then a kernel trace of the same main line for
# the replay-gap analysis (tools/replay_gaps.py).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/drv
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/drv/bench.log 2>&1 || { tail -5 gpurun_out/drv/bench.log; exit 1; }
grep '^{"metric"' gpurun_out/drv/bench.log | cut -c1-600
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/gpurun_out/drv/prof -o run -- \
    python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-staged --no-configs > gpurun_out/drv/prof.log 2>&1 \
    || { tail -5 gpurun_out/drv/prof.log; exit 1; }
python tools/replay_gaps.py gpurun_out/drv/prof
