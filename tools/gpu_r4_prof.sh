#!/bin/bash
# Round 4: kernel-trace statistics of the per-message latency tool and of
# the driver-argument bench (20 steps, 5 warmup), then the bench line itself.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/prof_msg gpurun_out/prof_bench
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_msg -o msg --output-format csv -- ./build/msg_latency > gpurun_out/msg_latency_prof.json 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o bench --output-format csv -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err || exit 1
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > gpurun_out/bench_r4a.json 2> gpurun_out/bench_r4a.err || exit 1
tail -1 gpurun_out/bench_r4a.json
find gpurun_out/prof_msg gpurun_out/prof_bench -name "*kernel_stats.csv" | head
