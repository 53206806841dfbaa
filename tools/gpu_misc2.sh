#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 ./build/msg_latency || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/zprof -o run --output-format csv -- python tools/zmtp_bench.py || exit 1
