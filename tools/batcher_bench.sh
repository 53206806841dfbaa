#!/bin/bash
# Build tools/batcher_bench.cpp against the in-tree library (run it on the GPU box:
#   gpurun -- 'timeout -k 10 200 ./tools/bin/batcher_bench')
set -e
cd "$(dirname "$0")/.."
mkdir -p build
/opt/rocm/bin/hipcc -O2 -std=c++17 --offload-arch=gfx950 -o tools/bin/batcher_bench tools/batcher_bench.cpp \
    libzmq_amd/host/curve_batcher.cpp libzmq_amd/host/curve_encoding_gpu.cpp \
    -Llibzmq_amd -lzmqg_curve -Wl,-rpath,'$ORIGIN/../libzmq_amd'
