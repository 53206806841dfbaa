#!/bin/bash
# Round 4: the per-message kernel after its quad-lane Salsa20 -- the msg
# tests, per-call host time (msg_kernel_bench), the round trips
# (msg_latency) and k_msg's duration per message size (kernel trace).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/msg2
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_msg.py tests/test_host_adapter.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_msg.log 2>&1 || { tail -30 gpurun_out/pytest_msg.log; exit 1; }
tail -1 gpurun_out/pytest_msg.log
LD_LIBRARY_PATH=$PWD/libzmq_amd:$LD_LIBRARY_PATH timeout -k 10 120 ./build/msg_kernel_bench quad || exit 1
LD_LIBRARY_PATH=$PWD/libzmq_amd:$LD_LIBRARY_PATH timeout -k 10 120 ./build/msg_kernel_bench quad || exit 1
timeout -k 10 120 ./build/msg_latency > gpurun_out/msg2/msg_latency.json 2>&1 || exit 1
grep '^{' gpurun_out/msg2/msg_latency.json
LD_LIBRARY_PATH=$PWD/libzmq_amd:$LD_LIBRARY_PATH timeout -k 10 180 rocprofv3 --kernel-trace -d gpurun_out/msg2/tr -o k --output-format csv -- ./build/msg_kernel_bench quad > /dev/null 2>&1 || exit 1
python3 tools/msg_trace_sizes.py gpurun_out/msg2/tr/k_kernel_trace.csv quad
