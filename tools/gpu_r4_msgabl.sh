#!/bin/bash
# Round 4: k_msg ablations (build/abl<V>/libzmqg_curve.so, -DZMQG_MSG_ABLATE=V):
# per-call host time and the kernel's duration per message size (rocprofv3
# kernel trace, tools/msg_trace_sizes.py).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/msgabl
for v in ${ABL:-0 16 32 48 62}; do
  D=$PWD/libzmq_amd; [ $v != 0 ] && D=$PWD/build/abl$v
  LD_LIBRARY_PATH=$D:$LD_LIBRARY_PATH timeout -k 10 120 ./build/msg_kernel_bench abl$v || exit 1
  LD_LIBRARY_PATH=$D:$LD_LIBRARY_PATH timeout -k 10 180 rocprofv3 --kernel-trace -d gpurun_out/msgabl/v$v -o k --output-format csv -- ./build/msg_kernel_bench abl$v > /dev/null 2>&1 || exit 1
  python3 tools/msg_trace_sizes.py gpurun_out/msgabl/v$v/k_kernel_trace.csv abl$v
done
