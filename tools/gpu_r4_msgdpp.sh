#!/bin/bash
# Round 4: k_msg's Poly1305 power scan and lane sum on DPP (the tree's build)
# against the LDS-permute build (build/msgA): parity first, then per-call time
# alternating on one box.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_msg.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/msgdpp_tests.log 2>&1
rc=$?; tail -3 gpurun_out/msgdpp_tests.log; [ $rc -ne 0 ] && { grep -B5 -A30 "FAILED\|Error" gpurun_out/msgdpp_tests.log | head -60; exit 1; }
bash tools/gpu_r4_msgab.sh
