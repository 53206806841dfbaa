#!/bin/bash
# quick GPU iteration: parity tests then kernel timing (stop on a fault)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc, stopping"; exit $rc; fi
bash tools/ablate.sh "$@" 2>&1 | grep -v amdgpu.ids
