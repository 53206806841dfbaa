# quick GPU check: parity (forced one-lane kernel), kernel timings, phase stamps
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
ZMQG_FRAMES_G=0 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_seq.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_seq.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_seq.log
timeout -k 10 120 python tools/kbench.py --iters 20 || exit 1
timeout -k 10 120 ./build/seq_stamps > gpurun_out/seq_stamps.txt 2>&1 || exit 1
grep -E "code|slot  1:|slot  2:|slot  4:|slot 25:|slot  5:|slot 19:|slot 40:|slot 60|slot 61" gpurun_out/seq_stamps.txt
if [ -x ./build/seq_stamps_e ]; then
  timeout -k 10 120 ./build/seq_stamps_e > gpurun_out/seq_stamps_e.txt 2>&1 || exit 1
  echo "--- early VMEM variant"; grep -E "code|slot  1:|slot  5:|slot 19:|slot 60|slot 61" gpurun_out/seq_stamps_e.txt
fi
