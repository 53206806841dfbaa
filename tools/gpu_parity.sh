# GPU test round: parity suite with the default frame-kernel choice, again
# forcing the one-lane-per-frame kernel on every batch, then a short bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
ZMQG_FRAMES_G=0 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_seq.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_seq.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_seq.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-host-staged --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail gpurun_out/bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench.json')); r=d['roofline']; print('value', d['value'], 'ms/step', d['ms_per_step'], 'dec us', r['avg_launch_us'], 'enc us', r['encode_main_avg_us'], 'frac', r['frac'])"
