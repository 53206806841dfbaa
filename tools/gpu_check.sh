set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/sb
timeout -k 10 400 python -u -m pytest tests/test_gpu_session_batch.py tests/test_gpu_bench_batches.py tests/test_gpu_configs.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/sb/pytest.log 2>&1 || { tail -30 gpurun_out/sb/pytest.log; exit 1; }
tail -3 gpurun_out/sb/pytest.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-staged --no-deployable --hbm-sets 0 > gpurun_out/sb/bench.log 2>&1 || { tail -20 gpurun_out/sb/bench.log; exit 1; }
tail -1 gpurun_out/sb/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], {k:(v.get('value'), v.get('ms_per_step')) for k,v in d.get('configs',{}).items()})"
