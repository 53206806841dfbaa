#!/bin/bash
# A frame-kernel input change checked and timed in one call: the GPU suite,
# config 4's kernels over three rocprof runs (tools/gpu_cfg4_timing.sh), and
# two config-2 bench lines (main and hbm_fed, no other configs).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/skip5
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/skip5/pytest.log 2>&1 || { tail -30 gpurun_out/skip5/pytest.log; exit 1; }
tail -1 gpurun_out/skip5/pytest.log
bash tools/gpu_cfg4_timing.sh || exit 1
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-configs --no-host-staged --no-cpu-baseline \
      --no-deployable > gpurun_out/skip5/b$r.json 2> gpurun_out/skip5/b$r.err || { tail -5 gpurun_out/skip5/b$r.err; exit 1; }
  tail -1 gpurun_out/skip5/b$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; h=d['hbm_fed']; print('main', round(d['value'],1), 'dec', round(r['avg_launch_us'],1), 'enc', round(r['encode_main_avg_us'],1), 'hbm', round(h['value'],1), round(h['encode_us'],1), round(h['decode_us'],1))"
done
