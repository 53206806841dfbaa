#!/bin/bash
# Round 4: the bench line (driver arguments) of two library builds,
# alternating on one box.  A = build/libzmqg_curve_r4a.so, B = the tree's.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for r in 1 2; do
  for lib in build/libzmqg_curve_r4a.so libzmq_amd/libzmqg_curve.so; do
    ZMQG_CURVE_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-staged --no-configs > gpurun_out/benchab.json 2> gpurun_out/benchab.err || { tail -20 gpurun_out/benchab.err; exit 1; }
    tail -1 gpurun_out/benchab.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', round(d['value'],1), round(d['ms_per_step']*1000,1), round(d['roofline']['avg_launch_us'],1), round(d['roofline']['encode_main_avg_us'],1))"
  done
done
