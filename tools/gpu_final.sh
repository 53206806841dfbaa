#!/bin/bash
# Round-end evidence in one call: the GPU suite and smoke; rocprofv3
# kernel stats of the config-2 bench alone and of the bench with every
# config and the HBM-fed form; the driver-argument bench line; the ZMTP
# suite, bench and trace.  Outputs under gpurun_out/final/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=$PWD/gpurun_out/final
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
echo "smoke ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o c2 --output-format csv -- \
    python3 bench.py --steps 20 --warmup 5 --no-configs --no-host-staged --no-cpu-baseline --no-deployable --hbm-sets 0 \
    > $O/prof_c2.json 2> $O/prof_c2.err || { tail -20 $O/prof_c2.err; exit 1; }
echo "prof c2 ok"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_all -o all --output-format csv -- \
    python3 bench.py --steps 20 --warmup 5 --no-host-staged --no-cpu-baseline --no-deployable \
    > $O/prof_all.json 2> $O/prof_all.err || { tail -20 $O/prof_all.err; exit 1; }
echo "prof all ok"
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['hbm_fed']['value'], d['hbm_fed']['decode_us'], {k: round(v['value'],1) for k,v in d.get('configs',{}).items()})"
bash tools/gpu_zmtp_round6.sh || exit 1
