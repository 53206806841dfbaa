#!/bin/bash
# k_body diagnostics: kernel timings at config-5
# frame size (128 x 16 MiB, 8 sessions) for the default build and the timing
# ablations (tools/bin/libzmqg_body_ab<V>.so = -DZMQG_ABLATE=V; outputs garbage),
# per-tile phase stamps (tools/bin/libzmqg_curve_stamps.so, tools/stamps.py), a
# rocprofv3 kernel-stats pass over bench.py's configs 3/4/5, and one PMC pass
# of instruction counts and wave-cycle shares of k_body.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
SHAPE="--msgs ${MSGS:-128} --size ${SIZE:-16777216} --sessions ${SESS:-8}"
timeout -k 10 180 python tools/kbench.py --iters 5 $SHAPE --tag body || exit 1
for v in ${ABL:-2 3 4 5}; do
  [ -f tools/bin/libzmqg_body_ab$v.so ] || continue
  ZMQG_CURVE_LIB=$PWD/tools/bin/libzmqg_body_ab$v.so timeout -k 10 180 python tools/kbench.py --iters 5 $SHAPE --tag body_ab$v || exit 1
done
if [ -f tools/bin/libzmqg_curve_stamps.so ]; then
  timeout -k 10 180 python tools/stamps.py $SHAPE --tag stamps || exit 1
fi
[ -n "$NOPROF" ] && exit 0
O=gpurun_out/cfgprof
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$O -o run -- \
    python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-staged > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log
C="SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_LDS"
O=gpurun_out/pmc_body
mkdir -p $O
timeout -s KILL 180 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $PWD/$O -o pmc -- \
    python tools/kbench.py --iters 2 $SHAPE --tag pmc > $O/run.log 2>&1 || { echo "pmc pass failed"; tail -5 $O/run.log; exit 1; }
python - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/pmc_body/**/pmc_counter_collection.csv", recursive=True)
acc = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.Counter()
for r in csv.DictReader(open(f[0])):
    k = r["Kernel_Name"]
    kk = ("k_body" if "k_body" in k else "k_frames" if "k_frames" in k else None)
    if not kk: continue
    kk += "<dec>" if "ILb1E" in k else "<enc>"
    acc[kk][r["Counter_Name"]] += float(r["Counter_Value"]); cnt[(kk, r["Counter_Name"])] += 1
for kk, d in sorted(acc.items()):
    n = cnt[(kk, "SQ_WAVE_CYCLES")] or 1
    wc = d["SQ_WAVE_CYCLES"] or 1
    print(kk, "launches", n, " ".join(f"{c}={d[c]/n:.4g}" for c in sorted(d)),
          "| issue%", round(100 * d["SQ_ACTIVE_INST_ANY"] / wc, 1), "valu%", round(100 * d["SQ_ACTIVE_INST_VALU"] / wc, 1),
          "wait%", round(100 * d["SQ_WAIT_ANY"] / wc, 1), "stall%", round(100 * d["SQ_WAIT_INST_ANY"] / wc, 1))
PY
