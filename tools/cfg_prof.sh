#!/bin/bash
# rocprofv3 kernel statistics of BASELINE configs 3, 4 and 5, one bench.py
# run per config (main line shortened), summaries in gpurun_out/cfgprof/<c>/.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
for c in ${CFGS:-3 4 5}; do
  O=gpurun_out/cfgprof/c$c
  mkdir -p $O
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$O -o run -- \
      python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-staged --no-deployable --hbm-sets 0 --configs $c > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
  python - "$O" "$c" <<'PY'
import csv, glob, json, sys
o, c = sys.argv[1], sys.argv[2]
f = glob.glob(f"{o}/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
line = json.loads([l for l in open(f"{o}/bench.log") if l.startswith("{\"metric\"")][-1])
print("config", c, json.dumps({k: round(v["value"], 1) for k, v in line["configs"].items()}))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:8]:
    print("  %-60s calls %5s avg %10.1f us total %8.2f ms" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3,
                                                             float(r["TotalDurationNs"]) / 1e6))
PY
done
