#!/bin/bash
# Config 4's frame kernels per launch under rocprofv3 --kernel-trace --stats,
# three bench runs back to back on one box (encode / decode spread, DESIGN.md
# section 3.1).  Output gpurun_out/cfg4t/r*/.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
for r in 1 2 3; do
  O=gpurun_out/cfg4t/r$r
  mkdir -p $O
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$O -o c4 -- \
      python3 bench.py --steps 10 --warmup 5 --no-cpu-baseline --no-host-staged --no-deployable --hbm-sets 0 \
      --configs 4 > $O/bench.json 2> $O/run.err || { tail -5 $O/run.err; exit 1; }
  python3 - "$O/c4_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "k_frames_lds" in r["Name"]:
        print(r["Name"][:40], r["Calls"], round(float(r["AverageNs"]) / 1e6, 3), "ms")
PY
done
