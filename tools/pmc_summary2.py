#!/usr/bin/env python3
"""Mean per-dispatch counter values per kernel from rocprofv3 --pmc CSVs
(tools/pmc_frames.sh) -> JSON on stdout.  Kernels are keyed by a short name
(template arguments kept, parameter list dropped)."""
import collections
import csv
import glob
import json
import re
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        short = re.sub(r"\(.*$", "", name.split(" ", 1)[-1]) if "(" in name else name
        short = re.sub(r"\(anonymous namespace\)::|zmqg::", "", short)
        acc[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {}
for k, d in acc.items():
    if len(sys.argv) > 2 and not re.search(sys.argv[2], k):
        continue
    out[k] = {c: sum(v) / len(v) for c, v in sorted(d.items())}
    out[k]["dispatches"] = max(len(v) for v in d.values())
print(json.dumps(out, indent=1))
