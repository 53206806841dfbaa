#!/usr/bin/env python3
"""Per-launch VALU/SALU/VMEM wave-instruction counts of the frame kernels from
a rocprofv3 --pmc CSV (tools/pmc_valu_bench.sh) -> JSON for profiles/."""
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
        if "k_frames_seq" not in name:  # (the config-2 kernel only)
            continue
        k = "k_frames<decode>" if re.search(r"k_frames\w*<true", name) else "k_frames<encode>"
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {}
for k, d in acc.items():
    out[k] = {c: sum(v) / len(v) for c, v in sorted(d.items())}
    out[k]["dispatches"] = len(next(iter(d.values())))
print(json.dumps(out, indent=1))
