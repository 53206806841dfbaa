#!/usr/bin/env python3
"""Summarise tools/pmc_twowave.sh: per-launch average of each counter for
k_frames_seq encode / decode, one column per workload."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
res = defaultdict(lambda: defaultdict(list))  # (workload, kernel) -> counter -> values
for f in glob.glob(os.path.join(root, "*", "**", "*counter_collection.csv"), recursive=True):
    wl = os.path.relpath(f, root).split(os.sep)[0].split("_")[0]
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", "")
        if "k_frames_seq" not in name:
            continue
        kind = "dec" if "k_frames_seq<true" in name else "enc"
        res[(wl, kind)][r["Counter_Name"]].append(float(r["Counter_Value"]))
for key in sorted(res):
    print(key)
    for c, v in sorted(res[key].items()):
        print(f"  {c:40s} {sum(v) / len(v):16.0f}  (n={len(v)})")
