#!/usr/bin/env python3
"""Summarise rocprofv3 PMC CSVs: mean counter value per kernel (over dispatches)."""
import collections
import csv
import glob
import sys

root = sys.argv[1]
keys = sys.argv[2:] or ["k_body", "head"]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        short = next((k for k in keys if k in name), None)
        if not short:
            continue
        tag = short + ("<dec>" if ("ILb1E" in name or "<true>" in name) else
                       "<enc>" if ("ILb0E" in name or "<false>" in name) else "")
        acc[tag][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:28s} {sum(v)/len(v):16.1f}  (n={len(v)})")
