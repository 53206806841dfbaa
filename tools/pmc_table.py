#!/usr/bin/env python3
"""Mean PMC counters per kernel (full demangled-name prefix) from rocprofv3 CSV dirs."""
import collections, csv, glob, re, sys
root = sys.argv[1]
keys = sys.argv[2:]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        if keys and not any(k in name for k in keys):
            continue
        short = re.sub(r"\(.*", "", name)[:60]
        acc[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:28s} {sum(v)/len(v):16.1f}  (n={len(v)})")
