#!/usr/bin/env python3
"""k_msg durations per message size from a rocprofv3 kernel trace of
tools/msg_kernel_bench (three sizes in order, 2,050 encode+decode pairs each)."""
import csv
import statistics
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_msg" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
per = len(rows) // 3
for i, size in enumerate(("32", "1024", "4000")):
    seg = rows[i * per:(i + 1) * per]
    d = lambda kind: statistics.median(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg
                                       if kind in r["Kernel_Name"]) / 1e3
    print(f"{sys.argv[2]} size {size}: k_msg encode {d('false'):.2f} us, decode {d('true'):.2f} us (medians)")
