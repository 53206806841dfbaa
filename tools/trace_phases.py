#!/usr/bin/env python3
"""Frame-kernel durations of one bench.py run by phase, from a rocprofv3
kernel trace of it (tools/gpu_run.sh prof writes one): the runs of 2K
back-to-back frame launches (graph replays: gaps under 20 us) in order --
the untimed instantiation and settling replays, then the timed replay --
the eager pass of K steps after them, and bench.py's launch pass (K encodes,
then K decodes, back to back).  Shows whether the line's
roofline.avg_launch_us matches the kernels of the timed replay.

  trace_phases.py <trace dir> [K]"""
import csv
import glob
import json
import sys

d = sys.argv[1]
K = int(sys.argv[2]) if len(sys.argv) > 2 else 20
f = sorted(glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True))[0]
rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
              for r in csv.DictReader(open(f)))
fr = [r for r in rows if "k_frames" in r[2]]
# split into runs at gaps >= 20 us
runs, cur = [], [fr[0]]
for a, b in zip(fr, fr[1:]):
    if b[0] - a[1] >= 20000:
        runs.append(cur)
        cur = []
    cur.append(b)
runs.append(cur)


def stats(seg):
    dec = [(e - s) / 1e3 for s, e, k in seg if "<true" in k]
    enc = [(e - s) / 1e3 for s, e, k in seg if "<false" in k]
    span = (seg[-1][1] - seg[0][0]) / 1e3
    return {"launches": len(seg), "dec_avg_us": sum(dec) / max(len(dec), 1), "enc_avg_us": sum(enc) / max(len(enc), 1),
            "span_us_per_step": span / max(len(seg) // 2, 1)}


out = []
for i, seg in enumerate(runs):
    if len(seg) >= 4:
        o = stats(seg)
        o["run"] = i
        out.append(o)
print(json.dumps({"trace": f, "runs": out}, indent=1))
