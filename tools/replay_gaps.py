#!/usr/bin/env python3
"""Where the time of bench.py's timed graph replay goes: from a rocprofv3
kernel trace of the main line (tools/gpu_driver_bench.sh), the frame-kernel
launches of the replay (the K steps' encode/decode pairs launched back to
back), their durations, the gaps between them, and replay span vs kernel sum.
Usage: replay_gaps.py <trace dir> [steps]"""
import csv
import glob
import json
import sys

d = sys.argv[1]
K = int(sys.argv[2]) if len(sys.argv) > 2 else 20
f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(f))))
frames = [r for r in rows if "k_frames" in r[2]]
# the replay: the first run of 2K frame kernels whose gaps are all small
best = None
for s in range(len(frames) - 2 * K + 1):
    seg = frames[s:s + 2 * K]
    gaps = [seg[j + 1][0] - seg[j][1] for j in range(len(seg) - 1)]
    if max(gaps) < 20000:  # 20 us: launched from a graph, not from the host
        best = (s, seg, gaps)
        break
if best is None:
    print("no replay found")
    sys.exit(1)
s, seg, gaps = best
dur = [e - b for b, e, _ in seg]
span = seg[-1][1] - seg[0][0]
enc = [x for x, r in zip(dur, seg) if "ILb0E" in r[2] or "<false" in r[2]]
dec = [x for x, r in zip(dur, seg) if "ILb1E" in r[2] or "<true" in r[2]]
others = [r for r in rows if seg[0][0] <= r[0] <= seg[-1][1] and "k_frames" not in r[2]]
out = {"steps": K, "replay_span_us": span / 1e3, "per_step_us": span / 1e3 / K,
       "kernel_sum_per_step_us": sum(dur) / 1e3 / K,
       "gap_per_step_us": sum(gaps) / 1e3 / K, "max_gap_us": max(gaps) / 1e3,
       "enc_us": {"mean": sum(enc) / len(enc) / 1e3, "min": min(enc) / 1e3, "max": max(enc) / 1e3,
                  "first3": [x / 1e3 for x in enc[:3]], "last3": [x / 1e3 for x in enc[-3:]]},
       "dec_us": {"mean": sum(dec) / len(dec) / 1e3, "min": min(dec) / 1e3, "max": max(dec) / 1e3,
                  "first3": [x / 1e3 for x in dec[:3]], "last3": [x / 1e3 for x in dec[-3:]]},
       "other_kernels_in_replay": len(others)}
print(json.dumps(out))
