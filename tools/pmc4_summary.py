#!/usr/bin/env python3
"""Config-4 frame-kernel PMC (tools/gpu_run.sh pmc4 / pmc4b) summarised:
per-launch counters of k_frames_lds encode and decode (16 Mi x 256 B, 1,024
sessions, sid = i mod 1,024), per wave and per frame, the wave-cycle shares,
the store-ablation builds' counters, and the VALU-per-frame fit against the
frame's window count (k_frames_lds forced, 1 Mi frames of 128 ... 768 B) that
separates the per-window from the fixed per-frame part.

  pmc4_summary.py <gpurun_out> [out.json]
"""
import collections
import csv
import glob
import json
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
out_path = sys.argv[2] if len(sys.argv) > 2 else "profiles/round5_pmc_config4.json"


def per_kernel(d, want="k_frames"):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if want not in k:
                continue
            kk = ("decode" if "<true" in k else "encode") + " " + k.split("<")[0].split("::")[-1]
            acc[kk][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {kk: {c: sum(v) / len(v) for c, v in d.items()} for kk, d in acc.items()}


res = {"workload": "config 4: 16,777,216 x 256 B frames, 1,024 sessions (sid = i mod 1,024), tools/kbench.py "
                   "--sid-mod; k_frames_lds (two waves per SIMD)",
       "units": "per launch; *_per_wave = / 262,144 waves, *_per_frame = / 16,777,216 frames"}
WAVES, FRAMES = 16777216 / 64, 16777216
base = per_kernel(f"{root}/pmc4") or per_kernel(f"{root}/pmc4b/default")  # (pmc4b's default build: its counter set)
for kk, m in sorted(base.items()):
    o = {"counters": m}
    wc = m.get("SQ_WAVE_CYCLES")
    if wc:
        o["wave_cycle_shares"] = {n: m[n] / wc for n in ("SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_ANY",
                                                         "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_LDS",
                                                         "SQ_ACTIVE_INST_SCA") if n in m}
    o["per_wave"] = {n: m[n] / WAVES for n in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_WR",
                                               "SQ_INSTS_VMEM_RD", "SQ_INSTS_LDS") if n in m}
    o["valu_lane_ops_per_frame"] = m.get("SQ_INSTS_VALU", 0) * 64 / FRAMES
    res[kk] = o
abl = {}
for d in sorted(glob.glob(f"{root}/pmc4b/*")):
    name = os.path.basename(d)
    if not os.path.isdir(d) or name.startswith("sz"):
        continue
    m = per_kernel(d).get("encode k_frames_lds")
    if m:
        abl[name] = {"SQ_INSTS_VMEM_WR_per_wave": m.get("SQ_INSTS_VMEM_WR", 0) / WAVES,
                     "SQ_INSTS_VALU_per_wave": m.get("SQ_INSTS_VALU", 0) / WAVES,
                     "SQ_INSTS_SALU_per_wave": m.get("SQ_INSTS_SALU", 0) / WAVES,
                     "SQ_WAIT_INST_ANY": m.get("SQ_WAIT_INST_ANY"), "SQ_WAVE_CYCLES": m.get("SQ_WAVE_CYCLES")}
if abl:
    res["encode_store_ablations"] = abl
fit = {}
for d in sorted(d for d in glob.glob(f"{root}/pmc4b/sz*") if os.path.isdir(d)):
    P = int(os.path.basename(d)[2:])
    for kk, m in per_kernel(d).items():
        if "k_frames_lds" not in kk or "SQ_INSTS_VALU" not in m:
            continue
        tag = kk.split()[0]
        S = P + (33 if tag == "encode" else 33)  # stream bytes: 32 + flags byte + payload (both directions)
        fit.setdefault(tag, []).append({"payload": P, "windows": (S + 63) // 64,
                                        "valu_lane_ops_per_frame": m["SQ_INSTS_VALU"] * 64 / 1048576})
for tag, pts in fit.items():
    pts.sort(key=lambda p: p["payload"])
    n = len(pts)
    if n >= 2:
        xs = [p["windows"] for p in pts]
        ys = [p["valu_lane_ops_per_frame"] for p in pts]
        mx, my = sum(xs) / n, sum(ys) / n
        b = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / max(sum((x - mx) ** 2 for x in xs), 1e-9)
        a = my - b * mx
        res[f"valu_fit_{tag}"] = {"points": pts, "per_window": b, "fixed_per_frame": a}
json.dump(res, open(out_path, "w"), indent=1)
print(json.dumps({k: v for k, v in res.items() if k.startswith(("valu_fit", "encode_store"))}, indent=1))
for kk in sorted(base):
    print(kk, json.dumps(res[kk]["per_wave"]), json.dumps(res[kk].get("wave_cycle_shares")))
