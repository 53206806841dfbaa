#!/usr/bin/env python3
"""Summary of tools/pmc_configs.sh: per-launch counters of the chunked body
kernel (configs 3 and 5) and k_frames_lds (config 4), averaged over the
launches of each bench run, with wave-cycle shares and HBM bytes (FETCH_SIZE
x 1 KiB as reported; for k_body, whose reads are 16-byte-per-lane coalesced
LDS-DMA, also doubled -- gfx950 counts half of such a read; WRITE_SIZE x 1 KiB).  Usage:
pmc_configs.py <dir> [out.json]"""
import collections
import csv
import glob
import json
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmcc"
out_path = sys.argv[2] if len(sys.argv) > 2 else os.path.join(os.path.dirname(root.rstrip("/")), "pmc_configs.json")
WANT = {"3": ("k_body",), "4": ("k_frames_lds",), "5": ("k_body",)}
res = {}
for cdir in sorted(glob.glob(f"{root}/c*")):
    c = os.path.basename(cdir)[1:]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{cdir}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            base = next((w for w in WANT.get(c, ()) if w + "<" in k or w + "I" in k), None)
            if base is None:
                continue
            kk = base + ("<dec>" if ("<true" in k or "ILb1E" in k) else "<enc>")
            acc[kk][r["Counter_Name"]].append(float(r["Counter_Value"]))
    cfg = {}
    for kk, d in sorted(acc.items()):
        m = {n: sum(v) / len(v) for n, v in d.items()}
        wc = m.get("SQ_WAVE_CYCLES") or 1.0
        o = {"launches_profiled": max(len(v) for v in d.values()), "counters_per_launch": m,
             "wave_cycle_shares": {n: m[n] / wc for n in ("SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_ANY",
                                                           "SQ_WAIT_INST_ANY") if n in m}}
        if "FETCH_SIZE" in m:
            o["fetch_bytes_per_launch_reported"] = m["FETCH_SIZE"] * 1024
            if kk.startswith("k_body"):  # 16-B-per-lane coalesced LDS-DMA: FETCH_SIZE counts half (MI355X_MICROARCH.md, HBM)
                o["read_bytes_per_launch"] = 2 * m["FETCH_SIZE"] * 1024
        if "WRITE_SIZE" in m:
            o["write_bytes_per_launch"] = m["WRITE_SIZE"] * 1024
        cfg[kk] = o
    res["config" + c] = cfg
json.dump(res, open(out_path, "w"), indent=1)
for c, cfg in res.items():
    for kk, o in cfg.items():
        m = o["counters_per_launch"]
        print(c, kk, json.dumps({"shares": {k: round(v, 3) for k, v in o["wave_cycle_shares"].items()},
                                 "valu": m.get("SQ_INSTS_VALU"), "fetch_GB": o.get("fetch_bytes_per_launch_reported", 0) / 1e9,
                                 "write_GB": o.get("write_bytes_per_launch", 0) / 1e9}))
