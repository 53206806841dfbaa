#!/usr/bin/env python3
"""Summary of tools/pmc_body.sh: per-launch counters of k_body<enc>/<dec>
(averaged over the profiled launches), wave-cycle shares, instructions per
64-chunk tile, HBM bytes against the algorithmic bytes.  Usage:
pmc_body.py <dir> [payload_bytes_per_launch]"""
import collections
import csv
import glob
import json
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmcb"
payload = float(sys.argv[2]) if len(sys.argv) > 2 else 128 * 16 * 2**20
tiles = payload / 8192  # 64 chunks of 128 bytes
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "k_body" not in k:
            continue
        kk = "k_body<dec>" if "ILb1E" in k else "k_body<enc>"
        acc[kk][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {}
for kk, d in sorted(acc.items()):
    m = {c: sum(v) / len(v) for c, v in d.items()}
    wc = m.get("SQ_WAVE_CYCLES", 1.0)
    o = {"counters_per_launch": m}
    o["wave_cycle_shares"] = {c: m[c] / wc for c in ("SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_ANY",
                                                       "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_LDS")
                              if c in m}
    o["per_tile"] = {c: m[c] / tiles for c in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM", "SQ_INSTS_SALU",
                                                "SQ_INSTS_VMEM_WR", "SQ_INSTS_VMEM_RD", "SQ_LDS_BANK_CONFLICT")
                     if c in m}
    if "FETCH_SIZE" in m:
        o["read_bytes_per_launch"] = m["FETCH_SIZE"] * 1024
    if "WRITE_SIZE" in m:
        o["write_bytes_per_launch"] = m["WRITE_SIZE"] * 1024
    o["payload_bytes_per_launch"] = payload
    out[kk] = o
json.dump(out, open(f"{root}/../pmc_body.json", "w"), indent=1)
for kk, o in out.items():
    print(kk, json.dumps({"shares": {k: round(v, 3) for k, v in o["wave_cycle_shares"].items()},
                          "per_tile": {k: round(v, 1) for k, v in o["per_tile"].items()},
                          "read_GB": o.get("read_bytes_per_launch", 0) / 1e9,
                          "write_GB": o.get("write_bytes_per_launch", 0) / 1e9}))
