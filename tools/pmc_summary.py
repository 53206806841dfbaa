#!/usr/bin/env python3
"""Per-launch PMC counters of the frame kernels from rocprofv3 --pmc passes
(tools/pmc_cfg4.sh): every counter averaged over the
launches of each kernel (encode / decode), FETCH_SIZE doubled per the gfx950
note of MI355X_MICROARCH.md (HBM section) and both sizes in bytes, against the
algorithmic bytes of the workload; stamped with the source id of the library
the passes loaded (zmqg_build_id, from the bench line in each pass's log).

  pmc_summary.py <pass dir> <frames> <payload bytes> <out.json> [note]
"""
import collections
import csv
import glob
import json
import sys

root, frames, P, out = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
note = sys.argv[5] if len(sys.argv) > 5 else ""
acc = collections.defaultdict(lambda: collections.defaultdict(list))
src = set()
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "k_frames" not in k:
            continue
        kk = ("decode " if "<true" in k else "encode ") + k.split("<")[0].split("::")[-1]
        acc[kk][r["Counter_Name"]].append(float(r["Counter_Value"]))
for f in glob.glob(f"{root}/**/run.log", recursive=True):
    for line in open(f):
        if line.startswith('{"metric"'):
            src.add(json.loads(line)["build"]["source_id"])
W = 33
alg = {"encode": {"read": frames * (P + 4 + 8 + 4 + 1 + 8), "write": frames * (P + W)},
       "decode": {"read": frames * (P + W + 4 + 8 + 4 + 8), "write": frames * (P + 1 + 4)}}
res = {"source_id": sorted(src), "frames": frames, "payload_bytes": P, "note": note,
       "units": "per launch (average over the profiled launches); read/write bytes: FETCH_SIZE x 2 (gfx950 "
                "streaming-read note) and WRITE_SIZE, KiB -> bytes"}
for kk, m in sorted(acc.items()):
    c = {n: sum(v) / len(v) for n, v in m.items()}
    o = {"counters": c, "launches": max(len(v) for v in m.values())}
    waves = c.get("SQ_WAVES")
    if waves:
        o["per_wave"] = {n: c[n] / waves for n in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_WR",
                                                   "SQ_INSTS_VMEM_RD") if n in c}
    if "SQ_WAVE_CYCLES" in c:
        o["wait_inst_share"] = c.get("SQ_WAIT_INST_ANY", 0) / c["SQ_WAVE_CYCLES"]
        o["wait_lds_share"] = c.get("SQ_WAIT_INST_LDS", 0) / c["SQ_WAVE_CYCLES"]
    a = alg["decode" if kk.startswith("decode") else "encode"]
    if "FETCH_SIZE" in c:
        o["read_bytes"] = c["FETCH_SIZE"] * 1024 * 2
        o["read_vs_algorithmic"] = o["read_bytes"] / a["read"]
    if "WRITE_SIZE" in c:
        o["write_bytes"] = c["WRITE_SIZE"] * 1024
        o["write_vs_algorithmic"] = o["write_bytes"] / a["write"]
    o["algorithmic"] = a
    res[kk] = o
json.dump(res, open(out, "w"), indent=1)
print(json.dumps({k: {x: v[x] for x in ("per_wave", "wait_inst_share", "read_vs_algorithmic", "write_vs_algorithmic")
                      if x in v} for k, v in res.items() if isinstance(v, dict) and "counters" in v}, indent=1))
