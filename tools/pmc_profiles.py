#!/usr/bin/env python3
"""profiles/pmc_valu_config2.json and profiles/pmc_traffic_config2.json from
the PMC passes of tools/pmc_profiles.sh (gpurun_out/pmcv, gpurun_out/pmct):
per-launch VALU/SALU/VMEM wave-instruction counts and HBM bytes of the
config-2 frame kernels, FETCH_SIZE scaled by the calibration copy of the same
access shape (tools/framecopy.hip, LANE, one window in flight)."""
import collections
import csv
import glob
import json
import re
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
N, P = 65536, 1024


def per_kernel(d):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return acc


def pick(acc, pat, counter):
    for k, v in acc.items():
        if re.search(pat, k) and counter in v:
            return sum(v[counter]) / len(v[counter]), k
    raise KeyError(pat)


def build_of(log):
    """the bench line's build (zmqg_build_id of the library the pass loaded)"""
    for line in reversed(open(log).read().splitlines()):
        if line.startswith("{"):
            return json.loads(line)["build"]
    raise ValueError(f"no bench line in {log}")


logs = (glob.glob(f"{root}/pmcv/run.log") + glob.glob(f"{root}/pmcs/run.log")
        + glob.glob(f"{root}/pmct/resident/*/run.log") + glob.glob(f"{root}/pmct/hbm/*/run.log"))
builds = {build_of(f)["source_id"]: build_of(f) for f in logs}
assert len(builds) == 1, f"PMC passes of different builds: {sorted(builds)}"
build = next(iter(builds.values()))

valu = json.load(open(f"{root}/pmcv/summary.json"))
try:
    stall = json.load(open(f"{root}/pmcs/summary.json"))
except FileNotFoundError:
    stall = {}
fcal, wcal = per_kernel(f"{root}/pmct/cal/fetch"), per_kernel(f"{root}/pmct/cal/write")
moved_kib = N * P / 1024
# the frame kernels' reads: LDS-DMA of whole 16-byte granules in runs of a
# frame's five (k_frames_seq's staged input, k_frames_lds) -- the
# calibration copy's cooperative shape (4 lanes per frame window); writes:
# each lane's own 64-byte pieces -- the lane shape
cal_f, _ = pick(fcal, r"k_copy<true, 1>", "FETCH_SIZE")
cal_w, _ = pick(wcal, r"k_copy<false, 1>", "WRITE_SIZE")
cal_f_lane, _ = pick(fcal, r"k_copy<false, 1>", "FETCH_SIZE")
scale = moved_kib / cal_f
EA = ("TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_32B_sum", "TCC_EA0_WRREQ_sum", "TCC_EA0_WRREQ_64B_sum")


def traffic(form, dec):
    tag = "decode" if dec else "encode"
    pat = r"k_frames\w*<%s" % ("true" if dec else "false")
    fetch, write = per_kernel(f"{root}/pmct/{form}/fetch"), per_kernel(f"{root}/pmct/{form}/write")
    f, kname = pick(fetch, pat, "FETCH_SIZE")
    w, _ = pick(write, pat, "WRITE_SIZE")
    kshort = re.search(r"(k_frames\w*)<", kname).group(1) + "<%s>" % tag
    alg_r = N * (P + 49) if dec else N * (P + 25)
    alg_w = N * (P + 5) if dec else N * (P + 33)
    t = {"kernel": kshort, "read_bytes_per_launch": f * scale * 1024, "write_bytes_per_launch": w * 1024,
         "fetch_size_kib_raw": f, "write_size_kib_raw": w, "algorithmic_read_bytes_per_launch": alg_r,
         "algorithmic_write_bytes_per_launch": alg_w,
         "read_vs_algorithmic": f * scale * 1024 / alg_r, "write_vs_algorithmic": w * 1024 / alg_w}
    ea = per_kernel(f"{root}/pmct/{form}/ea")
    reqs = {}
    for c in EA:
        try:
            reqs[c] = pick(ea, pat, c)[0]
        except KeyError:
            pass
    if reqs:
        t["l2_memory_side_requests_per_launch"] = reqs
    return t


out_t, out_v = {}, {}
for dec in (True, False):
    tag = "decode" if dec else "encode"
    t = traffic("resident", dec)
    kshort = t["kernel"]
    v = valu["k_frames<%s>" % tag]
    vv = {"kernel": kshort, "valu_wave_instr_per_launch": v["SQ_INSTS_VALU"], "salu_instr_per_launch": v["SQ_INSTS_SALU"],
          "vmem_instr_per_launch": v["SQ_INSTS_VMEM"], "waves": v["SQ_WAVES"],
          "valu_lane_ops_per_frame": v["SQ_INSTS_VALU"] * 64 / N}
    st = stall.get("k_frames<%s>" % tag)
    if st:  # quad-cycle counters, summed over the launch's waves; shares of the waves' lifetime
        wc = st["SQ_WAVE_CYCLES"]
        vv["wave_cycle_shares"] = {
            "issuing (SQ_ACTIVE_INST_ANY)": st["SQ_ACTIVE_INST_ANY"] / wc,
            "of which VALU (SQ_ACTIVE_INST_VALU)": st["SQ_ACTIVE_INST_VALU"] / wc,
            "waiting at s_waitcnt / barriers (SQ_WAIT_ANY)": st["SQ_WAIT_ANY"] / wc,
            "stalled at issue (SQ_WAIT_INST_ANY)": st["SQ_WAIT_INST_ANY"] / wc}
    if dec:
        out_t.update(t)
        out_v.update(vv)
    else:
        out_t["encode"] = t
        out_v["encode"] = vv
out_t["hbm_fed"] = {"decode": traffic("hbm", True), "encode": traffic("hbm", False),
                    "form": "tools/hbm_probe.py --forms bench --stream-out: 8 config-2 batches with their own buffers, "
                            "8 encodes back to back then their 8 decodes with ZMQG_OPT_STREAM_OUT (bench.py hbm_fed); "
                            "every input from HBM"}
out_t.update({
    "source_id": build["source_id"], "commit": build["commit"],
    "workload": "config2: 65536 x 1024 B frames, one session, one lane per frame (1024 waves, 1 per SIMD)",
    "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / TCC_EA0_{RDREQ,RDREQ_32B,WRREQ,WRREQ_64B}_sum (separate "
              "passes, --kernel-trace) of python bench.py --eager --steps 3 --warmup 1 --no-deployable --hbm-sets 0 "
              "(MALL-resident, top level) and of tools/hbm_probe.py --forms bench (hbm_fed); calibration: the same "
              "counters over tools/framecopy (65536 x 1024 B, known bytes); tools/pmc_traffic.sh, "
              "tools/pmc_profiles.py",
    "units": "bytes per launch; request counts per launch", "fetch_scale": scale,
    "fetch_scale_note": "FETCH_SIZE under-reports on gfx950 (MI355X_MICROARCH.md HBM section): the calibration "
                        "copy's cooperative shape (the frame kernels' LDS-DMA granule runs) reads %.0f KiB "
                        "reported per %.0f KiB moved (the lane shape %.0f), so reads are scaled by %.3f.  "
                        "WRITE_SIZE is taken as reported; the calibration copy's lane stores show %.2fx the bytes "
                        "moved.  FETCH_SIZE counts the L2's memory-side requests, Infinity-Cache hits included: "
                        "the resident form's reads mostly hit the MALL, the HBM-fed form's come from HBM."
                        % (cal_f, moved_kib, cal_f_lane, scale, cal_w / moved_kib)})
out_v.update({
    "source_id": build["source_id"], "commit": build["commit"],
    "workload": out_t["workload"],
    "source": "rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES "
              "--kernel-trace of python bench.py --eager --steps 3 --warmup 1 (tools/pmc_valu_bench.sh)",
    "units": "wave instructions per launch (one VALU wave instruction = 64 lane operations; a wave alone on its "
             "SIMD issues one every 4 cycles)",
    "salsa20_lane_ops_per_frame_floor": 17 * 940,
    "simds": 1024, "lanes_per_simd_per_cycle": 16, "clock_ghz_spec": 2.4, "clock_ghz_measured": 2.09,
    "clock_note": "s_memtime over s_memrealtime per workgroup of the frame kernel (tools/frames_bench.hip): "
                  "2.05-2.12 GHz per XCD under this load",
    "peak_note": "16 lanes per cycle per SIMD: one wave per SIMD issues a VALU instruction every 4 cycles, and the "
                 "Salsa20 instruction mix issues at that rate at every occupancy (profiles/valu_rates_r02.md)"})
json.dump(out_t, open("profiles/pmc_traffic_config2.json", "w"), indent=1)
json.dump(out_v, open("profiles/pmc_valu_config2.json", "w"), indent=1)
print(json.dumps({"traffic": {k: out_t[k] for k in ("kernel", "read_bytes_per_launch", "write_bytes_per_launch")},
                  "valu": {k: out_v[k] for k in ("kernel", "valu_wave_instr_per_launch", "valu_lane_ops_per_frame")}}))
