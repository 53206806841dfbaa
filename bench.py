#!/usr/bin/env python3
"""Benchmark: device-resident CURVE MESSAGE encode+decode on MI355X.

Metric (BASELINE.json): GiB/s device-resident CURVE encode+decode, 1 KiB-msg
batches; msgs/s.  Workload at N=1 = BASELINE config 2: 65,536 x 1 KiB
frames, one CURVE session, encode (zmqg_encode_batch) then decode
(zmqg_decode_batch) of the produced wire frames, inputs resident in HBM.
One step = one such round trip over the batch (fresh nonces every step:
the decoder's replay rule would reject a repeated nonce).

Multi-GPU (torchrun, one process per GPU): every rank runs the same
per-GPU batch on its own device with its own sessions -- the path shards by
frame with no data exchange (weak scaling).  Ranks meet only at the
barriers around the timed region (gloo, control only).

Timing: W warmup steps, the K steps captured as one hipGraph, one untimed
replay (instantiation), untimed replays until --settle-ms of GPU time has
passed (the device's clock ramp under sustained load),
then ONE timed replay of exactly K steps between barriers and synchronises.

JSON line fields beyond the driver contract:
  settle        the untimed settling replays' time per step, in order
  roofline      dominant kernel (decode frame kernel) achieved algorithmic HBM-read
                GB/s vs the 8 TB/s peak.  HIP events cannot time a kernel
                inside a replayed graph, so the per-launch durations come
                from replays of the timed graph and of a graph of its
                encodes alone, alternating, just before the timed replay
                (graph_shares: decode = the difference per step);
                traffic = PMC-measured HBM bytes per launch from
                profiles/ if a PMC summary for this workload was committed;
                valu = the same kernel against the VALU issue peak (the bound
                that binds: PMC instruction count / live launch duration).
  host_paths    the same round trip starting and ending in host memory
                (PCIe-inclusive): zero-copy on pinned memory, pinned
                hipMemcpyAsync (with the GPU's PCIe link and NUMA placement),
                staged through zmqg_*_host from pageable buffers; and the
                deployable paths: the engine-hook bench and the libzmq CURVE
                PUSH/PULL pairs, stock against the batched GPU codec.
  hbm_fed       config 2 with every kernel input read from HBM (K batches with
                their own buffers, beyond the 256 MiB Infinity Cache), with
                its own decode roofline and PMC traffic; its encodes and
                decodes pass ZMQG_OPT_STREAM_OUT, the store hint for outputs
                no cache holds (--stream-out applies it to the main line's
                decodes too, for comparison).
  cpu_baseline  kind "reference": the stock libzmq build's curve_encoding_t
                on the host cores, rank 0 at N=1 only, on a bounded sample;
                beside it ("port") the oracle's C restatement of the framing
                with libsodium's crypto_box_easy_afternm/open (dlopen).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
ROOF_KERNEL = "k_frames_seq<decode>"  # the dominant kernel of the bench workload (one lane per frame)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--msgs", type=int, default=65536)
    p.add_argument("--size", type=int, default=1024)
    p.add_argument("--settle-ms", type=float, default=40.0,
                   help="untimed replays of the captured steps before the timed one, until this much GPU time "
                        "has passed (the clock ramp under sustained load; 0: none)")
    p.add_argument("--cold-pass", action="store_true",
                   help="also time each frame kernel on inputs from HBM (roofline.cold_launch_pass)")
    p.add_argument("--hbm-sets", type=int, default=8,
                   help="config-2 batches of the HBM-fed form (hbm_fed): each its own payload, wire and result "
                        "buffers, so no kernel reads what the Infinity Cache still holds (0: skip)")
    p.add_argument("--stream-out", action="store_true",
                   help="experiment: the main line's decodes with ZMQG_OPT_STREAM_OUT")
    p.add_argument("--no-deployable", action="store_true",
                   help="skip host_paths' deployable paths (the engine-hook bench and the libzmq CURVE pairs)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-host-staged", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=2.0, help="wall seconds of CPU baseline sampling")
    p.add_argument("--no-configs", action="store_true",
                   help="skip the other BASELINE configs (3, 4, 5) measured after the main line")
    p.add_argument("--configs", default="3,4,5", help="which of the other BASELINE configs to measure")
    p.add_argument("--eager", action="store_true",
                   help="launch every step from the host instead of replaying the captured K steps as one hipGraph")
    p.add_argument("--dry-run", action="store_true",
                   help="start the ranks, meet at one barrier, print one JSON line per rank and exit before any "
                        "GPU call (tests the multi-GPU launch on a CPU host)")
    return p.parse_args()


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args):
    """`python bench.py --gpus N` outside torchrun: start N ranks, one process
    per GPU, as a FRESH child `torch.distributed.run` (this process has made
    no GPU call, and it does not exec: it waits for the child and exits with
    its return code).  Rank 0's JSON line reaches our stdout through the
    inherited descriptors."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(cmd, env=env)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    if args.gpus != world:
        print(f"bench: --gpus {args.gpus} but WORLD_SIZE {world}; running {world} ranks", file=sys.stderr)
    if args.dry_run:
        if world > 1:
            dist.barrier()
        # one write(2) per line (atomic on a pipe), so the ranks' lines never interleave
        sys.stdout.flush()
        os.write(1, (json.dumps({"dry_run": True, "rank": rank, "local_rank": local, "world": world}) + "\n").encode())
        if world > 1:
            dist.destroy_process_group()
        return
    # one process per GPU; (a rehearsal with more ranks than GPUs shares them,
    # and the line then reports the devices actually used, not the ranks)
    local = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    n_devices, shared_devices = device_census(torch, world, local)

    from libzmq_amd import curve as C

    n, P = args.msgs, args.size
    W = C.wire_size(0, 0, P)
    g = torch.Generator(device=dev)
    g.manual_seed(0x5EED + rank)
    payload = torch.randint(0, 256, (n * P,), dtype=torch.uint8, device=dev, generator=g)
    precom = torch.randint(0, 256, (32,), dtype=torch.uint8, generator=torch.Generator().manual_seed(0x5EED + rank))
    precom = bytes(precom.tolist())

    enc = C.CurveContext(local, 1)
    enc.session_set(0, precom, C.CLIENT_PREFIX, C.SERVER_PREFIX)
    enc.set_nonce(0, 3)  # the handshake used nonces 1 and 2 (curve_client_t: HELLO, INITIATE)
    dec = C.CurveContext(local, 1)
    dec.session_set(0, precom, C.SERVER_PREFIX, C.CLIENT_PREFIX, False, 2)

    i64 = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)
    i32 = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).to(dev)
    sid = i32(np.zeros(n, np.uint32))
    flags_np = np.where(np.arange(n) % 16 == 15, 1, 0).astype(np.uint8)  # 1 in 16 with MORE
    flags = torch.from_numpy(flags_np).to(dev)
    in_off = i64(np.arange(n, dtype=np.uint64) * P)
    lens = i32(np.full(n, P, np.uint32))
    out_off = i64(np.arange(n, dtype=np.uint64) * W)
    wlen = i32(np.full(n, W, np.uint32))
    wire = torch.zeros(n * W, dtype=torch.uint8, device=dev)
    back = torch.zeros(n * P, dtype=torch.uint8, device=dev)
    fl_out = torch.zeros(n, dtype=torch.uint8, device=dev)
    st_out = torch.zeros(n, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)

    # One step = the I/O thread's batch call pair: encode with the nonces the
    # session's send counter assigns on the device (ZMQG_OPT_NONCE_AUTO: the
    # reference's get_and_inc_nonce per message), then decode of that wire.
    # max_len = P: the batcher knows its frames' lengths, and a bound within the
    # frame kernel's range skips the large-frame launches (include/zmqg_curve.h).
    def step_enc(st):
        enc.encode_batch(sid, None, flags, in_off, lens, payload, out_off, wire, st, max_len=P, nonce_auto=True)

    def step(st):
        step_enc(st)
        dec.decode_batch(sid, out_off, wlen, wire, in_off, back, fl_out, st_out, st, max_len=W,
                         stream_out=args.stream_out)

    for _ in range(args.warmup):
        step(stream)
    torch.cuda.synchronize(dev)
    # correctness of the work being timed (the timed steps are checked again below)
    if args.warmup > 0:
        assert int((st_out != 0).sum()) == 0, "decode failures in warmup"
        assert torch.equal(back, payload), "round trip mismatch"
        assert torch.equal(fl_out.cpu(), torch.from_numpy(flags_np)), "flags mismatch"

    # The K timed steps are captured once as a hipGraph (the kernels' per-call
    # state lives on the device, so replays are exact) and replayed as one
    # launch: the host's per-kernel launch cost stays out of the timed region.
    # HIP events cannot time kernels inside a graph, so the per-launch kernel
    # durations (roofline) come from graph replays just before the timed one
    # (graph_shares).  An eager pass of K more steps right after the timed
    # replay gives eager_ms_per_step (host-launched calls, hooks off), and a
    # second one with the ctx profiling hooks on the call spans
    # (roofline.hooked_eager).  --eager times the eager steps (events on)
    # instead.
    graph = None
    if not args.eager:
        try:
            graph = torch.cuda.CUDAGraph()
            cap = torch.cuda.Stream(dev)
            cap.wait_stream(stream)
            with torch.cuda.graph(graph, stream=cap):
                cs = torch.cuda.current_stream(dev)
                for _ in range(args.steps):
                    step(cs)
            torch.cuda.synchronize(dev)
            graph.replay()  # untimed replay: instantiation and first-touch costs
            torch.cuda.synchronize(dev)
        except Exception as e:  # capture unsupported: fall back to eager steps
            print(f"bench: graph capture failed ({e}); timing eager steps", file=sys.stderr)
            graph = None
    # Clock settling: the device ramps its clock over the first ~20 ms of
    # sustained load (tools/replay_series.py: 129 us per step on the first
    # replay, 105 us from the ninth on), so the timed replay follows untimed
    # replays (eager steps without a graph) until --settle-ms of GPU time has
    # passed; each one's time per step is reported beside the line.
    settle_us = []
    settle_t = 0.0
    while settle_t < args.settle_ms and len(settle_us) < 1000:
        s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s0.record(stream)
        if graph is not None:
            graph.replay()
        else:
            for _ in range(args.steps):
                step(stream)
        s1.record(stream)
        torch.cuda.synchronize(dev)
        ms = s0.elapsed_time(s1)
        settle_t += ms
        settle_us.append(round(1e3 * ms / args.steps, 1))
    # The frame kernels' per-launch durations at the timed replay's clock:
    # replays alternating with an encode-only graph, between the settling and
    # the timed replay (the device ramps down within milliseconds of idling,
    # so after the timed replay's checks they would measure another clock).
    if graph is not None:
        enc_avg_s, dec_avg_s, shares = graph_shares(torch, dev, stream, graph, step_enc, args.steps)
    if graph is None:
        enc.set_profiling(True)
        dec.set_profiling(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    g0, g1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    g0.record(stream)
    if graph is not None:
        graph.replay()
    else:
        for _ in range(args.steps):
            step(stream)
    g1.record(stream)
    t_launched = time.perf_counter()
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    # where the timed region's time went: the stream's own span (events
    # around the launch) and the host's launch call
    timed_split = {"stream_span_ms": g0.elapsed_time(g1), "host_launch_ms": 1e3 * (t_launched - t0),
                   "host_total_ms": 1e3 * (t1 - t0)}
    if world > 1:
        dist.barrier()
    elapsed = t1 - t0
    eager_elapsed = None
    if graph is not None:
        # the same K steps launched from the host call by call (what a caller
        # without a graph gets), right after the timed replay while the clock
        # is still up, the profiling hooks off (their event pairs add a
        # dispatch each); host clock
        e0 = time.perf_counter()
        for _ in range(args.steps):
            step(stream)
        torch.cuda.synchronize(dev)
        eager_elapsed = time.perf_counter() - e0
    if graph is not None:  # the replayed (and eager) work is correct too
        assert int((st_out != 0).sum()) == 0 and torch.equal(back, payload), "graph replay mismatch"
        # the call spans of roofline.hooked_eager: one more eager pass, hooks on
        enc.set_profiling(True)
        dec.set_profiling(True)
        for _ in range(args.steps):
            step(stream)
        torch.cuda.synchronize(dev)
    from libzmq_amd import shard
    elapsed = shard.max_over_ranks(elapsed)  # the slowest rank times the job
    # the eager pass's event pairs (the hooks were off during the capture)
    enc_body_ms, enc_body_n = enc.get_profile(C.CurveContext.PROF_ENCODE_MAIN)
    dec_body_ms, dec_body_n = dec.get_profile(C.CurveContext.PROF_DECODE_MAIN)
    enc_call_ms, _ = enc.get_profile(C.CurveContext.PROF_ENCODE_CALL)
    dec_call_ms, _ = dec.get_profile(C.CurveContext.PROF_DECODE_CALL)
    enc.set_profiling(False)
    dec.set_profiling(False)
    assert int((st_out != 0).sum()) == 0
    assert torch.equal(back, payload)
    # per-launch durations of the two frame kernels for the roofline, as they
    # run in the timed replay (graph_shares, measured just before it); without
    # a graph, the hooks' event pairs around each eager launch
    if graph is None:
        enc_avg_s = enc_body_ms / max(enc_body_n, 1) / 1e3
        dec_avg_s = dec_body_ms / max(dec_body_n, 1) / 1e3
        shares = None
    cold = None
    if args.cold_pass:
        ce, cd = launch_pass(torch, dev, stream, enc, dec, args.steps, n, W, P, sid, flags, in_off, lens, payload,
                             out_off, wlen, back, fl_out)
        cold = {"encode_us": ce * 1e6, "decode_us": cd * 1e6,
                "note": f"{args.steps} encodes into {args.steps} wire buffers, then their {args.steps} decodes, each "
                        "run back to back between one event pair: inputs from HBM, not the MALL (launch_pass)"}

    hbm = None
    if args.hbm_sets > 0:
        hbm = hbm_fed(torch, dev, stream, enc, dec, args.hbm_sets, n, W, P, sid, flags, in_off, lens, out_off, wlen,
                      payload)

    total_msgs = n * args.steps * world
    gib = total_msgs * P / 2**30
    value = gib / elapsed
    ms_per_step = 1e3 * elapsed / args.steps

    # roofline of the dominant kernel: the decode frame kernel.  Algorithmic HBM-read
    # bytes of decode per frame: wire W + sid 4 + offset 8 +
    # length 4 = P + 49.
    dec_read = n * (P + 49)
    achieved = dec_read / dec_avg_s / 1e9 if dec_avg_s > 0 else None
    # traffic: HBM read bytes per launch of the same kernel from the committed
    # PMC pass (FETCH_SIZE, doubled per the gfx950 note in MI355X_MICROARCH.md);
    # the write side is reported beside it
    # PMC files count only when they measured THIS library: each carries the
    # source id (zmqg_build_id) of the build its passes loaded
    src_id, commit = C.build_id()
    pmc_notes = {}

    def pmc_file(name):
        path = os.path.join(ROOT, "profiles", name)
        if not (os.path.exists(path) and n == 65536 and P == 1024):
            pmc_notes[name] = "absent"
            return None
        try:
            d = json.load(open(path))
        except Exception:
            pmc_notes[name] = "unreadable"
            return None
        if d.get("kernel") != ROOF_KERNEL:
            pmc_notes[name] = "other kernel"
            return None
        if d.get("source_id") != src_id:
            pmc_notes[name] = f"measured build {d.get('source_id')}, loaded {src_id}: not used"
            return None
        pmc_notes[name] = f"build {src_id} (commit {d.get('commit')})"
        return d

    traffic = traffic_write = None
    d = pmc_file("pmc_traffic_config2.json")
    if d:
        traffic = d.get("read_bytes_per_launch")
        traffic_write = d.get("write_bytes_per_launch")
        # the HBM-fed form's own pass (tools/hbm_probe.py --forms bench, same build)
        hd = (d.get("hbm_fed") or {}).get("decode")
        if hbm and hd:
            hbm["roofline"]["traffic"] = hd.get("read_bytes_per_launch")
            hbm["roofline"]["traffic_write"] = hd.get("write_bytes_per_launch")
            hbm["roofline"]["l2_memory_side_requests"] = hd.get("l2_memory_side_requests_per_launch")
    # The kernel is VALU-issue bound: its VALU
    # instruction count per launch (committed PMC pass) over the same live
    # launch duration, against the chip's VALU issue peak (1024 SIMDs x 16
    # lanes per cycle) at the spec clock and at the clock measured under
    # this load.
    valu = None
    d = pmc_file("pmc_valu_config2.json")
    if d and dec_avg_s > 0:
        try:
            ops = d["valu_wave_instr_per_launch"] * 64 / dec_avg_s
            peak = d["simds"] * d["lanes_per_simd_per_cycle"] * d["clock_ghz_spec"] * 1e9
            peak_m = d["simds"] * d["lanes_per_simd_per_cycle"] * d["clock_ghz_measured"] * 1e9
            valu = {"achieved": ops / 1e12, "peak": peak / 1e12, "unit": "T lane-ops/s", "frac": ops / peak,
                    "frac_at_measured_clock": ops / peak_m, "clock_ghz_measured": d["clock_ghz_measured"],
                    "lane_ops_per_frame": d["valu_lane_ops_per_frame"]}
        except (KeyError, TypeError):
            valu = None
    roofline = {"bound": "hbm", "kernel": ROOF_KERNEL, "achieved": achieved, "peak": HBM_PEAK_GBPS,
                "unit": "GB/s", "frac": (achieved / HBM_PEAK_GBPS) if achieved else None, "traffic": traffic,
                "traffic_write": traffic_write, "valu": valu, "pmc_files": pmc_notes,
                "algorithmic_bytes_per_launch": dec_read, "avg_launch_us": dec_avg_s * 1e6,
                "encode_main_avg_us": enc_avg_s * 1e6,
                "duration_source": "graph replays: (K-step replay - K-encode replay) / K for decode, the K-encode "
                                   "replay / K for encode, medians of 5 alternating replays each, between the "
                                   "settling and the timed replay (graph_shares)" if shares
                                   else "event pairs around each eager launch",
                "graph_shares": shares, "cold_launch_pass": cold,
                "hooked_eager": {"decode_main_us": dec_body_ms / max(dec_body_n, 1) * 1e3,
                                 "encode_main_us": enc_body_ms / max(enc_body_n, 1) * 1e3,
                                 "decode_call_us": dec_call_ms / max(dec_body_n, 1) * 1e3,
                                 "encode_call_us": enc_call_ms / max(enc_body_n, 1) * 1e3},
                "path_read_frac": (n * (2 * P + 74)) / (elapsed / args.steps) / 1e9 / HBM_PEAK_GBPS * world
                if world == 1 else None}

    result = {
        "metric": "GiB/s device-resident CURVE encode+decode, 1 KiB-msg batches; msgs/s",
        "value": value,
        "unit": "GiB/s",
        "msgs_per_s": total_msgs / elapsed,
        "n_gpus": n_devices,
        "ranks": world,
        "shared_devices": shared_devices,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (seeded random payload bytes, random precomputed key)",
        "launch": "hipGraph replay of the K captured steps" if graph is not None else "eager host launches",
        "eager_ms_per_step": 1e3 * (eager_elapsed if eager_elapsed is not None else elapsed) / args.steps,
        "timed_split": timed_split,
        "settle": {"gpu_ms": settle_t, "replays_us_per_step": settle_us},
        "config": {"workload": f"config2: {n} x {P} B frames, 1 CURVE session per GPU, encode+decode round trip",
                   "frames_per_gpu": n, "payload_bytes": P, "wire_bytes": W, "sessions": 1,
                   "parallelism": f"frame-sharded x{world}, no collective"},
        "roofline": roofline,
        "hbm_fed": hbm,
        "build": {"source_id": src_id, "commit": commit},
    }

    if not args.no_configs:
        result["configs"] = other_configs(C, torch, dev, local, rank, world, args.configs.split(","),
                                          settle_ms=args.settle_ms)

    if rank == 0 and world == 1 and not args.no_host_staged:
        result["host_paths"] = host_paths(C, torch, dev, local, payload, precom, flags, flags_np, sid, in_off, lens,
                                          out_off, wlen, n, P, W)
    if rank == 0 and world == 1 and not args.no_deployable:
        result.setdefault("host_paths", {}).update(deployable_paths())

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        port = cpu_baseline(payload.cpu().numpy(), precom, n, P, W, flags_np, args.cpu_seconds)
        ref = cpu_baseline_reference(P, args.cpu_seconds)
        if ref is not None:
            ref["port"] = port
            result["cpu_baseline"] = ref
        else:
            result["cpu_baseline"] = port

    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def graph_shares(torch, dev, stream, graph, step_enc, K, reps=5):
    """Per-launch durations of the encode and decode frame kernels as they
    run in the timed replay.  HIP events cannot time a kernel inside a
    replayed graph, and an event pair around each eager launch also spans
    its dispatch (~5 us), so: a second graph of the K
    steps' encodes alone is captured, and the timed graph and it are
    replayed alternately `reps` times each, every replay between one event
    pair; encode = median(encode-only replay) / K, decode = (median(full
    replay) - median(encode-only replay)) / K -- each a kernel plus its
    launch gap inside a graph, the same inputs and the same cache state as
    the timed steps (the encode-only replays advance the encoder's nonces;
    the decoder accepts the higher ones that follow).  Returns (encode s,
    decode s, the replay times)."""
    ge = torch.cuda.CUDAGraph()
    cap = torch.cuda.Stream(dev)
    cap.wait_stream(stream)
    with torch.cuda.graph(ge, stream=cap):
        cs = torch.cuda.current_stream(dev)
        for _ in range(K):
            step_enc(cs)
    torch.cuda.synchronize(dev)
    ge.replay()  # (untimed: first-replay costs)
    torch.cuda.synchronize(dev)

    def timed(g):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        g.replay()
        b.record(stream)
        torch.cuda.synchronize(dev)
        return a.elapsed_time(b) / 1e3

    full, enc_only = [], []
    for _ in range(reps):
        full.append(timed(graph))
        enc_only.append(timed(ge))
    med = lambda v: sorted(v)[len(v) // 2]
    e = med(enc_only) / K
    d = med(full) / K - e
    return e, d, {"full_replay_ms": [round(1e3 * x, 4) for x in full],
                  "encode_only_replay_ms": [round(1e3 * x, 4) for x in enc_only]}


def launch_pass(torch, dev, stream, enc, dec, K, n, W, P, sid, flags, in_off, lens, payload, out_off, wlen, back,
                fl_out):
    """Per-launch durations of the two frame kernels on inputs read from HBM
    (--cold-pass): K encodes of the batch into K wire buffers (fresh device nonces each),
    back to back on the launch stream between one HIP event pair, then the K
    decodes of those buffers in order (each a valid batch of the session),
    between another; each kernel's duration = its pair's span / K.  (An
    event pair around every single launch -- the ctx profiling hooks of the
    eager pass, `hooked_eager` -- also spans that launch's dispatch, ~5 us
    here: DESIGN.md section 4.)  Every decode's statuses and payload are
    checked.  Returns (encode s, decode s)."""
    wires = [torch.empty(n * W, dtype=torch.uint8, device=dev) for _ in range(K)]
    sts = [torch.full((n,), -1, dtype=torch.int32, device=dev) for _ in range(K)]
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    torch.cuda.synchronize(dev)
    ev[0].record(stream)
    for w in wires:
        enc.encode_batch(sid, None, flags, in_off, lens, payload, out_off, w, stream, max_len=P, nonce_auto=True)
    ev[1].record(stream)
    ev[2].record(stream)
    for w, st in zip(wires, sts):
        dec.decode_batch(sid, out_off, wlen, w, in_off, back, fl_out, st, stream, max_len=W)
    ev[3].record(stream)
    torch.cuda.synchronize(dev)
    assert all(int((st != 0).sum()) == 0 for st in sts), "launch pass: decode failures"
    assert torch.equal(back, payload), "launch pass: round trip mismatch"
    return ev[0].elapsed_time(ev[1]) / K / 1e3, ev[2].elapsed_time(ev[3]) / K / 1e3


def hbm_fed(torch, dev, stream, enc, dec, K, n, W, P, sid, flags, in_off, lens, out_off, wlen, payload):
    """Config 2 with every input fed from HBM (verdict r5 item 2): K batches,
    each with its own payload, wire and result buffers (K x ~200 MB, against
    the 256 MiB Infinity Cache), encoded back to back between one event pair
    (each reads a payload last touched K batches ago), then decoded back to
    back between another (each reads a wire written K encodes ago).  Rate =
    the K round trips' payload over the two spans; per-launch durations =
    span / K, with the decode frame kernel's roofline as in the main line.
    Every decode's statuses and payload are checked."""
    g = torch.Generator(device=dev)
    g.manual_seed(0xFEED)
    pays = [payload] + [torch.randint(0, 256, (n * P,), dtype=torch.uint8, device=dev, generator=g)
                        for _ in range(K - 1)]
    wires = [torch.empty(n * W, dtype=torch.uint8, device=dev) for _ in range(K)]
    backs = [torch.empty(n * P, dtype=torch.uint8, device=dev) for _ in range(K)]
    fls = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(K)]
    sts = [torch.full((n,), -1, dtype=torch.int32, device=dev) for _ in range(K)]

    def run():
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        ev[0].record(stream)
        for k in range(K):
            enc.encode_batch(sid, None, flags, in_off, lens, pays[k], out_off, wires[k], stream, max_len=P,
                             nonce_auto=True, stream_out=True)
        ev[1].record(stream)
        ev[2].record(stream)
        for k in range(K):
            dec.decode_batch(sid, out_off, wlen, wires[k], in_off, backs[k], fls[k], sts[k], stream, max_len=W,
                             stream_out=True)
        ev[3].record(stream)
        torch.cuda.synchronize(dev)
        return ev[0].elapsed_time(ev[1]) / 1e3, ev[2].elapsed_time(ev[3]) / 1e3

    run()  # first touch of the new buffers; the clock stays up from the main line
    es, ds = run()
    for k in range(K):
        assert int((sts[k] != 0).sum()) == 0 and torch.equal(backs[k], pays[k]), "hbm_fed: round trip mismatch"
    e, d = es / K, ds / K
    dec_read = n * (P + 49)
    achieved = dec_read / d / 1e9
    out = {"value": K * n * P / 2**30 / (es + ds), "unit": "GiB/s", "msgs_per_s": K * n / (es + ds),
           "ms_per_step": 1e3 * (es + ds) / K, "encode_us": e * 1e6, "decode_us": d * 1e6,
           "roofline": {"bound": "hbm", "kernel": ROOF_KERNEL, "achieved": achieved, "peak": HBM_PEAK_GBPS,
                        "unit": "GB/s", "frac": achieved / HBM_PEAK_GBPS, "algorithmic_bytes_per_launch": dec_read,
                        "avg_launch_us": d * 1e6},
           "sets": K, "bytes_per_set": n * (2 * P + W),
           "note": f"{K} config-2 batches with their own buffers ({K * n * (2 * P + W) / 2**20:.0f} MiB against "
                   f"the 256 MiB Infinity Cache): {K} encodes back to back, then their {K} decodes, one event pair "
                   "each; every input comes from HBM; encodes and decodes pass ZMQG_OPT_STREAM_OUT, the cache hint "
                   "for outputs no cache holds (staged whole-window stores, 16 frames per store instruction)"}
    del pays, wires, backs
    torch.cuda.empty_cache()
    return out


def device_census(torch, world, local):
    """(distinct physical GPUs the ranks run on, whether ranks share one).
    Each rank names its device by host and PCI location (UUID when torch
    exposes it); the names are gathered over the control-plane group, so a
    rehearsal with more ranks than GPUs cannot report more GPUs than it used."""
    import socket
    p = torch.cuda.get_device_properties(local)
    uuid = str(getattr(p, "uuid", "") or "")
    pci = tuple(getattr(p, f, -1) for f in ("pci_domain_id", "pci_bus_id", "pci_device_id"))
    name = (socket.gethostname(), uuid if uuid else (pci if pci != (-1, -1, -1) else ("index", local)))
    names = [name]
    if world > 1:
        import torch.distributed as dist
        names = [None] * world
        dist.all_gather_object(names, name)
    n = len(set(names))
    if world > torch.cuda.device_count():  # (one node: ranks beyond its GPUs must share)
        n = min(n, torch.cuda.device_count())
    return n, n < world


def config_batches(which, rank, world):
    """Per-rank share of BASELINE configs 3-5: (name, sizes, sessions, scaling, note).
    Config 3 is one GPU's batch (run on every rank: weak); configs 4 and 5
    split one batch over the ranks with shard.partition (strong scaling),
    each session's frames on one rank, so there is no exchange."""
    from libzmq_amd import shard
    if which == "3":
        rng = np.random.default_rng(3 + rank)
        return ("config3: 49,152 frames of {64 B, 1 KiB, 64 KiB}, 256 sessions per GPU",
                rng.choice([64, 1024, 65536], 49152).astype(np.int64), 256, "weak")
    if which == "4":
        n_all, size, S = 16 << 20, 256, 1024
    elif which == "5":
        n_all, size, S = 1 << 10, 16 << 20, 8
    else:
        raise ValueError(which)
    lo, hi = shard.partition(shard.stream_blocks(np.full(n_all, 33 + size, np.int64)), world)[rank]
    name = ("config4: 16 Mi x 256 B frames, 1024 sessions, split over the GPUs" if which == "4" else
            "config5: 1 Ki x 16 MiB frames, 8 sessions, split over the GPUs")
    return name, np.full(hi - lo, size, np.int64), max(1, S // world), "strong"


def config_inputs(C, torch, dev, local, rank, w, world=1):
    """The device-resident batch and sessions of BASELINE config `w` as
    other_configs times it (tests/test_gpu_bench_batches.py checks this exact
    batch against the oracle): sizes from config_batches, session keys from
    a seeded rng, payload from a seeded device generator, frames packed back
    to back, a connection's frames together, encode nonces from each
    session's send counter starting at 3."""
    name, sizes, S, scaling = config_batches(w, rank, world)
    n = len(sizes)
    g = torch.Generator(device=dev)
    g.manual_seed(0xC0 + 7 * rank + int(w))
    enc, dec = C.CurveContext(local, S), C.CurveContext(local, S)
    rng = np.random.default_rng(0xC0 + rank)
    keys = [rng.integers(0, 256, 32, dtype=np.uint8).tobytes() for _ in range(S)]
    # one install launch per context (zmqg_session_set_batch_ex): the client
    # side continues from nonce 3 after HELLO and INITIATE, the server expects
    # peer nonces above 2
    precom = torch.from_numpy(np.frombuffer(b"".join(keys), np.uint8).copy()).to(dev)
    enc.session_set_batch(np.arange(S), precom, C.CLIENT_PREFIX, C.SERVER_PREFIX, send_nonce=np.full(S, 3))
    dec.session_set_batch(np.arange(S), precom, C.SERVER_PREFIX, C.CLIENT_PREFIX, peer_nonce=np.full(S, 2))
    torch.cuda.current_stream(dev).synchronize()
    t = lambda a, d: torch.from_numpy(np.ascontiguousarray(a).view(d)).to(dev)
    in_off = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64)
    W = sizes + 33
    out_off = np.concatenate([[0], np.cumsum(W)[:-1]]).astype(np.uint64)
    sid = (np.arange(n) * S // max(n, 1)).astype(np.uint32)  # a connection's frames together
    total = int(sizes.sum())
    ml = int(sizes.max())
    return dict(name=name, sizes=sizes, S=S, scaling=scaling, n=n, keys=keys, enc=enc, dec=dec, sid=sid,
                in_off=in_off, out_off=out_off, W=W, total=total,
                d_sid=t(sid, np.int32), d_in=t(in_off, np.int64), d_out=t(out_off, np.int64),
                d_len=t(sizes.astype(np.uint32), np.int32), d_wl=t(W.astype(np.uint32), np.int32),
                flags=torch.zeros(n, dtype=torch.uint8, device=dev),
                payload=torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev, generator=g),
                wire=torch.empty(int(W.sum()), dtype=torch.uint8, device=dev),
                back=torch.empty(total, dtype=torch.uint8, device=dev),
                fl=torch.empty(n, dtype=torch.uint8, device=dev), st=torch.empty(n, dtype=torch.int32, device=dev),
                bound=ml if ml + 43 <= 4608 else 0)  # the frame kernel's range: skip the large-frame launches


def config_step(b):
    """One timed step of a config: encode with device-assigned nonces, decode."""
    b["enc"].encode_batch(b["d_sid"], None, b["flags"], b["d_in"], b["d_len"], b["payload"], b["d_out"], b["wire"],
                          max_len=b["bound"], nonce_auto=True)
    b["dec"].decode_batch(b["d_sid"], b["d_out"], b["d_wl"], b["wire"], b["d_in"], b["back"], b["fl"], b["st"],
                          max_len=b["bound"] + 33 if b["bound"] else 0)


def other_configs(C, torch, dev, local, rank, world, which, steps=10, warmup=1, settle_ms=40.0):
    """BASELINE configs 3, 4, 5: encode (device-assigned nonces) + decode round
    trips of device-resident batches, every result checked, timed like the
    main line (barrier + synchronize, max over ranks); payload GiB/s of the
    whole job.  Untimed warmup steps: at least `warmup`, and more until
    settle_ms of GPU time has passed since the last idle gap (the clock ramp,
    DESIGN.md section 4; the inputs' preparation idles the device)."""
    import torch.distributed as dist
    from libzmq_amd import shard
    out = {}
    for w in which:
        b = config_inputs(C, torch, dev, local, rank, w, world)
        name, S, scaling, n, total = b["name"], b["S"], b["scaling"], b["n"], b["total"]
        wu, gpu_ms = 0, 0.0
        while wu < warmup or (gpu_ms < settle_ms and wu < 200):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            config_step(b)
            e1.record()
            torch.cuda.synchronize(dev)
            gpu_ms += e0.elapsed_time(e1)
            wu += 1
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            config_step(b)
        torch.cuda.synchronize(dev)
        dt = shard.max_over_ranks(time.perf_counter() - t0)
        ok = int((b["st"] != 0).sum()) == 0 and torch.equal(b["back"], b["payload"])
        oks = shard.max_over_ranks(0.0 if ok else 1.0) == 0.0
        assert oks, f"config {w}: round trip mismatch"
        job_bytes = total * world if scaling == "weak" else sum_over_ranks(total)
        job_frames = n * world if scaling == "weak" else sum_over_ranks(n)
        out["config" + w] = {"workload": name, "scaling": scaling, "value": job_bytes / 2**30 * steps / dt,
                             "unit": "GiB/s", "msgs_per_s": job_frames * steps / dt, "ms_per_step": 1e3 * dt / steps,
                             "frames_per_gpu": n, "sessions_per_gpu": S, "steps": steps, "warmup": wu,
                             "warmup_gpu_ms": gpu_ms,
                             "checked": "every frame: status 0, decoded payload == input; the same batch is "
                                        "oracle-checked by tests/test_gpu_bench_batches.py"}
        del b
        torch.cuda.empty_cache()
    return out


def sum_over_ranks(v):
    import torch
    import torch.distributed as dist
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return float(v)
    x = torch.tensor([float(v)], dtype=torch.float64)
    dist.all_reduce(x)
    return float(x.item())


def host_paths(C, torch, dev, local, payload, precom, flags, flags_np, sid, in_off, lens, out_off, wlen, n, P, W):
    """PCIe-inclusive round-trip rates (payload GiB/s of encode+decode), the
    batch starting and ending in host memory:
      zerocopy_pinned  payload, wire and result in pinned host memory, which
                       the kernels read and write in place over PCIe
                       (descriptors in HBM) -- the curve_batcher_t path
      pageable_staged  zmqg_encode_host / zmqg_decode_host from pageable
                       buffers (host memcpy into pinned staging, H2D, kernels,
                       D2H, memcpy out)"""
    out = {}
    hp = payload.cpu().pin_memory()
    wire_h = torch.zeros(n * W, dtype=torch.uint8).pin_memory()
    back_h = torch.zeros(n * P, dtype=torch.uint8).pin_memory()
    zenc = C.CurveContext(local, 1)
    zenc.session_set(0, precom, C.CLIENT_PREFIX, C.SERVER_PREFIX)
    zdec = C.CurveContext(local, 1)
    zdec.session_set(0, precom, C.SERVER_PREFIX, C.CLIENT_PREFIX, False, 2)
    fl = torch.zeros(n, dtype=torch.uint8, device=dev)
    st = torch.zeros(n, dtype=torch.int32, device=dev)
    nonces = [torch.from_numpy(np.arange(3 + r * n, 3 + (r + 1) * n, dtype=np.uint64).view(np.int64)).to(dev)
              for r in range(5)]
    torch.cuda.synchronize(dev)
    t0 = None
    for r in range(5):  # the first round trip is untimed
        if r == 1:
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
        zenc.encode_batch(sid, nonces[r], flags, in_off, lens, hp, out_off, wire_h)
        zdec.decode_batch(sid, out_off, wlen, wire_h, in_off, back_h, fl, st)
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    assert int((st != 0).sum()) == 0 and torch.equal(back_h, hp), "zero-copy round trip"
    out["zerocopy_pinned"] = {"value": 4 * n * P / 2**30 / (t1 - t0), "unit": "GiB/s",
                              "note": "encode+decode, kernels on pinned host memory over PCIe"}

    place = gpu_placement(torch, local)
    place["payload_buffer_node"] = page_node(hp.data_ptr())
    out["pinned_dma"] = pinned_dma(C, torch, dev, local, hp, precom, flags, flags_np, n, P, W)
    out["pinned_dma"]["placement"] = place
    # the same with the pinned buffers allocated (and this thread running) on
    # the GPU's own NUMA node, when that is not where they were
    try:
        gnode = int(place.get("numa_node") or -1)
    except ValueError:
        gnode = -1
    cpus = node_cpus(gnode) if gnode >= 0 else set()
    if cpus and place["payload_buffer_node"] not in (None, gnode):
        keep = os.sched_getaffinity(0)
        try:
            os.sched_setaffinity(0, cpus)
            hpl = payload.cpu().pin_memory()
            local_dma = pinned_dma(C, torch, dev, local, hpl, precom, flags, flags_np, n, P, W)
            local_dma["payload_buffer_node"] = page_node(hpl.data_ptr())
            out["pinned_dma_gpu_node"] = local_dma
        finally:
            os.sched_setaffinity(0, keep)

    hpn = hp.numpy()
    hin = np.arange(n, dtype=np.uint64) * P
    hout = np.arange(n, dtype=np.uint64) * W
    hctx = C.CurveContext(local, 1)
    hctx.session_set(0, precom, C.CLIENT_PREFIX, C.SERVER_PREFIX)
    hdec = C.CurveContext(local, 1)
    hdec.session_set(0, precom, C.SERVER_PREFIX, C.CLIENT_PREFIX, False, 2)
    z32 = np.zeros(n, np.uint32)
    lens_h = np.full(n, P, np.uint32)
    wl_h = np.full(n, W, np.uint32)
    reps = 3
    t0 = time.perf_counter()
    for r in range(reps):
        nn = np.arange(3 + r * n, 3 + (r + 1) * n, dtype=np.uint64)
        w = hctx.encode_host(z32, nn, flags_np, hin, lens_h, hpn, hout, n * W)
        pl, _, stt = hdec.decode_host(z32, hout, wl_h, w, hin, n * P)
    t1 = time.perf_counter()
    assert (stt == 0).all() and np.array_equal(pl, hpn)
    out["pageable_staged"] = {"value": reps * n * P / 2**30 / (t1 - t0), "unit": "GiB/s",
                              "note": "zmqg_encode_host + zmqg_decode_host, pageable buffers, H2D+D2H included"}
    return out


def page_node(addr):
    """NUMA node holding the page at host address `addr` (get_mempolicy with
    MPOL_F_NODE | MPOL_F_ADDR), or None."""
    import ctypes
    try:
        libc = ctypes.CDLL(None, use_errno=True)
        mode = ctypes.c_int(-1)
        rc = libc.syscall(239, ctypes.byref(mode), None, ctypes.c_ulong(0), ctypes.c_void_p(addr), ctypes.c_ulong(3))
        return mode.value if rc == 0 else None
    except Exception:
        return None


def gpu_placement(torch, local):
    """The GPU's PCIe link and NUMA node (sysfs), and the NUMA nodes of the
    CPUs this process may run on (verdict r5 item 7: the pinned-DMA rate's
    spread from box to box)."""
    def rd(path):
        try:
            return open(path).read().strip()
        except OSError:
            return None
    p = torch.cuda.get_device_properties(local)
    addr = None
    dom, bus, devn = (getattr(p, f, None) for f in ("pci_domain_id", "pci_bus_id", "pci_device_id"))
    if bus is not None:
        addr = f"{dom or 0:04x}:{bus:02x}:{devn:02x}.0"
    out = {"pci": addr}
    if addr:
        base = f"/sys/bus/pci/devices/{addr}"
        for k in ("numa_node", "current_link_width", "current_link_speed", "max_link_width", "max_link_speed"):
            out[k] = rd(f"{base}/{k}")
    nodes = set()
    for c in os.sched_getaffinity(0):
        try:
            nodes.update(int(x[4:]) for x in os.listdir(f"/sys/devices/system/cpu/cpu{c}") if x.startswith("node"))
        except OSError:
            pass
    out["process_cpu_nodes"] = sorted(nodes)
    return out


def node_cpus(node):
    """The CPUs of NUMA node `node` this process may use."""
    try:
        txt = open(f"/sys/devices/system/node/node{node}/cpulist").read().strip()
    except OSError:
        return set()
    cpus = set()
    for part in txt.split(","):
        a, _, b = part.partition("-")
        cpus.update(range(int(a), int(b or a) + 1))
    return cpus & os.sched_getaffinity(0)


def pinned_dma(C, torch, dev, local, hp, precom, flags, flags_np, n, P, W, chunks=8, reps=4):
    """The north_star's host-memory round trip through pinned hipMemcpyAsync:
    payload and wire in pinned host buffers (the I/O thread's socket side),
    the batch cut into `chunks` slices, each path on its own three streams --
      send path:    H2D payload slice -> encode -> D2H wire slice
      receive path: H2D wire slice (the bytes just sent) -> decode -> D2H payload
    -- so copies of one slice overlap the kernels and copies of the others
    (device buffers per slice).  Every byte
    crosses PCIe four times per round trip (P + W each way), as in the
    zero-copy form.  Payload GiB/s of round trips, whole batch checked."""
    m = n // chunks
    assert m * chunks == n
    i64 = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)
    i32 = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).to(dev)
    enc = C.CurveContext(local, 1)
    enc.session_set(0, precom, C.CLIENT_PREFIX, C.SERVER_PREFIX)
    enc.set_nonce(0, 3)
    dec = C.CurveContext(local, 1)
    dec.session_set(0, precom, C.SERVER_PREFIX, C.CLIENT_PREFIX, False, 2)
    sid = i32(np.zeros(m, np.uint32))
    in_off = i64(np.arange(m, dtype=np.uint64) * P)
    out_off = i64(np.arange(m, dtype=np.uint64) * W)
    lens = i32(np.full(m, P, np.uint32))
    wlen = i32(np.full(m, W, np.uint32))
    wire_h = torch.zeros(n * W, dtype=torch.uint8).pin_memory()
    back_h = torch.zeros(n * P, dtype=torch.uint8).pin_memory()
    d_pay = [torch.empty(m * P, dtype=torch.uint8, device=dev) for _ in range(chunks)]
    d_wire = [torch.empty(m * W, dtype=torch.uint8, device=dev) for _ in range(chunks)]
    d_wire2 = [torch.empty(m * W, dtype=torch.uint8, device=dev) for _ in range(chunks)]
    d_back = [torch.empty(m * P, dtype=torch.uint8, device=dev) for _ in range(chunks)]
    fl = [torch.empty(m, dtype=torch.uint8, device=dev) for _ in range(chunks)]
    st = [torch.empty(m, dtype=torch.int32, device=dev) for _ in range(chunks)]
    fls = [flags[c * m:(c + 1) * m] for c in range(chunks)]
    # The send and the receive pipeline each get their own copy streams in
    # both directions and their own compute stream, so a slice's receive
    # copies never queue behind another slice's send copies (one H2D stream
    # for both measured 5.3 GiB/s: its in-order queue waited on the D2H of
    # the wire it was about to read back).
    S_ = lambda: torch.cuda.Stream(dev)
    s_h2d, s_comp, s_d2h = S_(), S_(), S_()
    r_h2d, r_comp, r_d2h = S_(), S_(), S_()
    ev = lambda: torch.cuda.Event()

    def one():
        sent = [None] * chunks
        for q in (s_h2d, r_h2d):  # the previous round trip's readers of the slice buffers are done
            for w in (s_comp, s_d2h, r_comp, r_d2h):
                q.wait_stream(w)
        for c in range(chunks):  # send pipeline
            with torch.cuda.stream(s_h2d):
                d_pay[c].copy_(hp[c * m * P:(c + 1) * m * P], non_blocking=True)
                a = ev()
                a.record(s_h2d)
            s_comp.wait_event(a)
            enc.encode_batch(sid, None, fls[c], in_off, lens, d_pay[c], out_off, d_wire[c], s_comp, max_len=P,
                             nonce_auto=True)
            b = ev()
            b.record(s_comp)
            s_d2h.wait_event(b)
            with torch.cuda.stream(s_d2h):
                wire_h[c * m * W:(c + 1) * m * W].copy_(d_wire[c], non_blocking=True)
                sent[c] = ev()
                sent[c].record(s_d2h)
        for c in range(chunks):  # receive pipeline: the wire as it left
            r_h2d.wait_event(sent[c])
            with torch.cuda.stream(r_h2d):
                d_wire2[c].copy_(wire_h[c * m * W:(c + 1) * m * W], non_blocking=True)
                a = ev()
                a.record(r_h2d)
            r_comp.wait_event(a)
            dec.decode_batch(sid, out_off, wlen, d_wire2[c], in_off, d_back[c], fl[c], st[c], r_comp, max_len=W)
            b = ev()
            b.record(r_comp)
            r_d2h.wait_event(b)
            with torch.cuda.stream(r_d2h):
                back_h[c * m * P:(c + 1) * m * P].copy_(d_back[c], non_blocking=True)

    one()  # untimed: first touch
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(reps):
        one()
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    assert all(int((s != 0).sum()) == 0 for s in st) and torch.equal(back_h, hp), "pinned DMA round trip"
    return {"value": reps * n * P / 2**30 / (t1 - t0), "unit": "GiB/s",
            "note": f"encode+decode round trip, pinned host buffers, hipMemcpyAsync H2D/D2H, send and receive "
                    f"pipelines on their own copy and compute streams, {chunks} slices (P + W bytes each way per "
                    f"message)"}


def deployable_paths():
    """What a libzmq user gets from the batched codec (verdict r5 item 4):
      engine_hook    tests/host/test_engine_hook.cpp bench -- two epoll I/O
                     threads, client engines encoding on the GPU, socketpairs,
                     server engines decoding on the GPU (curve_io_hook_t /
                     curve_engine_link_t), messages/s;
      libzmq_pairs   CURVE PUSH/PULL over tcp://127.0.0.1 between two builds
                     of the reference libzmq (tests/host/build_libzmq.sh):
                     stock (libsodium) and zmqgb (the batched GPU codec inside
                     the stream engine), 1,000,000 messages of config 1's plan
                     per run, receiver's msg/s, runs interleaved
                     (tools/libzmq_pair_bench.py)."""
    import subprocess
    out = {}
    exe = os.path.join(ROOT, "tests", "host", "bin", "engine_hook_bench")
    if os.path.exists(exe):
        runs = {}
        for conns, msgs, size in ((16, 20000, 1024), (64, 20000, 256)):
            r = subprocess.run(["timeout", "-k", "10", "120", exe, "bench", str(conns), str(msgs), str(size)],
                               capture_output=True, text=True)
            f = r.stdout.split()
            if r.returncode == 0 and f and f[0] == "RATE":
                runs[f"{conns}x{msgs}x{size}B"] = {"msgs_per_s": float(f[f.index("msgs_per_s") + 1]),
                                                    "payload_MB_per_s": float(f[f.index("payload_MB_per_s") + 1])}
            else:
                runs[f"{conns}x{msgs}x{size}B"] = {"error": (r.stderr or r.stdout)[-300:]}
        out["engine_hook"] = {"runs": runs, "unit": "msgs/s",
                              "note": "tests/host/test_engine_hook.cpp bench: two epoll I/O threads, GPU encode "
                                      "and decode through curve_io_hook_t, non-blocking socketpairs"}
    else:
        out["engine_hook"] = None
    try:
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import libzmq_pair_bench as lpb
        if os.path.exists(os.path.join(lpb.BIN, "interop_zmqgb")):
            r = lpb.run((("stock", "stock"), ("zmqgb", "zmqgb")), reps=3, n=1000000)
            out["libzmq_pairs"] = {k: {"msgs_per_s": v["msgs_per_s"], "median_msgs_per_s": v["median_msgs_per_s"]}
                                   for k, v in r.items()}
            out["libzmq_pairs"]["note"] = ("CURVE PUSH/PULL over tcp://127.0.0.1, 1,000,000 messages (1 KiB plus "
                                           "config 1's 0 B - 64 KiB and multipart ones), every byte checked, "
                                           "heartbeats every 5 ms; stock = reference libzmq + libsodium, zmqgb = "
                                           "the same sources with the batched GPU codec in the stream engine")
        else:
            out["libzmq_pairs"] = None
    except Exception as e:  # a failed pairing is reported, not fatal to the line
        out["libzmq_pairs"] = {"error": str(e)[-300:]}
    return out


def cpu_baseline_reference(P, seconds):
    """cpu_baseline of kind "reference": the stock libzmq build's own
    zmq::curve_encoding_t (src/curve_mechanism_base.cpp compiled where it lies,
    libsodium 1.0.18), driven as unittests/unittest_curve_encoding.cpp:26-71
    drives it -- tests/host/curve_encoding_ref_bench.cpp, one client/server
    pair per thread, every decoded payload checked.  None when the program was
    not built (no reference at build time)."""
    import subprocess
    exe = os.path.join(ROOT, "tests", "host", "_ref", "libzmq", "curve_encoding_ref_bench")
    if not os.path.exists(exe):
        return None
    threads, affinity, quota = host_cores()
    r = subprocess.run(["timeout", "-k", "10", str(int(seconds) + 60), exe, str(threads), str(P), str(seconds)],
                       capture_output=True, text=True)
    f = r.stdout.split()
    if r.returncode != 0 or not f or f[0] != "RATE":
        return None
    msgs_s = float(f[f.index("msgs_per_s") + 1])
    return {"value": float(f[f.index("payload_GiB_per_s") + 1]), "unit": "GiB/s", "cores": threads,
            "affinity_cpus": affinity, "cgroup_cpu_quota": quota, "host_cpus": os.cpu_count(), "kind": "reference",
            "msgs_per_s": msgs_s,
            "sample": f"{int(f[f.index('msgs') + 1])} encode+decode round trips of {P} B over "
                      f"{float(f[f.index('seconds') + 1]):.2f} s on {threads} threads: the stock build's "
                      "zmq::curve_encoding_t (tests/host/curve_encoding_ref_bench.cpp)"}


def host_cores():
    """(threads to use, CPUs in the affinity mask, cgroup v2 CPU quota or None)."""
    affinity = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, -(-int(q) // int(period)))
    except (OSError, ValueError):
        pass
    return (min(affinity, quota) if quota else affinity), affinity, quota


def cpu_baseline(payload, precom, n, P, W, flags_np, seconds):
    from oracle import oracle as O

    # one thread per host core this process may use (every
    # core): the CPUs in its affinity mask, capped by its cgroup CPU quota
    # (a GPU box's share of a larger host: the mask shows the whole host)
    threads, affinity, quota = host_cores()
    # sessions partitioned across threads (one I/O thread owns a connection)
    S = threads
    sess = O.make_sessions([precom] * S)
    sid = (np.arange(n) % S).astype(np.uint32)
    nonce = np.arange(3, 3 + n, dtype=np.uint64)
    in_off = np.arange(n, dtype=np.uint64) * P
    lens = np.full(n, P, np.uint32)
    wire_off = np.arange(n, dtype=np.uint64) * W
    kind = "libsodium 1.0.18 crypto_box_easy_afternm/open (dlopen)"
    secs, ok = O.bench_roundtrip(True, threads, sess, sid, nonce, flags_np, in_off, lens, payload, wire_off, n * W)
    use_sodium = secs is not None
    if not use_sodium:
        kind = "portable C XSalsa20-Poly1305 restatement"
    total_s, passes, oks = 0.0, 0, 0
    while total_s < seconds or passes < 2:
        s, ok = O.bench_roundtrip(use_sodium, threads, sess, sid, nonce, flags_np, in_off, lens, payload, wire_off,
                                  n * W)
        total_s += s
        passes += 1
        oks += ok
    assert oks == passes * n
    return {"value": passes * n * P / 2**30 / total_s, "unit": "GiB/s", "cores": threads,
            "affinity_cpus": affinity, "cgroup_cpu_quota": quota, "host_cpus": os.cpu_count(), "kind": "port",
            "msgs_per_s": passes * n / total_s,
            "sample": f"{passes} passes x {n} x {P} B encode+decode round trips ({total_s:.2f} s wall, "
                      f"{threads} threads, {S} sessions); crypto: {kind}; framing: oracle/curve_oracle.c "
                      f"restatement of curve_encoding_t"}


if __name__ == "__main__":
    main()
