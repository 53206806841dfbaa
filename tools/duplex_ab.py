#!/usr/bin/env python3
"""A/B of the pipelined step (zmqg_duplex_batch: decode of batch k-1 and
encode of batch k in one launch) against the sequential one (encode batch k,
then decode it), both as bench.py times them: K steps captured as one
hipGraph, replayed; config 2 (65,536 x 1 KiB, one session) by default.
Checks every decode's status and the round trip after the timed replays.
ZMQG_DUPLEX_LDS (bytes) sets the duplex launch's dynamic LDS (0: workgroups
co-resident); ZMQG_DUPLEX_OFF runs the pair as two calls.

  duplex_ab.py [--msgs N] [--size P] [--steps K] [--reps R]"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from libzmq_amd import curve as C  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--msgs", type=int, default=65536)
ap.add_argument("--size", type=int, default=1024)
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--modes", default="sequential,pipelined")
a = ap.parse_args()
assert a.steps % 2 == 0
dev = torch.device("cuda", 0)
n, P = a.msgs, a.size
W = C.wire_size(0, 0, P)
t = lambda x, d: torch.from_numpy(np.ascontiguousarray(x).view(d)).to(dev)
payload = torch.randint(0, 256, (n * P,), dtype=torch.uint8, device=dev)
key = bytes(range(32))
sid = t(np.zeros(n, np.uint32), np.int32)
flags = t(np.where(np.arange(n) % 16 == 15, 1, 0).astype(np.uint8), np.uint8)
in_off = t(np.arange(n, dtype=np.uint64) * P, np.int64)
lens = t(np.full(n, P, np.uint32), np.int32)
out_off = t(np.arange(n, dtype=np.uint64) * W, np.int64)
wl = t(np.full(n, W, np.uint32), np.int32)
wire = [torch.zeros(n * W, dtype=torch.uint8, device=dev) for _ in range(2)]
back = torch.zeros(n * P, dtype=torch.uint8, device=dev)
fl = torch.zeros(n, dtype=torch.uint8, device=dev)
st = torch.zeros(n, dtype=torch.int32, device=dev)


def ctxs():
    enc = C.CurveContext(0, 1)
    enc.session_set(0, key, C.CLIENT_PREFIX, C.SERVER_PREFIX)
    enc.set_nonce(0, 3)
    dec = C.CurveContext(0, 1)
    dec.session_set(0, key, C.SERVER_PREFIX, C.CLIENT_PREFIX, False, 2)
    return enc, dec


def eargs(w):
    return dict(sid=sid, nonce=None, flags=flags, in_off=in_off, length=lens, inp=payload, out_off=out_off, out=w,
                max_len=P, nonce_auto=True)


def dargs(w):
    return dict(sid=sid, in_off=out_off, wire_len=wl, inp=w, out_off=in_off, out=back, flags_out=fl, status_out=st,
                max_len=W)


def run(mode):
    enc, dec = ctxs()
    s = torch.cuda.current_stream(dev)
    if mode == "pipelined":
        enc.encode_batch(**eargs(wire[1]), stream=s)  # the pipeline's fill

        def step(j, cs):
            dec.duplex_batch(dargs(wire[(j + 1) % 2]), (enc, eargs(wire[j % 2])), stream=cs)
    else:
        def step(j, cs):
            enc.encode_batch(**eargs(wire[0]), stream=cs)
            dec.decode_batch(**dargs(wire[0]), stream=cs)
    for j in range(4):  # warmup (even: the buffers' parity is kept)
        step(j, s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    cap = torch.cuda.Stream(dev)
    cap.wait_stream(s)
    with torch.cuda.graph(g, stream=cap):
        cs = torch.cuda.current_stream(dev)
        for j in range(a.steps):
            step(j, cs)
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    us = []
    for _ in range(a.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        g.replay()
        e1.record(s)
        torch.cuda.synchronize()
        us.append(e0.elapsed_time(e1) * 1e3 / a.steps)
    ok = bool((st == 0).all().item()) and bool(torch.equal(back, payload))
    # eager steps with the profiling hooks: the frame-kernel launch durations
    enc.set_profiling(True)
    dec.set_profiling(True)
    for j in range(a.steps):
        step(j, s)
    torch.cuda.synchronize()
    ok = ok and bool((st == 0).all().item()) and bool(torch.equal(back, payload))
    dm, dn = dec.get_profile(C.CurveContext.PROF_DECODE_MAIN)
    em, en = enc.get_profile(C.CurveContext.PROF_ENCODE_MAIN)
    reps = [round(u, 1) for u in us]
    us.sort()
    return {"mode": mode, "reps_us": reps, "step_us_median": us[len(us) // 2], "step_us_min": us[0],
            "gib_s": n * P / 2**30 / (us[len(us) // 2] * 1e-6), "dec_main_us": dm / max(dn, 1) * 1e3,
            "enc_main_us": em / max(en, 1) * 1e3, "ok": ok}


for m in a.modes.split(","):
    r = run(m)
    r.update(msgs=n, size=P, duplex_lds=os.environ.get("ZMQG_DUPLEX_LDS", "default"),
             duplex_off=bool(os.environ.get("ZMQG_DUPLEX_OFF")))
    print(json.dumps(r), flush=True)
