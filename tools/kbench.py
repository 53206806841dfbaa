#!/usr/bin/env python3
"""Kernel timing probe (experiments): times encode/decode frame kernels (and
the chunked body kernel, when the frames are above 4.5 KiB) and
whole calls with the ctx profiling hooks.  ZMQG_CURVE_LIB selects a build.
Outputs are not checked (ablation builds compute garbage on purpose)."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from libzmq_amd import curve as C  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--msgs", type=int, default=65536)
ap.add_argument("--size", type=int, default=1024)
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--sessions", type=int, default=1)
ap.add_argument("--tag", default=os.environ.get("ZMQG_CURVE_LIB", "default"))
ap.add_argument("--wire-align", type=int, default=1, help="wire frames at multiples of this many bytes")
ap.add_argument("--sid-mod", action="store_true", help="frame i on session i mod sessions (bench config 4) "
                "instead of contiguous blocks")
a = ap.parse_args()
dev = torch.device("cuda", 0)
n, P = a.msgs, a.size
W = C.wire_size(0, 0, P)
payload = torch.randint(0, 256, (n * P,), dtype=torch.uint8, device=dev)
enc = C.CurveContext(0, a.sessions)
dec = C.CurveContext(0, a.sessions)
for s in range(a.sessions):
    enc.session_set(s, bytes((s + j) % 256 for j in range(32)), C.CLIENT_PREFIX, C.SERVER_PREFIX)
    dec.session_set(s, bytes((s + j) % 256 for j in range(32)), C.SERVER_PREFIX, C.CLIENT_PREFIX, False, 2)
t = lambda x, d: torch.from_numpy(np.ascontiguousarray(x).view(d)).to(dev)
sid = t(((np.arange(n) % a.sessions) if a.sid_mod else (np.arange(n) * a.sessions // n)).astype(np.uint32), np.int32)
flags = torch.zeros(n, dtype=torch.uint8, device=dev)
in_off = t(np.arange(n, dtype=np.uint64) * P, np.int64)
lens = t(np.full(n, P, np.uint32), np.int32)
WS = (W + a.wire_align - 1) // a.wire_align * a.wire_align  # wire stride
out_off = t(np.arange(n, dtype=np.uint64) * WS, np.int64)
wl = t(np.full(n, W, np.uint32), np.int32)
nonce = t(np.arange(3, 3 + n, dtype=np.uint64), np.int64)
wire = torch.zeros(n * WS, dtype=torch.uint8, device=dev)
back = torch.zeros(n * P, dtype=torch.uint8, device=dev)
fl = torch.zeros(n, dtype=torch.uint8, device=dev)
st = torch.zeros(n, dtype=torch.int32, device=dev)


def step():
    enc.encode_batch(sid, nonce, flags, in_off, lens, payload, out_off, wire)
    dec.decode_batch(sid, out_off, wl, wire, in_off, back, fl, st)
    nonce.add_(n)


for _ in range(3):
    step()
torch.cuda.synchronize()
enc.set_profiling(True)
dec.set_profiling(True)
t0 = time.perf_counter()
for _ in range(a.iters):
    step()
torch.cuda.synchronize()
t1 = time.perf_counter()
r = {"tag": a.tag, "wire_stride": WS, "msgs": n, "size": P, "step_us": (t1 - t0) / a.iters * 1e6}
for name, ctx, k in [("enc_body_us", enc, 0), ("dec_body_us", dec, 1), ("enc_call_us", enc, 2),
                     ("dec_call_us", dec, 3), ("enc_kbody_us", enc, 4), ("dec_kbody_us", dec, 5)]:
    ms, cnt = ctx.get_profile(k)
    if cnt or k < 4:
        r[name] = ms / max(cnt, 1) * 1e3
r["gib_s"] = 2 * n * P / 2**30 / (r["step_us"] * 1e-6)
r["ok"] = bool((st == 0).all().item()) and bool(torch.equal(back, payload))
print(json.dumps(r), flush=True)
