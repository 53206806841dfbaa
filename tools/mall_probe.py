#!/usr/bin/env python3
"""Where config 2's frame kernels read from: bench.py's launch pass (K
encodes of the batch into K wire buffers back to back, then their K decodes)
for K = 1 ... 20, so the wire bytes written since a decode's buffer was
written grow from one buffer (69 MB) to twenty (1.4 GB).  If the decode's
time steps up once those bytes pass the 256 MB MALL, the warm/cold gap of
DESIGN.md section 4 is the MALL's.  Each K also runs the decodes in reverse
order (the most recently written buffer first, each buffer with its own
decoder so every frame decodes).  Every measurement follows 40 queued
encodes with no host gap (the clock ramp).

  mall_probe.py [--ks 1,2,3,4,6,8,12,20]"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from libzmq_amd import curve as C  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--ks", default="1,2,3,4,6,8,12,20")
a = ap.parse_args()
dev = torch.device("cuda", 0)
n, P = 65536, 1024
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
back = torch.zeros(n * P, dtype=torch.uint8, device=dev)
fl = torch.zeros(n, dtype=torch.uint8, device=dev)
enc = C.CurveContext(0, 1)
enc.session_set(0, key, C.CLIENT_PREFIX, C.SERVER_PREFIX)
enc.set_nonce(0, 3)
s = torch.cuda.current_stream(dev)
wires = [torch.empty(n * W, dtype=torch.uint8, device=dev) for _ in range(20)]
sts = [torch.zeros(n, dtype=torch.int32, device=dev) for _ in range(20)]


def ev():
    return torch.cuda.Event(enable_timing=True)


scratch = torch.empty(n * W, dtype=torch.uint8, device=dev)
decs = []
for k in range(20):
    d = C.CurveContext(0, 1)
    d.session_set(0, key, C.SERVER_PREFIX, C.CLIENT_PREFIX, False, 2)
    decs.append(d)
SETTLE = 40  # encodes (~2.2 ms) queued right before every measurement, no host gap between
# first touch of every buffer and decoder
for k in range(20):
    enc.encode_batch(sid, None, flags, in_off, lens, payload, out_off, wires[k], s, max_len=P, nonce_auto=True)
    decs[k].set_peer_nonce(0, enc.get_nonce(0) - n - 1)
    decs[k].decode_batch(sid, out_off, wl, wires[k], in_off, back, fl, sts[k], s, max_len=W)
torch.cuda.synchronize()
out = []
for K in [int(x) for x in a.ks.split(",")]:
    for order in ("fifo", "lifo"):
        base = enc.get_nonce(0) + SETTLE * n
        # each buffer's decoder: peer nonce just below the buffer's first
        # nonce, so either order decodes every frame successfully
        for k in range(K):
            decs[k].set_peer_nonce(0, base + k * n - 1)
        torch.cuda.synchronize()
        a0, a1, b0, b1 = ev(), ev(), ev(), ev()
        for _ in range(SETTLE):
            enc.encode_batch(sid, None, flags, in_off, lens, payload, out_off, scratch, s, max_len=P,
                             nonce_auto=True)
        a0.record(s)
        for k in range(K):
            enc.encode_batch(sid, None, flags, in_off, lens, payload, out_off, wires[k], s, max_len=P, nonce_auto=True)
        a1.record(s)
        b0.record(s)
        for k in (range(K) if order == "fifo" else range(K - 1, -1, -1)):
            decs[k].decode_batch(sid, out_off, wl, wires[k], in_off, back, fl, sts[k], s, max_len=W)
        b1.record(s)
        torch.cuda.synchronize()
        ok = all(int((sts[k] != 0).sum()) == 0 for k in range(K)) and bool(torch.equal(back, payload))
        out.append({"K": K, "order": order, "encode_us": a0.elapsed_time(a1) * 1e3 / K,
                    "decode_us": b0.elapsed_time(b1) * 1e3 / K, "wire_mb_per_buffer": n * W / 1e6, "ok": ok})
        print(json.dumps(out[-1]), flush=True)
# the bench step's order (encode k, then decode k), 20 steps back to back,
# with one wire buffer or twenty, one decoder or twenty
for nw_, nd_ in ((1, 1), (20, 1), (1, 20), (20, 20), (1, 1)):
    base = enc.get_nonce(0) + SETTLE * n
    for k in range(20):
        decs[k].set_peer_nonce(0, base - 1 + (k - k % nd_) * n if nd_ > 1 else base - 1)
    torch.cuda.synchronize()
    for _ in range(SETTLE):
        enc.encode_batch(sid, None, flags, in_off, lens, payload, out_off, scratch, s, max_len=P, nonce_auto=True)
    a0, a1 = ev(), ev()
    a0.record(s)
    for k in range(20):
        w = wires[k % nw_]
        enc.encode_batch(sid, None, flags, in_off, lens, payload, out_off, w, s, max_len=P, nonce_auto=True)
        decs[k % nd_].decode_batch(sid, out_off, wl, w, in_off, back, fl, sts[k], s, max_len=W)
    a1.record(s)
    torch.cuda.synchronize()
    ok = all(int((sts[k] != 0).sum()) == 0 for k in range(20))
    print(json.dumps({"order": "step", "wire_buffers": nw_, "decoders": nd_, "step_us": a0.elapsed_time(a1) * 1e3 / 20,
                      "ok": ok}), flush=True)
