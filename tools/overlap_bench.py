#!/usr/bin/env python3
"""Config-2 round trips, two schedules, GPU-side time only (experiment for
bench.py):
  serial     encode_k -> decode_k -> encode_k+1 ... on one stream
  pipelined  encodes on one stream, decodes on another; decode_k waits for
             encode_k only, so decode_k runs alongside encode_k+1 (two wire
             buffers, encode_k+2 waits for decode_k to have read wire k % 2)
torch's graph capture of forked streams crashes on this image (tools/
mscap_probe.py), so the K steps are launched eagerly behind a spin kernel
that holds the stream until every launch is queued; the time is the span
between events after the spin and after the last step.
Prints one JSON line per schedule and round: us per step, GiB/s."""
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
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--spin", type=int, default=40_000_000, help="cycles the stream is held while the steps are queued")
a = ap.parse_args()
dev = torch.device("cuda", 0)
n, P, K = a.msgs, a.size, a.steps
W = C.wire_size(0, 0, P)
payload = torch.randint(0, 256, (n * P,), dtype=torch.uint8, device=dev)
precom = bytes(range(32))
i64 = lambda x: torch.from_numpy(np.ascontiguousarray(x).view(np.int64)).to(dev)
i32 = lambda x: torch.from_numpy(np.ascontiguousarray(x).view(np.int32)).to(dev)
sid = i32(np.zeros(n, np.uint32))
flags = torch.zeros(n, dtype=torch.uint8, device=dev)
in_off = i64(np.arange(n, dtype=np.uint64) * P)
lens = i32(np.full(n, P, np.uint32))
out_off = i64(np.arange(n, dtype=np.uint64) * W)
wlen = i32(np.full(n, W, np.uint32))
wires = [torch.zeros(n * W, dtype=torch.uint8, device=dev) for _ in range(2)]
back = torch.zeros(n * P, dtype=torch.uint8, device=dev)
fl_out = torch.zeros(n, dtype=torch.uint8, device=dev)
st_out = torch.zeros(n, dtype=torch.int32, device=dev)
enc = C.CurveContext(0, 1)
enc.session_set(0, precom, C.CLIENT_PREFIX, C.SERVER_PREFIX)
enc.set_nonce(0, 3)
dec = C.CurveContext(0, 1)
dec.session_set(0, precom, C.SERVER_PREFIX, C.CLIENT_PREFIX, False, 2)
cur = torch.cuda.current_stream(dev)
se, sd = torch.cuda.Stream(dev), torch.cuda.Stream(dev)


def encode(st, w):
    enc.encode_batch(sid, None, flags, in_off, lens, payload, out_off, w, st, max_len=P, nonce_auto=True)


def decode(st, w):
    dec.decode_batch(sid, out_off, wlen, w, in_off, back, fl_out, st_out, st, max_len=W)


def serial():
    for k in range(K):
        encode(cur, wires[0])
        decode(cur, wires[0])


def pipelined():
    se.wait_stream(cur)
    sd.wait_stream(cur)
    done = []
    for k in range(K):
        if k >= 2:
            se.wait_event(done[k - 2])
        encode(se, wires[k % 2])
        e = torch.cuda.Event()
        e.record(se)
        sd.wait_event(e)
        decode(sd, wires[k % 2])
        d = torch.cuda.Event()
        d.record(sd)
        done.append(d)
    cur.wait_stream(se)
    cur.wait_stream(sd)


for f in (serial, pipelined):  # warmup
    f()
torch.cuda.synchronize(dev)
for r in range(a.rounds):
    for f in (serial, pipelined):
        back.zero_()
        st_out.fill_(-1)
        torch.cuda._sleep(a.spin)
        g0, g1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        g0.record(cur)
        f()
        g1.record(cur)
        torch.cuda.synchronize(dev)
        ms = g0.elapsed_time(g1)
        ok = bool(int((st_out != 0).sum()) == 0 and torch.equal(back, payload))
        print(json.dumps({"schedule": f.__name__, "round": r, "steps": K, "us_per_step": 1e3 * ms / K,
                          "gib_s": K * n * P / 2**30 / (ms / 1e3), "ok": ok}), flush=True)
