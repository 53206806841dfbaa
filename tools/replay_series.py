#!/usr/bin/env python3
"""Step time of bench.py's timed replay, replay after replay: config 2
(65,536 x 1 KiB, one session) captured as one hipGraph of K steps (encode
with device-assigned nonces, then decode of that wire) as bench.py does,
replayed R times, each replay timed with events on the stream.  The series
shows the device's clock ramp under sustained load (DESIGN.md section 4:
~129 us per step on the first replay, ~105 us from about 20 ms of load on),
the reason bench.py replays the graph untimed before its timed replay.
Checks every decode's status and the round trip after the replays.

  replay_series.py [--msgs N] [--size P] [--steps K] [--reps R]"""
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
ap.add_argument("--reps", type=int, default=40)
a = ap.parse_args()
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
wire = torch.zeros(n * W, dtype=torch.uint8, device=dev)
back = torch.zeros(n * P, dtype=torch.uint8, device=dev)
fl = torch.zeros(n, dtype=torch.uint8, device=dev)
st = torch.zeros(n, dtype=torch.int32, device=dev)
enc = C.CurveContext(0, 1)
enc.session_set(0, key, C.CLIENT_PREFIX, C.SERVER_PREFIX)
enc.set_nonce(0, 3)
dec = C.CurveContext(0, 1)
dec.session_set(0, key, C.SERVER_PREFIX, C.CLIENT_PREFIX, False, 2)


def step(cs):
    enc.encode_batch(sid, None, flags, in_off, lens, payload, out_off, wire, cs, max_len=P, nonce_auto=True)
    dec.decode_batch(sid, out_off, wl, wire, in_off, back, fl, st, cs, max_len=W)


s = torch.cuda.current_stream(dev)
for _ in range(4):
    step(s)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
cap = torch.cuda.Stream(dev)
cap.wait_stream(s)
with torch.cuda.graph(g, stream=cap):
    cs = torch.cuda.current_stream(dev)
    for _ in range(a.steps):
        step(cs)
torch.cuda.synchronize()
us = []
for _ in range(a.reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    g.replay()
    e1.record(s)
    torch.cuda.synchronize()
    us.append(e0.elapsed_time(e1) * 1e3 / a.steps)
# the same K steps launched eagerly from the host, back to back, right after
# the settled replays (events around the whole sequence), then one more replay
eager = []
for _ in range(3):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    g.replay()
    e0.record(s)
    for _ in range(a.steps):
        step(s)
    e1.record(s)
    torch.cuda.synchronize()
    eager.append(round(e0.elapsed_time(e1) * 1e3 / a.steps, 1))
ok = bool((st == 0).all().item()) and bool(torch.equal(back, payload))
tail = sorted(us[len(us) // 2:])
print(json.dumps({"msgs": n, "size": P, "steps_per_replay": a.steps, "reps_us": [round(u, 1) for u in us],
                  "first_us": us[0], "settled_median_us": tail[len(tail) // 2],
                  "settled_gib_s": n * P / 2**30 / (tail[len(tail) // 2] * 1e-6),
                  "eager_after_replay_us": eager, "ok": ok}), flush=True)
