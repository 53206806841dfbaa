#!/usr/bin/env python3
"""Throughput of BASELINE configs 3 and 4 on one MI355X (not bench lines:
bench.py measures config 2).  Encode + decode round trips of device-resident
batches, payload GiB/s, with the per-call kernel breakdown from rocprof if run
under it.
  config 3: 49,152 frames, sizes drawn from {64, 1024, 65536}, 256 sessions
  config 4: 16 Mi x 256 B frames, 1024 sessions (one GPU's whole batch)"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from libzmq_amd import curve as C  # noqa: E402


def run(name, sizes, ns, reps=5):
    dev = torch.device("cuda", 0)
    n = len(sizes)
    rng = np.random.default_rng(7)
    enc, dec = C.CurveContext(0, ns), C.CurveContext(0, ns)
    for s in range(ns):
        k = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
        enc.session_set(s, k, C.CLIENT_PREFIX, C.SERVER_PREFIX)
        dec.session_set(s, k, C.SERVER_PREFIX, C.CLIENT_PREFIX, False, 2)
    t = lambda a, d: torch.from_numpy(np.ascontiguousarray(a).view(d)).to(dev)
    sizes = np.asarray(sizes, np.uint64)
    in_off = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64)
    W = sizes + 33
    out_off = np.concatenate([[0], np.cumsum(W)[:-1]]).astype(np.uint64)
    sid = (np.arange(n) % ns).astype(np.uint32)
    nonce = (3 + np.arange(n) // ns).astype(np.uint64)
    d_sid, d_in, d_out = t(sid, np.int32), t(in_off, np.int64), t(out_off, np.int64)
    d_len, d_wl = t(sizes.astype(np.uint32), np.int32), t(W.astype(np.uint32), np.int32)
    d_nonce = t(nonce, np.int64)
    flags = torch.zeros(n, dtype=torch.uint8, device=dev)
    total = int(sizes.sum())
    payload = torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev)
    wire = torch.zeros(int(W.sum()), dtype=torch.uint8, device=dev)
    back = torch.zeros(total, dtype=torch.uint8, device=dev)
    fl = torch.zeros(n, dtype=torch.uint8, device=dev)
    st = torch.zeros(n, dtype=torch.int32, device=dev)
    per = n // ns + 1

    def step():
        enc.encode_batch(d_sid, d_nonce, flags, d_in, d_len, payload, d_out, wire)
        dec.decode_batch(d_sid, d_out, d_wl, wire, d_in, back, fl, st)
        d_nonce.add_(per)

    step()
    torch.cuda.synchronize()
    assert int((st != 0).sum()) == 0 and torch.equal(back, payload)
    enc.set_profiling(True)
    dec.set_profiling(True)
    t0 = time.perf_counter()
    for _ in range(reps):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    assert int((st != 0).sum()) == 0 and torch.equal(back, payload)
    r = {"config": name, "frames": n, "sessions": ns, "payload_bytes": total, "step_us": dt * 1e6,
         "payload_GiB_s": total / dt / 2**30, "msgs_per_s": n / dt}
    for k, (ctx, kind) in {"enc_call_us": (enc, 2), "dec_call_us": (dec, 3), "enc_main_us": (enc, 0),
                           "dec_main_us": (dec, 1), "enc_body_us": (enc, 4), "dec_body_us": (dec, 5)}.items():
        ms, cnt = ctx.get_profile(kind)
        r[k] = ms / max(cnt, 1) * 1e3
    print(json.dumps(r), flush=True)


def main():
    which = sys.argv[1:] or ["3", "4"]
    if "3" in which:
        rng = np.random.default_rng(3)
        run("config3", rng.choice([64, 1024, 65536], 49152), 256)
    if "4" in which:
        run("config4", [256] * (16 << 20), 1024, reps=3)
    for w in which:
        if w.startswith("u"):  # uSIZE:N:SESSIONS, uniform sizes
            size, n, ns = (int(x) for x in w[1:].split(":"))
            run("uniform %d x %d B, %d sessions" % (n, size, ns), [size] * n, ns, reps=3)


if __name__ == "__main__":
    main()
