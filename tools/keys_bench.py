#!/usr/bin/env python3
"""Batched handshake key derivation rate on one MI355X: crypto_box_beforenm
(X25519 + HSalsa20) and crypto_scalarmult_base for N random keys, keys/s;
handshake boxes (zmqg_box_afternm_batch / _open_) of HELLO (64 B) and
INITIATE-like (256 B) plaintexts, boxes/s;
and the CPU reference for scale (libsodium via the oracle's dlopen is not
exposed, so the oracle's portable C X25519 on one core)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from libzmq_amd import curve as C  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    rng = np.random.default_rng(1)
    pk = torch.from_numpy(rng.integers(0, 256, 32 * n, dtype=np.uint8)).cuda()
    sk = torch.from_numpy(rng.integers(0, 256, 32 * n, dtype=np.uint8)).cuda()
    k = torch.zeros(32 * n, dtype=torch.uint8, device="cuda")
    st = torch.zeros(n, dtype=torch.int32, device="cuda")
    ctx = C.CurveContext(0, 1)
    for name, fn in (("beforenm", lambda: ctx.box_beforenm_batch(pk, sk, k, st)),
                     ("scalarmult_base", lambda: ctx.scalarmult_batch(sk, None, k, st))):
        fn()
        torch.cuda.synchronize()
        reps = 3
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / reps
        print(f"{name:16s} {n} keys  {dt * 1e3:8.2f} ms  {n / dt / 1e6:6.3f} M keys/s")
    key = torch.from_numpy(rng.integers(0, 256, 32 * n, dtype=np.uint8)).cuda()
    nonce = torch.from_numpy(rng.integers(0, 256, 24 * n, dtype=np.uint8)).cuda()
    for L in (64, 256):
        i = torch.arange(n, device="cuda", dtype=torch.int64)
        m = torch.from_numpy(rng.integers(0, 256, L * n, dtype=np.uint8)).cuda()
        box = torch.zeros((L + 16) * n, dtype=torch.uint8, device="cuda")
        back = torch.zeros(L * n, dtype=torch.uint8, device="cuda")
        ln = torch.full((n,), L, dtype=torch.int32, device="cuda")
        lb = torch.full((n,), L + 16, dtype=torch.int32, device="cuda")
        for name, fn in (("box seal %d B" % L,
                          lambda: ctx.box_afternm_batch(key, nonce, i * L, ln, m, i * (L + 16), box)),
                         ("box open %d B" % L,
                          lambda: ctx.box_open_afternm_batch(key, nonce, i * (L + 16), lb, box, i * L, back, st))):
            fn()
            torch.cuda.synchronize()
            reps = 5
            t0 = time.perf_counter()
            for _ in range(reps):
                fn()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / reps
            print(f"{name:16s} {n} boxes {dt * 1e3:8.3f} ms  {n / dt / 1e6:6.2f} M boxes/s")
        assert bool((st == 0).all()) and torch.equal(back, m)
    from oracle import oracle as O
    m = 200
    t0 = time.perf_counter()
    for i in range(m):
        O.box_beforenm(bytes(pk[32 * i:32 * i + 32].cpu().numpy()), bytes(sk[32 * i:32 * i + 32].cpu().numpy()))
    dt = time.perf_counter() - t0
    print(f"oracle beforenm (portable C, 1 core): {m / dt / 1e3:.1f} k keys/s")


if __name__ == "__main__":
    main()
