#!/usr/bin/env python3
"""Device ZMTP framing cost at the config-2 shape (65,536 x 1 KiB, one
connection): zmqg_encode_batch vs zmqg_encode_zmtp (frames laid out with
headers in one send buffer), and zmqg_decode_batch on known descriptors vs
zmqg_decode_zmtp parsing the received byte stream itself (synchronous)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from libzmq_amd import curve as C  # noqa: E402


def main():
    n, P = 65536, 1024
    W = C.wire_size(0, 0, P)
    F = W + 9
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(1)
    pay = torch.randint(0, 256, (n * P,), dtype=torch.uint8, device=dev, generator=g)
    precom = bytes(range(32))
    i64 = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)
    i32 = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).to(dev)
    sid = i32(np.zeros(n, np.uint32))
    flags = torch.zeros(n, dtype=torch.uint8, device=dev)
    in_off = i64(np.arange(n, dtype=np.uint64) * P)
    lens = i32(np.full(n, P, np.uint32))
    wire_off = i64(np.arange(n, dtype=np.uint64) * W)
    wlen = i32(np.full(n, W, np.uint32))
    wire = torch.zeros(n * W, dtype=torch.uint8, device=dev)
    framed = torch.zeros(n * F, dtype=torch.uint8, device=dev)
    foff = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    back = torch.zeros(n * P, dtype=torch.uint8, device=dev)
    fl = torch.zeros(n, dtype=torch.uint8, device=dev)
    st = torch.zeros(n, dtype=torch.int32, device=dev)
    d_foff = torch.zeros(n, dtype=torch.int64, device=dev)
    d_flen = torch.zeros(n, dtype=torch.int32, device=dev)
    d_poff = torch.zeros(n, dtype=torch.int64, device=dev)
    enc = C.CurveContext(0, 1)
    enc.session_set(0, precom, C.CLIENT_PREFIX, C.SERVER_PREFIX)
    nonce0 = [3]

    def nonces():
        t = i64(np.arange(nonce0[0], nonce0[0] + n, dtype=np.uint64))
        nonce0[0] += n
        return t

    def timed(fn, reps=10):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps * 1e6

    nn = [nonces() for _ in range(12)]
    k = [0]

    def e_batch():
        enc.encode_batch(sid, nn[k[0] % 12], flags, in_off, lens, pay, wire_off, wire)
        k[0] += 1

    def e_zmtp():
        enc.encode_zmtp(sid, nn[k[0] % 12], flags, in_off, lens, pay, framed, foff)
        k[0] += 1

    te, tz = timed(e_batch), timed(e_zmtp)
    total = int(foff[n].item())
    print(f"encode_batch {te:8.1f} us   encode_zmtp {tz:8.1f} us  ({total} framed bytes)")

    # decode: the peer nonce is reset before each call (the same stream again)
    d = C.CurveContext(0, 1)
    d.session_set(0, precom, C.SERVER_PREFIX, C.CLIENT_PREFIX, False, 2)

    def d_batch():
        d.set_peer_nonce(0, 2)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        d.decode_batch(sid, wire_off, wlen, wire, in_off, back, fl, st)
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    def d_zmtp(maxmsg=-1):
        d.set_peer_nonce(0, 2)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = d.decode_zmtp(0, framed, total, maxmsg, n, d_foff, d_flen, d_poff, zback, fl, st)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        assert r["frames"] == n and r["consumed"] == total and r["error"] == 0
        return dt

    e_batch()  # wire holds a fresh encode
    torch.cuda.synchronize()
    d_batch()
    tb = min(d_batch() for _ in range(5)) * 1e6
    assert int((st != 0).sum()) == 0 and torch.equal(back, pay)
    zback = torch.zeros(total, dtype=torch.uint8, device=dev)  # payloads at their bodies' offsets
    d_zmtp()
    tzd = min(d_zmtp() for _ in range(5)) * 1e6
    idx = d_poff[:, None] + torch.arange(P, device=dev)[None, :]
    assert int((st != 0).sum()) == 0 and torch.equal(zback[idx].reshape(-1), pay)
    print(f"decode_batch {tb:8.1f} us   decode_zmtp {tzd:8.1f} us  (parse + decode, synchronous)")
    # the engine's ZMQ_MAXMSGSIZE (options.maxmsgsize, checked by the v2
    # decoder against each frame's size, src/v2_decoder.cpp:74-84) at the
    # frames' own size: every frame is known to fit the frame kernel, so the
    # large-frame launches are skipped
    zback.zero_()
    d_zmtp(W)
    tzm = min(d_zmtp(W) for _ in range(5)) * 1e6
    assert int((st != 0).sum()) == 0 and torch.equal(zback[idx].reshape(-1), pay)
    print(f"decode_zmtp_maxmsgsize {tzm:8.1f} us  (max_msg_size = {W})")

    # the same call through the C ABI alone: arguments built once, the
    # library's own stream synchronisation the only wait (the Python
    # wrapper's argument conversion and the extra device synchronisation
    # above are not part of the call)
    lib = C._lib
    r = C.ZmtpResult()
    args = (d._ctx, 0, C._ptr(framed), total, W, n, C._ptr(d_foff), C._ptr(d_flen), C._ptr(d_poff), C._ptr(zback),
            C._ptr(fl), C._ptr(st), C.ctypes.byref(r), C._stream_handle(None))

    def d_abi():
        d.set_peer_nonce(0, 2)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        rc = lib.zmqg_decode_zmtp(*args)
        dt = time.perf_counter() - t0
        assert rc == 0 and r.frames == n and r.consumed == total and r.error == 0
        return dt

    d_abi()
    ta = sorted(d_abi() for _ in range(20))
    assert int((st != 0).sum()) == 0
    print(f"decode_zmtp_abi {ta[0] * 1e6:8.1f} us min, {ta[10] * 1e6:8.1f} us median  (C call, max_msg_size = {W})")


if __name__ == "__main__":
    main()
