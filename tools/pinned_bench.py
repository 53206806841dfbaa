#!/usr/bin/env python3
"""Host-to-host CURVE encode / decode rates on one MI355X (config 2 shape):
  device    inputs and outputs resident in HBM (reference)
  zerocopy  payload / wire in pinned host memory, the kernels read and write
            it over PCIe directly (descriptors in HBM)
  pipelined pinned host buffers, chunks copied H2D, processed and copied D2H
            on two streams so the copies overlap the kernels
Each figure is payload GiB/s of one direction (encode: payload -> wire;
decode: wire -> payload), averaged over several batches."""
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
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(1)
    pay_h = torch.randint(0, 256, (n * P,), dtype=torch.uint8, generator=g).pin_memory()
    back_h = torch.zeros(n * P, dtype=torch.uint8).pin_memory()
    pay_d, back_d = pay_h.to(dev), torch.zeros(n * P, dtype=torch.uint8, device=dev)
    precom = bytes(range(32))
    enc = C.CurveContext(0, 1)
    enc.session_set(0, precom, C.CLIENT_PREFIX, C.SERVER_PREFIX)
    dec = C.CurveContext(0, 1)
    dec.session_set(0, precom, C.SERVER_PREFIX, C.CLIENT_PREFIX, False, 2)
    i64 = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)
    i32 = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).to(dev)
    sid = i32(np.zeros(n, np.uint32))
    flags = torch.zeros(n, dtype=torch.uint8, device=dev)
    in_off = i64(np.arange(n, dtype=np.uint64) * P)
    out_off = i64(np.arange(n, dtype=np.uint64) * W)
    lens = i32(np.full(n, P, np.uint32))
    wlen = i32(np.full(n, W, np.uint32))
    fl = torch.zeros(n, dtype=torch.uint8, device=dev)
    st = torch.zeros(n, dtype=torch.int32, device=dev)
    nonce0 = [3]
    s0 = torch.cuda.current_stream(dev)

    def nonces():
        t = i64(np.arange(nonce0[0], nonce0[0] + n, dtype=np.uint64))
        nonce0[0] += n
        return t

    # decode needs fresh nonces every batch (a repeated frame is a replay):
    # R wire batches encoded in nonce order, decoded in the same order
    R = 9
    wires_d = [torch.zeros(n * W, dtype=torch.uint8, device=dev) for _ in range(R)]
    wires_h = [torch.zeros(n * W, dtype=torch.uint8).pin_memory() for _ in range(R)]

    def timed_seq(fn, reps=R):
        torch.cuda.synchronize()
        fn(0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for r in range(1, reps):
            fn(r)
        torch.cuda.synchronize()
        return (reps - 1) * n * P / 2**30 / (time.perf_counter() - t0)

    res = {}
    # device-resident
    res["device encode"] = timed_seq(
        lambda r: enc.encode_batch(sid, nonces(), flags, in_off, lens, pay_d, out_off, wires_d[r]))
    res["device decode"] = timed_seq(lambda r: dec.decode_batch(sid, out_off, wlen, wires_d[r], in_off, back_d, fl, st))
    torch.cuda.synchronize()
    assert int((st != 0).sum()) == 0 and torch.equal(back_d, pay_d), "device round trip"
    # zero-copy: kernels read/write pinned host memory
    res["zerocopy encode"] = timed_seq(
        lambda r: enc.encode_batch(sid, nonces(), flags, in_off, lens, pay_h, out_off, wires_h[r]))
    res["zerocopy decode"] = timed_seq(lambda r: dec.decode_batch(sid, out_off, wlen, wires_h[r], in_off, back_h, fl, st))
    torch.cuda.synchronize()
    assert int((st != 0).sum()) == 0 and torch.equal(back_h, pay_h), "zero-copy round trip"
    # pipelined chunks: the ctx's kernels on one compute stream (a ctx is
    # stream-ordered), copies on an H2D and a D2H stream, double buffers
    K = 8
    m = n // K
    s_in, s_c, s_out = torch.cuda.Stream(dev), torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    cin_off = i64(np.arange(m, dtype=np.uint64) * P)
    cout_off = i64(np.arange(m, dtype=np.uint64) * W)
    csid, cfl, clen, cwl = sid[:m], flags[:m], lens[:m], wlen[:m]
    cst = torch.zeros(K, m, dtype=torch.int32, device=dev)
    cflo = torch.zeros(m, dtype=torch.uint8, device=dev)
    pbuf = [torch.empty(m * P, dtype=torch.uint8, device=dev) for _ in range(2)]
    wbuf = [torch.empty(m * W, dtype=torch.uint8, device=dev) for _ in range(2)]

    def pipeline(src_h, src_buf, src_chunk, dst_h, dst_buf, dst_chunk, kernel):
        loaded = [torch.cuda.Event() for _ in range(K)]
        done = [torch.cuda.Event() for _ in range(K)]
        drained = [torch.cuda.Event() for _ in range(K)]
        # the previous call's last kernels / copies still own the buffers
        s_in.wait_stream(s_c)
        s_c.wait_stream(s_out)
        s_c.wait_stream(s0)
        for k in range(K):
            b = k & 1
            with torch.cuda.stream(s_in):
                if k >= 2:
                    s_in.wait_event(done[k - 2])  # the kernel of chunk k-2 has read buffer b
                src_buf[b].copy_(src_h[k * m * src_chunk:(k + 1) * m * src_chunk], non_blocking=True)
                loaded[k].record(s_in)
            with torch.cuda.stream(s_c):
                s_c.wait_event(loaded[k])
                if k >= 2:
                    s_c.wait_event(drained[k - 2])  # chunk k-2's output left buffer b
                kernel(k, src_buf[b], dst_buf[b], s_c)
                done[k].record(s_c)
            with torch.cuda.stream(s_out):
                s_out.wait_event(done[k])
                dst_h[k * m * dst_chunk:(k + 1) * m * dst_chunk].copy_(dst_buf[b], non_blocking=True)
                drained[k].record(s_out)

    keep = []

    def pipe_encode_to(r):
        base = nonce0[0]
        nonce0[0] += n
        nn = [i64(np.arange(base + k * m, base + (k + 1) * m, dtype=np.uint64)) for k in range(K)]
        keep.append(nn)  # allocated on s0, read on s_c: keep alive past this call
        pipeline(pay_h, pbuf, P, wires_h[r], wbuf, W,
                 lambda k, src, dst, s: enc.encode_batch(csid, nn[k], cfl, cin_off, clen, src, cout_off, dst, s))

    def pipe_decode_from(r):
        pipeline(wires_h[r], wbuf, W, back_h, pbuf, P,
                 lambda k, src, dst, s: dec.decode_batch(csid, cout_off, cwl, src, cin_off, dst, cflo, cst[k], s))

    fails = 0
    for trial in range(4):
        back_h.zero_()
        cst.fill_(-1)
        torch.cuda.synchronize()
        res["pipelined encode"] = timed_seq(pipe_encode_to)
        res["pipelined decode"] = timed_seq(pipe_decode_from)
        torch.cuda.synchronize()
        bad = [(k, int((cst[k] != 0).sum()), sorted(set(cst[k].tolist()))[:4],
                int((back_h[k * m * P:(k + 1) * m * P] != pay_h[k * m * P:(k + 1) * m * P]).sum())) for k in range(K)]
        if any(b[1] or b[3] for b in bad):
            fails += 1
            print(f"trial {trial}: pipelined mismatch per chunk (k, bad status, codes, bad bytes):", bad, flush=True)
            # the same wire decoded chunk by chunk on one stream, device-resident
            ref_w = wires_h[R - 1].to(dev)
            dec2 = C.CurveContext(0, 1)
            dec2.session_set(0, precom, C.SERVER_PREFIX, C.CLIENT_PREFIX, False, 2)
            for k in range(K):
                dec2.decode_batch(csid, cout_off, cwl, ref_w[k * m * W:(k + 1) * m * W], cin_off,
                                  back_d[k * m * P:(k + 1) * m * P], cflo, cst[k])
            torch.cuda.synchronize()
            print("  sequential chunked decode of that wire: bad status", int((cst != 0).sum()),
                  "bad bytes", int((back_d != pay_d).sum()), flush=True)
    for k, v in res.items():
        print(f"{k:18s} {v:8.1f} GiB/s payload")
    assert fails == 0, "pipelined round trip"

if __name__ == "__main__":
    main()
