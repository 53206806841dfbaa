#!/usr/bin/env python3
"""Config 2's HBM-fed decode (bench.py hbm_fed): K
batches with their own buffers, K encodes back to back, then K decodes, each
span timed by one event pair.  Forms:
  bench   the bench's order (the decodes run while the encodes' dirty wire
          lines are still being written back from the Infinity Cache);
  clean   a 1 GiB read sweep between the encodes and the decodes (the cache
          then holds clean lines: what the decodes pay for HBM reads alone);
  warm    each decode right after its own encode (the MALL-resident step).
Each form for the decode frame kernels in turn (ZMQG_FRAMES_G: 0 =
k_frames_seq, 8 = k_frames_lds), every decode checked.

With --time-enc the bench form's K encodes are timed too (--enc-stream-out:
ZMQG_OPT_STREAM_OUT on them).

  hbm_probe.py [--sets 8] [--reps 3]"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

ap = argparse.ArgumentParser()
ap.add_argument("--sets", type=int, default=8)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--variants", default="0,8")
ap.add_argument("--forms", default="bench,clean,warm")
ap.add_argument("--stream-out", action="store_true", help="decode with ZMQG_OPT_STREAM_OUT (cache hint)")
ap.add_argument("--enc-stream-out", action="store_true", help="encode with ZMQG_OPT_STREAM_OUT")
ap.add_argument("--time-enc", action="store_true", help="also time the encodes of the bench form")
ap.add_argument("--no-check", action="store_true", help="(ablated timing builds: outputs are not the codec's)")
ap.add_argument("--side-prefetch", action="store_true",
                help="experiment: a reduction over each wire on a second stream, concurrent with its decode")
ap.add_argument("--stream-prefetch", type=int, default=0,
                help="experiment: tools/bin/libprefetch_probe.so's address-order read of each wire, this many "
                     "workgroups, on a second stream beside its decode")
a = ap.parse_args()

dev = torch.device("cuda", 0)
n, P = 65536, 1024
K = a.sets


def make(variant):
    os.environ["ZMQG_FRAMES_G"] = str(variant)  # (read at zmqg_ctx_create)
    from libzmq_amd import curve as C
    precom = bytes(range(32))
    enc = C.CurveContext(0, 1)
    enc.session_set(0, precom, C.CLIENT_PREFIX, C.SERVER_PREFIX)
    enc.set_nonce(0, 3)
    dec = C.CurveContext(0, 1)
    dec.session_set(0, precom, C.SERVER_PREFIX, C.CLIENT_PREFIX, False, 2)
    del os.environ["ZMQG_FRAMES_G"]
    return C, enc, dec


def main():
    from libzmq_amd import curve as C
    W = C.wire_size(0, 0, P)
    i64 = lambda x: torch.from_numpy(np.ascontiguousarray(x).view(np.int64)).to(dev)
    i32 = lambda x: torch.from_numpy(np.ascontiguousarray(x).view(np.int32)).to(dev)
    sid = i32(np.zeros(n, np.uint32))
    flags = torch.zeros(n, dtype=torch.uint8, device=dev)
    in_off = i64(np.arange(n, dtype=np.uint64) * P)
    lens = i32(np.full(n, P, np.uint32))
    out_off = i64(np.arange(n, dtype=np.uint64) * W)
    wlen = i32(np.full(n, W, np.uint32))
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    pays = [torch.randint(0, 256, (n * P,), dtype=torch.uint8, device=dev, generator=g) for _ in range(K)]
    wires = [torch.empty(n * W, dtype=torch.uint8, device=dev) for _ in range(K)]
    backs = [torch.empty(n * P, dtype=torch.uint8, device=dev) for _ in range(K)]
    fls = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(K)]
    sts = [torch.empty(n, dtype=torch.int32, device=dev) for _ in range(K)]
    sweep = torch.ones(1 << 28, dtype=torch.int32, device=dev)  # 1 GiB
    stream = torch.cuda.current_stream(dev)
    side = torch.cuda.Stream(dev)
    sinks = []
    sink = torch.zeros(65536, dtype=torch.int32, device=dev)
    pf = None
    if a.stream_prefetch:
        import ctypes
        pf = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "bin", "libprefetch_probe.so"))
    for v in [int(x) for x in a.variants.split(",")]:
        _, enc, dec = make(v)

        def encs():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for k in range(K):
                enc.encode_batch(sid, None, flags, in_off, lens, pays[k], out_off, wires[k], stream, max_len=P,
                                 nonce_auto=True, stream_out=a.enc_stream_out)
            e1.record(stream)
            return e0, e1

        def decs():
            for k in range(K):
                sts[k].fill_(-1)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for k in range(K):
                if a.stream_prefetch:
                    f = torch.cuda.Event()
                    f.record(stream)
                    side.wait_event(f)
                    pf.prefetch_launch(C.ctypes.c_void_p(wires[k].data_ptr()), C.ctypes.c_uint64(n * W),
                                       a.stream_prefetch, C.ctypes.c_void_p(sink.data_ptr()),
                                       C.ctypes.c_void_p(side.cuda_stream))
                if a.side_prefetch:
                    f = torch.cuda.Event()
                    f.record(stream)
                    side.wait_event(f)
                    with torch.cuda.stream(side):
                        sinks.append(wires[k][: n * W // 8 * 8].view(torch.int64).max())
                dec.decode_batch(sid, out_off, wlen, wires[k], in_off, backs[k], fls[k], sts[k], stream, max_len=W,
                                 stream_out=a.stream_out)
            e1.record(stream)
            return e0, e1

        def check():
            if a.no_check:
                return
            for k in range(K):
                assert int((sts[k] != 0).sum()) == 0 and torch.equal(backs[k], pays[k])

        forms = a.forms.split(",")
        res = {f: [] for f in forms}
        if a.time_enc:
            res["encode"] = []
        for r in range(a.reps + 1):
            if "bench" in forms:
                c0, c1 = encs()
                e0, e1 = decs()
                torch.cuda.synchronize()
                check()
                if r:
                    res["bench"].append(e0.elapsed_time(e1) * 1e3 / K)
                    if a.time_enc:
                        res["encode"].append(c0.elapsed_time(c1) * 1e3 / K)
            if "clean" in forms:
                encs()
                s = sweep.sum()  # clean lines in the cache
                e0, e1 = decs()
                torch.cuda.synchronize()
                check()
                del s
                if r:
                    res["clean"].append(e0.elapsed_time(e1) * 1e3 / K)
            if "warm" in forms:
                # encode k then decode k, the decode alone timed
                t = 0.0
                for k in range(K):
                    sts[k].fill_(-1)
                    enc.encode_batch(sid, None, flags, in_off, lens, pays[k], out_off, wires[k], stream, max_len=P,
                                     nonce_auto=True, stream_out=a.enc_stream_out)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                    dec.decode_batch(sid, out_off, wlen, wires[k], in_off, backs[k], fls[k], sts[k], stream,
                                     max_len=W)
                    e1.record(stream)
                    torch.cuda.synchronize()
                    t += e0.elapsed_time(e1) * 1e3
                check()
                if r:
                    res["warm"].append(t / K)
        print(f"variant G={v}: " + "  ".join(f"{k} {min(x):6.1f}/{sorted(x)[len(x) // 2]:6.1f} us"
                                             for k, x in res.items()) + "  (decode per launch, min/median)")
        enc.close()
        dec.close()
    import json
    sid_, commit = C.build_id()
    print(json.dumps({"build": {"source_id": sid_, "commit": commit}}))


if __name__ == "__main__":
    main()
