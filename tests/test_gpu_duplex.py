"""zmqg_duplex_batch (include/zmqg_curve.h): the decode of batch k and the
encode of batch k+1 of another ctx in one launch (k_frames_duplex), as the
I/O thread pipelines them.  Each round's encoded wire is bit-exact against
the oracle's encode (src/curve_mechanism_base.cpp:111-168) with the nonces
the device assigns (continuing across rounds), and each decode -- a replay
and a tampered frame spliced in -- equals the oracle's sequential decode
(:170-260), peer nonce included.  Sizes on both sides of the one-launch
range (one lane per frame: 2/3 ... 1 wave slots) and pairs outside it, which
the call runs as the two separate batch calls."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _batch(rng, n, sizes):
    lens = rng.choice(sizes, n).astype(np.uint32)
    flags = rng.choice([0, 1, 2, 3], n).astype(np.uint8)
    in_off = np.zeros(n, np.uint64)
    in_off[1:] = np.cumsum(lens.astype(np.uint64))[:-1]
    inp = rng.integers(0, 256, int(lens.sum()) + 1, dtype=np.uint8)
    wl = np.array([O.wire_size(int(f), 0, int(l)) for f, l in zip(flags, lens)], np.uint32)
    woff = np.zeros(n, np.uint64)
    woff[1:] = np.cumsum(wl.astype(np.uint64))[:-1]
    return dict(lens=lens, flags=flags, in_off=in_off, inp=inp, wl=wl, woff=woff, total=int(wl.sum()))


def _spliced(ref, b, tamper):
    frames = [ref[int(b["woff"][i]):int(b["woff"][i]) + int(b["wl"][i])].tobytes() for i in range(len(b["wl"]))]
    if tamper:
        j = len(frames) // 2
        frames.insert(j + 5, frames[j])                           # replay
        f = bytearray(frames[j + 9]); f[-1] ^= 1; frames[j + 9] = bytes(f)  # MAC failure
    m = len(frames)
    dwl = np.array([len(x) for x in frames], np.uint32)
    doff = np.zeros(m, np.uint64)
    doff[1:] = np.cumsum(dwl.astype(np.uint64))[:-1]
    dwire = np.frombuffer(b"".join(frames) + b"\0" * 64, np.uint8)
    plen = np.maximum(dwl.astype(np.int64) - 33, 0)
    pout = np.zeros(m, np.uint64)
    pout[1:] = np.cumsum(plen.astype(np.uint64))[:-1]
    return dict(m=m, dwl=dwl, doff=doff, dwire=dwire, plen=plen, pout=pout, psize=int(plen.sum()) + 1)


@pytest.mark.parametrize("which", ["slots", "two_thirds", "mixed_sizes", "enc_split", "dec_small", "enc_small"])
def test_duplex_rounds_bitexact(torch_cuda, C, which):
    torch = torch_cuda
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    slots = 256 * cus
    lo = (2 * slots - 1) // 3 + 1  # the smallest one-lane-per-frame batch
    # (frames of the decode batch before splicing in round 0 and of the encode
    # batch in round 1; frames of the encode batch in round 0)
    nd, ne, sizes = {"slots": (slots - 1, slots - 1, [1024]), "two_thirds": (lo, lo + 7, [256]),
                     "mixed_sizes": (slots - 2, lo, [0, 1, 33, 100, 1000, 2000, 4000, 4565]),
                     "enc_split": (slots - 2, slots + 1, [300]),  # encode beyond one lane per frame: two calls
                     "dec_small": (1000, slots, [512]),
                     "enc_small": (slots - 2, 100, [512])}[which]
    rng = np.random.default_rng(sum(which.encode()))
    key = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a).view(dt).copy()).cuda()
    enc = C.CurveContext(0, 1)
    enc.session_set(0, key, O.CLIENT_PREFIX, O.SERVER_PREFIX)
    enc.set_nonce(0, 3)
    dec = C.CurveContext(0, 1)
    dec.session_set(0, key, O.SERVER_PREFIX, O.CLIENT_PREFIX, False, 2)
    osess_e = O.make_sessions([key])
    osess_d = O.make_sessions([key], dec_prefix=O.CLIENT_PREFIX)
    peer = np.array([2], np.uint64)
    next_nonce = 3

    def oracle_encode(b):
        nonlocal next_nonce
        n = len(b["lens"])
        nonce = np.arange(next_nonce, next_nonce + n, dtype=np.uint64)
        next_nonce += n
        return O.encode_batch(osess_e, np.zeros(n, np.uint32), nonce, b["flags"], b["in_off"], b["lens"], b["inp"],
                              b["woff"], b["total"])

    def enc_args(b, wire):
        n = len(b["lens"])
        return dict(sid=t(np.zeros(n, np.uint32), np.int32), nonce=None, flags=t(b["flags"], np.uint8),
                    in_off=t(b["in_off"], np.int64), length=t(b["lens"], np.int32), inp=t(b["inp"], np.uint8),
                    out_off=t(b["woff"], np.int64), out=wire, max_len=4565, nonce_auto=True)

    # round 0: batch 0 encoded alone (the pipeline's fill)
    b = _batch(rng, nd, sizes)
    wire = torch.zeros(b["total"] + 64, dtype=torch.uint8, device="cuda")
    enc.encode_batch(**enc_args(b, wire))
    torch.cuda.synchronize()
    ref = oracle_encode(b)
    assert np.array_equal(wire.cpu().numpy()[:b["total"]], ref)

    for rnd in range(2):
        # decode of the previous round's wire (replay + tamper spliced in: the
        # frame count grows by one) with the next batch's encode
        s = _spliced(ref, b, tamper=True)
        if which == "dec_small" and rnd == 0:
            assert s["m"] < lo
        rout, rfl, rst = O.decode_batch(osess_d, peer, np.zeros(s["m"], np.uint32), s["doff"], s["dwl"], s["dwire"],
                                        s["pout"], s["psize"])
        out = torch.zeros(s["psize"], dtype=torch.uint8, device="cuda")
        fl = torch.zeros(s["m"], dtype=torch.uint8, device="cuda")
        st = torch.zeros(s["m"], dtype=torch.int32, device="cuda")
        b2 = _batch(rng, ne if rnd == 0 else nd, sizes)
        wire2 = torch.zeros(b2["total"] + 64, dtype=torch.uint8, device="cuda")
        dec.duplex_batch(dict(sid=t(np.zeros(s["m"], np.uint32), np.int32), in_off=t(s["doff"], np.int64),
                              wire_len=t(s["dwl"], np.int32), inp=t(s["dwire"], np.uint8),
                              out_off=t(s["pout"], np.int64), out=out, flags_out=fl, status_out=st, max_len=4608),
                         (enc, enc_args(b2, wire2)))
        torch.cuda.synchronize()
        gst = st.cpu().numpy()
        assert np.array_equal(gst, rst), (rnd, np.flatnonzero(gst != rst)[:5])
        assert (rst != 0).sum() == 2
        assert np.array_equal(fl.cpu().numpy(), rfl)
        o = out.cpu().numpy()
        mask = np.zeros(s["psize"], bool)
        for i in np.flatnonzero(rst == 0):
            mask[int(s["pout"][i]):int(s["pout"][i]) + int(s["plen"][i])] = True
        assert np.array_equal(o[mask], rout[mask])
        assert not o[~mask].any()  # failed frames' payload regions zero-filled
        assert dec.get_peer_nonce(0) == int(peer[0])
        ref = oracle_encode(b2)
        got = wire2.cpu().numpy()[:b2["total"]]
        assert np.array_equal(got, ref), (rnd, int(np.flatnonzero(got != ref)[0]))
        assert enc.get_nonce(0) == next_nonce
        b = b2


def test_duplex_same_ctx_runs_two_calls(torch_cuda, C):
    """A pair on one ctx (not independent state) is valid and runs as the two
    separate calls: the decode first, then the encode."""
    torch = torch_cuda
    rng = np.random.default_rng(7)
    key = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a).view(dt).copy()).cuda()
    ctx = C.CurveContext(0, 1)
    ctx.session_set(0, key, O.CLIENT_PREFIX, O.CLIENT_PREFIX, False, 2)  # decodes what it encodes
    ctx.set_nonce(0, 3)
    b = _batch(rng, 5000, [64])
    wire = torch.zeros(b["total"] + 64, dtype=torch.uint8, device="cuda")
    ea = dict(sid=t(np.zeros(5000, np.uint32), np.int32), nonce=None, flags=t(b["flags"], np.uint8),
              in_off=t(b["in_off"], np.int64), length=t(b["lens"], np.int32), inp=t(b["inp"], np.uint8),
              out_off=t(b["woff"], np.int64), out=wire, max_len=4565, nonce_auto=True)
    ctx.encode_batch(**ea)
    s = _spliced(wire.cpu().numpy(), b, tamper=False)
    out = torch.zeros(s["psize"], dtype=torch.uint8, device="cuda")
    fl = torch.zeros(s["m"], dtype=torch.uint8, device="cuda")
    st = torch.zeros(s["m"], dtype=torch.int32, device="cuda")
    wire2 = torch.zeros(b["total"] + 64, dtype=torch.uint8, device="cuda")
    ea["out"] = wire2
    ctx.duplex_batch(dict(sid=t(np.zeros(s["m"], np.uint32), np.int32), in_off=t(s["doff"], np.int64),
                          wire_len=t(s["dwl"], np.int32), inp=t(s["dwire"], np.uint8), out_off=t(s["pout"], np.int64),
                          out=out, flags_out=fl, status_out=st, max_len=4608), (ctx, ea))
    torch.cuda.synchronize()
    assert not st.cpu().numpy().any()
    assert ctx.get_peer_nonce(0) == 3 + 5000 - 1
    assert ctx.get_nonce(0) == 3 + 2 * 5000
    # the second batch carries the nonces after the first
    ref = O.encode_batch(O.make_sessions([key]), np.zeros(5000, np.uint32), np.arange(5003, 10003, dtype=np.uint64),
                         b["flags"], b["in_off"], b["lens"], b["inp"], b["woff"], b["total"])
    assert np.array_equal(wire2.cpu().numpy()[:b["total"]], ref)
