"""The frame-kernel variant rule (zmqg_curve.hip lanes_per_frame: slots =
CUs x 256 one-wave-per-SIMD lanes; n < slots/2 -> 4 lanes per frame, < 2/3
slots -> 2, <= slots -> k_frames_seq, <= 1.5 slots -> k_frames_split (the
first `slots` frames one lane each, the remainder 8, 4 or 2 lanes each in the
same launch), above -> k_frames_lds) at both sides of every boundary, on the
library's own choice (no forcing): each batch's wire bit-exact against the
oracle (src/curve_mechanism_base.cpp:111-205) with device-assigned nonces,
and its decode (one session: the in-kernel look-back, across the split's two
bodies) equal to the oracle's sequential decode, a replay and a tampered
frame included.  The split sizes also run with frames of up to 4.5 KiB (the
remainder lanes' Poly1305 combine over 8 / 4 / 2 lanes) and with 1 KiB
frames at 70,000 (DESIGN.md section 3.1's sweep row)."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _bounds(cus):
    slots = 256 * cus
    b = [slots // 2 - 1, slots // 2, (2 * slots - 1) // 3, (2 * slots - 1) // 3 + 1, 3 * slots // 2,
         3 * slots // 2 + 1,
         # k_frames_seq | split, and the split's remainder widths 8 | 4 | 2
         slots, slots + 1, slots + slots // 8, slots + slots // 8 + 1, slots + slots // 4, slots + slots // 4 + 1]
    return b


SMALL = [0, 1, 31, 64, 95, 130]
MIXED = [0, 1, 33, 100, 500, 1000, 1024, 2000, 3000, 4000, 4575, 4576]  # (4575 | 4576: the frame kernel | the body kernel)


@pytest.mark.parametrize("which,sizes", [(k, SMALL) for k in range(12)] + [(k, MIXED) for k in (7, 8, 9, 10, 11, 4)]
                         + [(70000, [1024])])
def test_variant_boundaries_bitexact(torch_cuda, C, which, sizes):
    torch = torch_cuda
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    n = _bounds(cus)[which] if which < 100 else which
    rng = np.random.default_rng(100 + which + len(sizes))
    key = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    lens = rng.choice(sizes, n).astype(np.uint32)
    flags = rng.choice([0, 1, 2, 3], n).astype(np.uint8)
    in_off = np.zeros(n, np.uint64)
    in_off[1:] = np.cumsum(lens.astype(np.uint64))[:-1]
    inp = rng.integers(0, 256, int(lens.sum()) + 1, dtype=np.uint8)
    wl = np.array([O.wire_size(int(f), 0, int(l)) for f, l in zip(flags, lens)], np.uint32)
    woff = np.zeros(n, np.uint64)
    woff[1:] = np.cumsum(wl.astype(np.uint64))[:-1]
    total = int(wl.sum())
    nonce = np.arange(3, 3 + n, dtype=np.uint64)
    ref = O.encode_batch(O.make_sessions([key]), np.zeros(n, np.uint32), nonce, flags, in_off, lens, inp, woff, total)

    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a).view(dt).copy()).cuda()
    enc = C.CurveContext(0, 1)
    enc.session_set(0, key, O.CLIENT_PREFIX, O.SERVER_PREFIX)
    enc.set_nonce(0, 3)
    sid = t(np.zeros(n, np.uint32), np.int32)
    wire = torch.zeros(total + 64, dtype=torch.uint8, device="cuda")
    enc.encode_batch(sid, None, t(flags, np.uint8), t(in_off, np.int64), t(lens, np.int32), t(inp, np.uint8),
                     t(woff, np.int64), wire, nonce_auto=True)
    torch.cuda.synchronize()
    got = wire.cpu().numpy()[:total]
    assert np.array_equal(got, ref), (n, int(np.flatnonzero(got != ref)[0]))

    # decode the wire with one replay and one tampered frame spliced in
    frames = [ref[int(woff[i]):int(woff[i]) + int(wl[i])].tobytes() for i in range(n)]
    j = n // 2
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
    psize = int(plen.sum()) + 1
    peer = np.array([2], np.uint64)
    rout, rfl, rst = O.decode_batch(O.make_sessions([key], dec_prefix=O.CLIENT_PREFIX), peer, np.zeros(m, np.uint32),
                                    doff, dwl, dwire, pout, psize)
    dec = C.CurveContext(0, 1)
    dec.session_set(0, key, O.SERVER_PREFIX, O.CLIENT_PREFIX, False, 2)
    out = torch.zeros(psize, dtype=torch.uint8, device="cuda")
    fl = torch.zeros(m, dtype=torch.uint8, device="cuda")
    st = torch.zeros(m, dtype=torch.int32, device="cuda")
    dec.decode_batch(t(np.zeros(m, np.uint32), np.int32), t(doff, np.int64), t(dwl, np.int32), t(dwire, np.uint8),
                     t(pout, np.int64), out, fl, st)
    torch.cuda.synchronize()
    gst = st.cpu().numpy()
    assert np.array_equal(gst, rst)
    assert (rst != 0).sum() >= 2
    assert np.array_equal(fl.cpu().numpy(), rfl)
    ok = rst == 0
    o = out.cpu().numpy()
    for i in np.flatnonzero(ok)[:: max(1, m // 4000)]:  # a spread sample of the payloads, plus the totals
        a, b = int(pout[i]), int(pout[i]) + int(plen[i])
        assert np.array_equal(o[a:b], rout[a:b]), i
    mask = np.zeros(psize, bool)
    for i in np.flatnonzero(ok):
        mask[int(pout[i]):int(pout[i]) + int(plen[i])] = True
    assert np.array_equal(o[mask], rout[mask])
    assert dec.get_peer_nonce(0) == int(peer[0])
