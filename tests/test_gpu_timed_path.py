"""GPU parity of the exact launch mode bench.py times, and
of the send-nonce pre-pass over many tiles.

* The bench step: 65,536 x 1 KiB on one session, encode with
  ZMQG_OPT_NONCE_AUTO (the session's device send counter assigns the nonces,
  as get_and_inc_nonce does, src/curve_mechanism_base.cpp:114-116) and
  max_len = P, then decode with max_len = W -- checked byte for byte against
  the oracle on two consecutive steps (the counter carries over), for every
  one-lane-per-frame variant.
* One-session decode at 65,536 frames with replays, reorders, a nonce jump,
  MAC and header tampering spread over many workgroups: the cross-workgroup
  replay rule (src/curve_mechanism_base.cpp:98-106, the peer nonce advanced
  before the MAC check) against the oracle's sequential decode.
* NONCE_AUTO over several sessions above 262,144 frames, where the nonce
  pre-pass scans its tile table in two or more row blocks.
* ZMQG_OPT_STREAM_OUT (decode, a cache hint: whole-segment output stores
  staged through LDS) on the replay batch and on mixed lengths whose payloads
  start 64-byte aligned, so lanes reach their last window at different
  steps -- the same bytes, statuses and flags as the oracle; and on encode
  (staged 64-byte windows at 4-byte-aligned places) over ragged payloads,
  packed wire frames and several sessions."""
import os

import numpy as np
import pytest

from oracle import oracle as O
from tests.test_gpu_parity import dev, host

pytestmark = pytest.mark.gpu

N, P = 65536, 1024
W = P + 33
VARIANTS = ["default", "0", "8"]  # the library's choice, k_frames_seq, k_frames_lds


def _ctx(C, variant, sessions=1):
    old = os.environ.pop("ZMQG_FRAMES_G", None)
    try:
        if variant != "default":
            os.environ["ZMQG_FRAMES_G"] = variant
        return C.CurveContext(0, sessions)
    finally:
        os.environ.pop("ZMQG_FRAMES_G", None)
        if old is not None:
            os.environ["ZMQG_FRAMES_G"] = old


@pytest.mark.parametrize("variant", VARIANTS)
def test_bench_step_bitexact(torch_cuda, C, variant):
    torch = torch_cuda
    rng = np.random.default_rng(77)
    precom = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    enc = _ctx(C, variant)
    enc.session_set(0, precom, O.CLIENT_PREFIX, O.SERVER_PREFIX)
    enc.set_nonce(0, 3)
    dec = _ctx(C, variant)
    dec.session_set(0, precom, O.SERVER_PREFIX, O.CLIENT_PREFIX, False, 2)
    inp = rng.integers(0, 256, N * P, dtype=np.uint8)
    flags = np.where(np.arange(N) % 16 == 15, 1, 0).astype(np.uint8)
    sid = np.zeros(N, np.uint32)
    in_off = np.arange(N, dtype=np.uint64) * P
    out_off = np.arange(N, dtype=np.uint64) * W
    d_sid, d_fl, d_in, d_off = dev(torch, sid), dev(torch, flags), dev(torch, inp), dev(torch, in_off)
    d_len, d_out, d_wl = dev(torch, np.full(N, P, np.uint32)), dev(torch, out_off), dev(torch, np.full(N, W, np.uint32))
    wire = torch.zeros(N * W, dtype=torch.uint8, device="cuda")
    back = torch.zeros(N * P, dtype=torch.uint8, device="cuda")
    fl = torch.zeros(N, dtype=torch.uint8, device="cuda")
    st = torch.full((N,), -1, dtype=torch.int32, device="cuda")
    sess = O.make_sessions([precom])
    for step in range(2):
        back.zero_()
        enc.encode_batch(d_sid, None, d_fl, d_off, d_len, d_in, d_out, wire, max_len=P, nonce_auto=True)
        dec.decode_batch(d_sid, d_out, d_wl, wire, d_off, back, fl, st, max_len=W)
        torch.cuda.synchronize()
        nonce = np.arange(3 + step * N, 3 + (step + 1) * N, dtype=np.uint64)
        ref = O.encode_batch(sess, sid, nonce, flags, in_off, np.full(N, P, np.uint32), inp, out_off, N * W)
        got = host(wire, np.uint8)
        bad = np.nonzero(got != ref)[0]
        assert bad.size == 0, f"step {step}: {bad.size} wire bytes differ, first at frame {int(bad[0]) // W}"
        assert (host(st, np.int32) == 0).all()
        assert np.array_equal(host(fl, np.uint8), flags)
        assert np.array_equal(host(back, np.uint8), inp)
        assert enc.get_nonce(0) == 3 + (step + 1) * N
        assert dec.get_peer_nonce(0) == 2 + (step + 1) * N


@pytest.mark.parametrize("stream_out", [False, True])
@pytest.mark.parametrize("variant", VARIANTS)
def test_one_session_decode_replays_across_workgroups(torch_cuda, C, variant, stream_out):
    torch = torch_cuda
    rng = np.random.default_rng(78)
    precom = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    nonce = np.arange(3, 3 + N, dtype=np.uint64)
    nonce[40000] = nonce[100]                            # replay of a frame 155 workgroups earlier
    nonce[20000], nonce[20300] = nonce[20300], nonce[20000]  # reorder across a workgroup seam: 20001..20300 fail
    nonce[777] = nonce[776]                              # replay of the frame just before
    nonce[65000] = 3 + N + 100                           # jump: the 535 frames after it fail
    nonce[5000:5010] = nonce[5000:5010][::-1].copy()     # reversed run inside one workgroup
    flags = (rng.integers(0, 4, N) == 0).astype(np.uint8)
    inp = rng.integers(0, 256, N * P, dtype=np.uint8)
    in_off = np.arange(N, dtype=np.uint64) * P
    out_off = np.arange(N, dtype=np.uint64) * W
    sid = np.zeros(N, np.uint32)
    sess = O.make_sessions([precom])
    wire = O.encode_batch(sess, sid, nonce, flags, in_off, np.full(N, P, np.uint32), inp, out_off, N * W)
    wire[out_off[12345] + 500] ^= 0x10   # MAC failure (advances the peer nonce)
    wire[out_off[23456] + 3] ^= 0x01     # "\x07MESSAGE" broken: UNEXPECTED_COMMAND (peer unchanged)
    wire[out_off[33333] + 20] ^= 0x80    # tag byte: MAC failure
    dsess = O.make_sessions([precom], enc_prefix=O.SERVER_PREFIX, dec_prefix=O.CLIENT_PREFIX)
    peer = np.array([2], np.uint64)
    rpl, rfl, rst = O.decode_batch(dsess, peer, sid, out_off, np.full(N, W, np.uint32), wire, in_off, N * P)
    assert (rst != 0).sum() > 540
    dec = _ctx(C, variant)
    dec.session_set(0, precom, O.SERVER_PREFIX, O.CLIENT_PREFIX, False, 2)
    back = torch.full((N * P,), 0xEE, dtype=torch.uint8, device="cuda")
    fl = torch.zeros(N, dtype=torch.uint8, device="cuda")
    st = torch.zeros(N, dtype=torch.int32, device="cuda")
    dec.decode_batch(dev(torch, sid), dev(torch, out_off), dev(torch, np.full(N, W, np.uint32)), dev(torch, wire),
                     dev(torch, in_off), back, fl, st, max_len=W, stream_out=stream_out)
    torch.cuda.synchronize()
    gst = host(st, np.int32)
    assert np.array_equal(gst, rst[:N]), np.nonzero(gst != rst[:N])[0][:10]
    assert np.array_equal(host(fl, np.uint8), rfl[:N])
    assert np.array_equal(host(back, np.uint8), rpl[:N * P])
    assert dec.get_peer_nonce(0) == int(peer[0])


def test_nonce_auto_many_tiles_several_sessions(torch_cuda, C):
    """> 262,144 frames: the send-nonce pre-pass (k_nonce_*) runs its column
    scan in several row blocks; every frame's nonce must be its session's
    counter plus its rank among the session's earlier frames, and the
    counters must advance by the session counts, over two calls."""
    torch = torch_cuda
    rng = np.random.default_rng(79)
    n, S, L = 300_000, 7, 8
    precoms = [rng.integers(0, 256, 32, dtype=np.uint8).tobytes() for _ in range(S)]
    ctx = C.CurveContext(0, S)
    base = [3 + 1000 * s for s in range(S)]
    for s in range(S):
        ctx.session_set(s, precoms[s], O.CLIENT_PREFIX, O.SERVER_PREFIX)
        ctx.set_nonce(s, base[s])
    sid = rng.integers(0, S, n).astype(np.uint32)
    sid[:50_000] = 3  # a long run of one session, then the mix
    flags = np.zeros(n, np.uint8)
    inp = rng.integers(0, 256, n * L, dtype=np.uint8)
    in_off = np.arange(n, dtype=np.uint64) * L
    Wn = L + 33
    out_off = np.arange(n, dtype=np.uint64) * Wn
    out = torch.zeros(n * Wn, dtype=torch.uint8, device="cuda")
    d = [dev(torch, a) for a in (sid, flags, in_off, np.full(n, L, np.uint32), inp, out_off)]
    nxt = list(base)
    for call in range(2):
        ctx.encode_batch(d[0], None, d[1], d[2], d[3], d[4], d[5], out, nonce_auto=True)
        torch.cuda.synchronize()
        w = host(out, np.uint8).reshape(n, Wn)
        got = w[:, 8:16].copy().view(">u8").reshape(n).astype(np.uint64)
        want = np.zeros(n, np.uint64)
        for s in range(S):
            idx = np.nonzero(sid == s)[0]
            want[idx] = nxt[s] + np.arange(idx.size, dtype=np.uint64)
            nxt[s] += idx.size
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, f"call {call}: {bad.size} nonces differ, first at frame {bad[:5]}"
        for s in range(S):
            assert ctx.get_nonce(s) == nxt[s]
        # and the boxes under those nonces, on a sample of frames
        pick = np.sort(rng.choice(n, 3000, replace=False))
        sess = O.make_sessions(precoms)
        ref = O.encode_batch(sess, sid[pick], got[pick], flags[pick], in_off[pick], np.full(pick.size, L, np.uint32),
                             inp, np.arange(pick.size, dtype=np.uint64) * Wn, pick.size * Wn)
        assert np.array_equal(ref.reshape(pick.size, Wn), w[pick])


@pytest.mark.parametrize("variant", ["default", "0"])
def test_stream_out_mixed_lengths(torch_cuda, C, variant):
    """ZMQG_OPT_STREAM_OUT over payloads of 0 ... 4,400 bytes at 64-byte
    aligned offsets (the staged whole-segment stores apply), packed wire,
    one session with a replay and a tampered frame: lanes reach their last
    window at different steps, so staged chunks and each lane's own tail
    stores interleave -- against the oracle's sequential decode."""
    torch = torch_cuda
    rng = np.random.default_rng(80)
    n = 20000
    lens = rng.integers(0, 4400, n).astype(np.uint32)
    lens[::97] = 0
    lens[5::101] = 64 * rng.integers(1, 60, lens[5::101].size)
    slot = (lens.astype(np.uint64) + 63) // 64 * 64 + 64 * rng.integers(0, 2, n).astype(np.uint64)
    in_off = np.concatenate([[0], np.cumsum(slot)[:-1]]).astype(np.uint64)
    W_ = lens.astype(np.uint64) + 33
    out_off = np.concatenate([[0], np.cumsum(W_)[:-1]]).astype(np.uint64)
    precom = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    sid = np.zeros(n, np.uint32)
    nonce = np.arange(3, 3 + n, dtype=np.uint64)
    nonce[9000] = nonce[8000]  # replay across workgroups
    flags = (rng.integers(0, 4, n) == 0).astype(np.uint8)
    total = int(in_off[-1] + slot[-1])
    inp = rng.integers(0, 256, total, dtype=np.uint8)
    sess = O.make_sessions([precom])
    wtot = int(out_off[-1] + W_[-1])
    wire = O.encode_batch(sess, sid, nonce, flags, in_off, lens, inp, out_off, wtot)
    big = int(np.nonzero(lens > 2000)[0][3])
    wire[out_off[big] + 1500] ^= 0x04  # MAC failure
    dsess = O.make_sessions([precom], enc_prefix=O.SERVER_PREFIX, dec_prefix=O.CLIENT_PREFIX)
    peer = np.array([2], np.uint64)
    rpl, rfl, rst = O.decode_batch(dsess, peer, sid, out_off, W_.astype(np.uint32), wire, in_off, total)
    assert rst[9000] != 0 and rst[big] != 0
    dec = _ctx(C, variant)
    dec.session_set(0, precom, O.SERVER_PREFIX, O.CLIENT_PREFIX, False, 2)
    back = torch.full((total,), 0xEE, dtype=torch.uint8, device="cuda")
    fl = torch.zeros(n, dtype=torch.uint8, device="cuda")
    st = torch.zeros(n, dtype=torch.int32, device="cuda")
    dec.decode_batch(dev(torch, sid), dev(torch, out_off), dev(torch, W_.astype(np.uint32)), dev(torch, wire),
                     dev(torch, in_off), back, fl, st, max_len=int(W_.max()), stream_out=True)
    torch.cuda.synchronize()
    assert np.array_equal(host(st, np.int32), rst[:n])
    assert np.array_equal(host(fl, np.uint8), rfl[:n])
    got = host(back, np.uint8)
    # payload regions as the oracle writes them (the gaps between are untouched: 0xEE)
    for i in range(n):
        a, L = int(in_off[i]), int(lens[i])
        if not np.array_equal(got[a:a + L], rpl[a:a + L]):
            raise AssertionError(f"frame {i} (len {L}) differs")
    assert dec.get_peer_nonce(0) == int(peer[0])


@pytest.mark.parametrize("variant", ["default", "0"])
def test_stream_out_encode_mixed_lengths(torch_cuda, C, variant):
    """ZMQG_OPT_STREAM_OUT on encode: the one-lane kernel stages each
    window's 64 output bytes and stores them a step later, 16 frames per
    instruction, at frame_store's 4-byte-aligned places; each frame's last
    window stays per lane.  Payloads of 0 ... 4,400 bytes (and a few for the
    body kernel) at unaligned input offsets, packed wire frames at every
    alignment, three sessions, random flags: the whole output buffer against
    the oracle's sequential encode, bytes past the last frame untouched."""
    torch = torch_cuda
    rng = np.random.default_rng(81)
    n, S = 20000, 3
    lens = rng.integers(0, 4400, n).astype(np.uint32)
    lens[::97] = 0
    lens[7::1999] = rng.integers(5000, 12000, lens[7::1999].size)
    in_off = np.concatenate([[0], np.cumsum(lens.astype(np.uint64) + rng.integers(0, 8, n).astype(np.uint64))[:-1]])
    in_off = in_off.astype(np.uint64)
    W_ = lens.astype(np.uint64) + 33
    out_off = np.concatenate([[0], np.cumsum(W_)[:-1]]).astype(np.uint64)
    precoms = [rng.integers(0, 256, 32, dtype=np.uint8).tobytes() for _ in range(S)]
    sid = rng.integers(0, S, n).astype(np.uint32)
    nonce = rng.integers(1, 1 << 40, n).astype(np.uint64)
    flags = rng.integers(0, 4, n).astype(np.uint8)
    total = int(in_off[-1] + lens[-1]) + 8
    inp = rng.integers(0, 256, total, dtype=np.uint8)
    wtot = int(out_off[-1] + W_[-1])
    ref = O.encode_batch(O.make_sessions(precoms), sid, nonce, flags, in_off, lens, inp, out_off, wtot)
    enc = _ctx(C, variant, S)
    for s in range(S):
        enc.session_set(s, precoms[s], O.CLIENT_PREFIX, O.SERVER_PREFIX)
    out = torch.full((wtot + 256,), 0xEE, dtype=torch.uint8, device="cuda")
    enc.encode_batch(dev(torch, sid), dev(torch, nonce), dev(torch, flags), dev(torch, in_off), dev(torch, lens),
                     dev(torch, inp), dev(torch, out_off), out, stream_out=True)
    torch.cuda.synchronize()
    got = host(out, np.uint8)
    assert (got[wtot:] == 0xEE).all()
    bad = np.nonzero(got[:wtot] != ref[:wtot])[0]
    if bad.size:
        f = int(np.searchsorted(out_off, bad[0], side="right")) - 1
        raise AssertionError(f"{bad.size} bytes differ, first at {bad[0]} (frame {f}, len {lens[f]})")
