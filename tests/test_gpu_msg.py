"""GPU tests of the per-message entry points (zmqg_encode_msg /
zmqg_decode_msg, include/zmqg_curve.h), the calls the drop-in
zmq::curve_encoding_t makes once per message as the reference engine calls
its codec (src/stream_engine_base.cpp:281-291, :331-348), against the CPU
oracle (src/curve_mechanism_base.cpp:111-284 restated in oracle/):

* every flag / downgrade kind and sizes 0 .. 70,000 bytes (frames on both
  sides of the frame kernel's 4.5 KiB range), bit-exact wires;
* a message sequence decoded one call at a time with replays, reorders,
  tampering in every wire region, wrong-length and non-MESSAGE frames: the
  same statuses, payloads, flags and final peer nonce as the oracle's
  sequential decode;
* in-place decode (out == in) through the same buffer.
"""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _sessions(C, key, downgrade=False, peer=2):
    enc = C.CurveContext(0, 1)
    enc.session_set(0, key, O.CLIENT_PREFIX, O.SERVER_PREFIX, downgrade)
    dec = C.CurveContext(0, 1)
    dec.session_set(0, key, O.SERVER_PREFIX, O.CLIENT_PREFIX, False, peer)
    return enc, dec


def _oracle_wire(key, nonce, flags, payload, downgrade=False):
    sess = O.make_sessions([key], downgrade_sub=downgrade)
    p = np.frombuffer(payload, np.uint8) if payload else np.zeros(0, np.uint8)
    ws = O.wire_size(flags, 1 if downgrade else 0, len(p))
    w = O.encode_batch(sess, np.zeros(1, np.uint32), np.array([nonce], np.uint64), np.array([flags], np.uint8),
                       np.zeros(1, np.uint64), np.array([len(p)], np.uint32), p if len(p) else np.zeros(1, np.uint8),
                       np.zeros(1, np.uint64), ws)
    return bytes(w[:ws])


@pytest.mark.parametrize("downgrade", [False, True])
def test_encode_msg_matches_oracle(torch_cuda, C, downgrade):
    rng = np.random.default_rng(11 + downgrade)
    key = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    enc, _ = _sessions(C, key, downgrade)
    nonce = 3
    # 4052 ... 4064: the one-wave message kernel's limit (a 4,096-byte wire
    # frame) for every header length, on both sides
    for size in (0, 1, 31, 32, 33, 34, 63, 64, 65, 1024, 4052, 4053, 4054, 4056, 4062, 4063, 4064, 4400, 4500,
                 4600, 70000):
        for flags in (0, 1, 2, 3, 12, 13, 16, 17):
            pay = rng.integers(0, 256, size, dtype=np.uint8).tobytes()
            got = enc.encode_msg(0, nonce, flags, pay)
            assert got == _oracle_wire(key, nonce, flags, pay, downgrade), (size, flags)
            nonce += 1


def test_decode_msg_sequence_matches_oracle(torch_cuda, C):
    rng = np.random.default_rng(5)
    key = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    enc, dec = _sessions(C, key)
    frames, nonce = [], 3
    for size in (0, 5, 33, 1024, 4063, 4064, 5000, 70000):
        for flags in (0, 1, 2, 3):
            pay = rng.integers(0, 256, size, dtype=np.uint8).tobytes()
            frames.append(enc.encode_msg(0, nonce, flags, pay))
            nonce += 1
    seq = list(frames)
    seq.insert(3, frames[1])                     # replay
    seq.insert(7, frames[10])                    # from the future, then its predecessors fail
    t = bytearray(frames[12]); t[40] ^= 1        # ciphertext
    seq.append(bytes(t))
    t = bytearray(frames[13]); t[20] ^= 0x80     # tag
    seq.append(bytes(t))
    t = bytearray(frames[14]); t[1] ^= 1         # command name
    seq.append(bytes(t))
    seq.append(frames[15][:32])                  # too short for a MESSAGE
    seq.append(b"")                              # empty
    seq.append(frames[20][:-1])                  # truncated: MAC fails
    seq.append(frames[21])
    # oracle: the reference's sequential rule over the whole sequence
    wl = np.array([len(w) for w in seq], np.uint32)
    woff = np.zeros(len(seq), np.uint64)
    pos = 0
    for i, w in enumerate(seq):
        woff[i] = pos
        pos += len(w)
    wire = np.frombuffer(b"".join(seq) + b"\0" * 64, np.uint8)
    pout = np.zeros(len(seq), np.uint64)
    pp = 0
    for i, w in enumerate(seq):
        pout[i] = pp
        pp += max(len(w) - 33, 0)
    sess = O.make_sessions([key], dec_prefix=O.CLIENT_PREFIX)
    peer = np.array([2], np.uint64)
    out, fl, st = O.decode_batch(sess, peer, np.zeros(len(seq), np.uint32), woff, wl, wire, pout, pp + 1)
    for i, w in enumerate(seq):
        got, gfl, gst = dec.decode_msg(0, w)
        assert gst == int(st[i]), (i, gst, int(st[i]))
        if gst == 0:
            exp = bytes(out[int(pout[i]):int(pout[i]) + len(w) - 33])
            assert got == exp and gfl == int(fl[i]), i
    assert dec.get_peer_nonce(0) == int(peer[0])


def test_decode_msg_in_place(torch_cuda, C):
    """out == in: the payload lands at the front of the received bytes (the
    drop-in's decode then shrinks the msg_t to it)."""
    import ctypes
    from libzmq_amd import curve as CC
    rng = np.random.default_rng(9)
    key = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    enc, dec = _sessions(C, key)
    for i, size in enumerate((0, 40, 1024, 6000)):
        pay = rng.integers(0, 256, size, dtype=np.uint8).tobytes()
        w = np.frombuffer(enc.encode_msg(0, 3 + i, 1, pay), np.uint8).copy()
        fl = np.zeros(1, np.uint8)
        st = np.zeros(1, np.int32)
        p = w.ctypes.data_as(ctypes.c_void_p)
        rc = CC.lib().zmqg_decode_msg(dec._ctx, 0, p, len(w), p, fl.ctypes.data_as(ctypes.c_void_p),
                                      st.ctypes.data_as(ctypes.c_void_p))
        assert rc == 0 and st[0] == 0 and fl[0] == 1
        assert w[:size].tobytes() == pay


@pytest.mark.parametrize("where", ["side_stream", "null_stream"])
def test_msg_calls_follow_a_batch_on_another_stream(torch_cuda, C, where):
    """A per-message call right after a batch call of the same ctx on another
    stream, with no synchronisation between them: the message kernel runs on
    the ctx's own stream after the batch (msg_order), so it sees the peer
    nonce the batch advanced -- the next nonce decodes, an old one is a
    replay (src/curve_mechanism_base.cpp:98-106).  The batch stream is a
    torch side stream, or the null stream (handle 0): the ctx's own stream
    is non-blocking, so the null stream orders nothing by itself."""
    torch = torch_cuda
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(21)
    key = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    enc, dec = _sessions(C, key)
    n, P = 32768, 1024
    W = C.wire_size(0, 0, P)
    t = lambda a, d: torch.from_numpy(np.ascontiguousarray(a).view(d)).to(dev)
    sid = torch.zeros(n, dtype=torch.int32, device=dev)
    pay = torch.randint(0, 256, (n * P,), dtype=torch.uint8, device=dev)
    in_off = t(np.arange(n, dtype=np.uint64) * P, np.int64)
    lens = t(np.full(n, P, np.uint32), np.int32)
    w_off = t(np.arange(n, dtype=np.uint64) * W, np.int64)
    wl = t(np.full(n, W, np.uint32), np.int32)
    wire = torch.zeros(n * W, dtype=torch.uint8, device=dev)
    flags = torch.zeros(n, dtype=torch.uint8, device=dev)
    enc.encode_batch(sid, t(np.arange(3, 3 + n, dtype=np.uint64), np.int64), flags, in_off, lens, pay, w_off, wire)
    torch.cuda.synchronize()
    nxt = enc.encode_msg(0, 3 + n, 1, b"after the batch")
    old = bytes(wire[5 * W:6 * W].cpu().numpy())
    back = torch.zeros(n * P, dtype=torch.uint8, device=dev)
    fl = torch.zeros(n, dtype=torch.uint8, device=dev)
    st = torch.full((n,), -1, dtype=torch.int32, device=dev)
    if where == "side_stream":
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            dec.decode_batch(sid, w_off, wl, wire, in_off, back, fl, st, stream=s.cuda_stream)
    else:
        dec.decode_batch(sid, w_off, wl, wire, in_off, back, fl, st, stream=0)
    got, gfl, gst = dec.decode_msg(0, nxt)  # no synchronisation with the batch stream before this call
    assert gst == 0 and got == b"after the batch" and gfl == 1
    _, _, gst = dec.decode_msg(0, old)
    assert gst == C.ERR_INVALID_SEQUENCE
    torch.cuda.synchronize()
    assert int((st != 0).sum()) == 0 and torch.equal(back, pay)
    assert dec.get_peer_nonce(0) == 3 + n


def test_decode_msg_failed_frame_leaves_the_buffer(torch_cuda, C):
    """The message kernel stores the payload (into the ctx's staging area)
    while the tag is computed; a frame whose tag then fails must leave the
    caller's buffer as it was -- no speculative plaintext and no partial
    write (zmqg_decode_msg copies the payload out only after a status of 0),
    as for a frame failing its header checks.  The buffer starts out 0xAA."""
    import ctypes
    from libzmq_amd import curve as CC
    rng = np.random.default_rng(31)
    key = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    enc, dec = _sessions(C, key)
    nonce = 3
    for size in (0, 1, 40, 1024, 3000, 3935, 4000, 4063):
        for where in ("tag", "ciphertext", "command"):
            pay = rng.integers(0, 256, size, dtype=np.uint8).tobytes()
            w = bytearray(enc.encode_msg(0, nonce, 0, pay))
            nonce += 1
            pos = {"tag": 20, "ciphertext": 33 + size // 2 if size else 32, "command": 2}[where]
            w[pos] ^= 0x10
            w = np.frombuffer(bytes(w), np.uint8).copy()
            out = np.full(size + 64, 0xAA, np.uint8)
            fl = np.full(1, 7, np.uint8)
            st = np.zeros(1, np.int32)
            rc = CC.lib().zmqg_decode_msg(dec._ctx, 0, w.ctypes.data_as(ctypes.c_void_p), len(w),
                                          out.ctypes.data_as(ctypes.c_void_p), fl.ctypes.data_as(ctypes.c_void_p),
                                          st.ctypes.data_as(ctypes.c_void_p))
            exp = C.ERR_UNEXPECTED_COMMAND if where == "command" else C.ERR_CRYPTOGRAPHIC
            assert rc == 0 and st[0] == exp and fl[0] == 0, (size, where, st[0])
            assert (out == 0xAA).all(), (size, where)
    # the session still decodes its next frame
    pay = b"still in sequence"
    got, gfl, gst = dec.decode_msg(0, enc.encode_msg(0, nonce, 1, pay))
    assert gst == 0 and got == pay and gfl == 1


def _msg_poly_shape(stream_len):
    """(c, nl, levels) of k_msg's Poly1305 for a message of stream_len bytes
    after the 32-byte key (curve_msg.hpp, step 3)."""
    n = (stream_len + 15) // 16
    c = (n + 63) // 64 if n else 1
    nl = (n + c - 1) // c
    levels = 0
    while (1 << levels) < nl:
        levels += 1
    return c, nl, levels


def test_msg_poly_every_lane_shape(torch_cuda, C):
    """Payload sizes chosen so that k_msg's Poly1305 runs every shape it has:
    c = 1..4 blocks per lane (x = r, r^2, r^3, r^4) and 0..6 DPP prefix
    levels (row_shr 1-8, row_bcast 15 and 31), each at both ends of its
    range -- encode against the oracle, then decode back."""
    rng = np.random.default_rng(41)
    key = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    enc, dec = _sessions(C, key)
    # ciphertext m = 1 + P bytes (flags byte, no SUBSCRIBE/CANCEL prefix)
    sizes = sorted({0, 15, 16, 31, 32, 47, 48, 63, 64, 127, 128, 129, 255, 256, 257, 500, 511, 512, 513, 767,
                    1000, 1023, 1024, 1025, 1500, 2047, 2048, 2049, 2500, 3000, 3071, 3072, 3073, 3500, 3935})
    shapes = {_msg_poly_shape(1 + p)[0::2] for p in sizes}
    assert {(c, lv) for c in (1, 2, 3, 4) for lv in range(7) if c == 1 or lv == 6} <= shapes | {(1, 0)}
    nonce = 3
    for p in sizes:
        pay = rng.integers(0, 256, p, dtype=np.uint8).tobytes()
        w = enc.encode_msg(0, nonce, 1, pay)
        assert w == _oracle_wire(key, nonce, 1, pay), (p, _msg_poly_shape(1 + p))
        got, gfl, gst = dec.decode_msg(0, w)
        assert gst == 0 and got == pay and gfl == 1, (p, gst)
        nonce += 1


def test_decode_msg_random_tampering_matches_oracle(torch_cuda, C):
    """Random sizes across every inline class and the memory route, random
    flags, and for most frames one flipped bit at a random wire position (or
    a truncation): each frame's status, flags and payload equal the oracle's
    sequential decode of the same sequence (src/curve_mechanism_base.cpp:
    80-284), peer-nonce advance included."""
    rng = np.random.default_rng(77)
    key = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    enc, dec = _sessions(C, key)
    seq, nonce = [], 3
    for _ in range(160):
        size = int(rng.choice([rng.integers(0, 64), rng.integers(64, 1100), rng.integers(1100, 4064)]))
        flags = int(rng.integers(0, 4))
        w = bytearray(enc.encode_msg(0, nonce, flags, rng.integers(0, 256, size, dtype=np.uint8).tobytes()))
        nonce += int(rng.choice([1, 1, 1, 2]))
        r = rng.random()
        if r < 0.6:
            pos = int(rng.integers(0, len(w)))
            w[pos] ^= 1 << int(rng.integers(0, 8))
        elif r < 0.7:
            w = w[:int(rng.integers(0, len(w)))]
        seq.append(bytes(w))
        if rng.random() < 0.05 and len(seq) > 2:  # a replay of an earlier frame
            seq.append(seq[int(rng.integers(0, len(seq) - 1))])
    wl = np.array([len(w) for w in seq], np.uint32)
    woff = np.concatenate([[0], np.cumsum(wl[:-1])]).astype(np.uint64)
    wire = np.frombuffer(b"".join(seq) + b"\0" * 64, np.uint8)
    pout = np.concatenate([[0], np.cumsum([max(len(w) - 33, 0) for w in seq][:-1])]).astype(np.uint64)
    sess = O.make_sessions([key], dec_prefix=O.CLIENT_PREFIX)
    peer = np.array([2], np.uint64)
    out, fl, st = O.decode_batch(sess, peer, np.zeros(len(seq), np.uint32), woff, wl, wire, pout,
                                 int(pout[-1]) + len(seq[-1]) + 1)
    for i, w in enumerate(seq):
        got, gfl, gst = dec.decode_msg(0, w)
        assert gst == int(st[i]), (i, len(w), gst, int(st[i]))
        if gst == 0:
            assert got == bytes(out[int(pout[i]):int(pout[i]) + len(w) - 33]) and gfl == int(fl[i]), i
    assert dec.get_peer_nonce(0) == int(peer[0])
