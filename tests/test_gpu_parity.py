"""GPU parity: the HIP path (through the C ABI) against the CPU oracle and the
golden vectors.  Every comparison is bit-exact (integer / byte work).

Mirrors the reference's own hot-path test (unittests/unittest_curve_encoding.cpp:
round trips of empty, 32 B, 2048 B and empty+MORE messages) and widens it to
batches, every flag case, failure paths and the BASELINE.json configs.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from oracle import oracle as O
from tests.helpers import pack, random_batch, wire_layout

pytestmark = pytest.mark.gpu

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "curve_golden.json")))
H = bytes.fromhex


def dev(torch, a):
    a = np.ascontiguousarray(a)
    if a.dtype == np.uint64:
        a = a.view(np.int64)
    elif a.dtype == np.uint32:
        a = a.view(np.int32)
    return torch.from_numpy(a.copy()).to("cuda")


def host(t, dtype):
    return t.cpu().numpy().view(dtype)


def gpu_encode(torch, ctx, b, out_off, out_size):
    out = torch.zeros(max(out_size, 1), dtype=torch.uint8, device="cuda")
    ctx.encode_batch(dev(torch, b["sid"]), dev(torch, b["nonce"]), dev(torch, b["flags"]), dev(torch, b["in_off"]),
                     dev(torch, b["lens"]), dev(torch, b["inp"]), dev(torch, out_off), out)
    torch.cuda.synchronize()
    return host(out, np.uint8)[:out_size]


def gpu_decode(torch, ctx, sid, in_off, wire_len, inp, out_off, out_size, fill=0):
    n = len(sid)
    out = torch.full((max(out_size, 1),), fill, dtype=torch.uint8, device="cuda")
    fl = torch.zeros(n, dtype=torch.uint8, device="cuda")
    st = torch.zeros(n, dtype=torch.int32, device="cuda")
    ctx.decode_batch(dev(torch, np.asarray(sid, np.uint32)), dev(torch, np.asarray(in_off, np.uint64)),
                     dev(torch, np.asarray(wire_len, np.uint32)), dev(torch, inp),
                     dev(torch, np.asarray(out_off, np.uint64)), out, fl, st)
    torch.cuda.synchronize()
    return host(out, np.uint8)[:out_size], host(fl, np.uint8), host(st, np.int32)


# ------------------------------------------------------------------ golden
def test_golden_encode_batch(torch_cuda, C):
    vecs = GOLDEN["encode"]
    ctx = C.CurveContext(0, len(vecs))
    for i, v in enumerate(vecs):
        ctx.session_set(i, H(v["precom"]), v["prefix"].encode(), O.SERVER_PREFIX, v["downgrade_sub"])
    rng = np.random.default_rng(1)
    payloads = [H(v["payload"]) for v in vecs]
    inp, in_off = pack(payloads, rng, max_gap=17)
    b = dict(sid=np.arange(len(vecs), dtype=np.uint32), nonce=np.array([v["nonce"] for v in vecs], np.uint64),
             flags=np.array([v["flags"] for v in vecs], np.uint8), in_off=in_off,
             lens=np.array([len(p) for p in payloads], np.uint32), inp=inp)
    wires = [H(v["wire"]) for v in vecs]
    out_off = pack(wires, rng, max_gap=13)[1]
    size = int(out_off[-1]) + len(wires[-1])
    out = gpu_encode(torch_cuda, ctx, b, out_off, size)
    for i, w in enumerate(wires):
        got = out[int(out_off[i]):int(out_off[i]) + len(w)].tobytes()
        assert got == w, f"vector {i} (len {len(payloads[i])}, flags {vecs[i]['flags']})"


def test_golden_survey_pin(torch_cuda, C):
    v = GOLDEN["survey_pin"]
    ctx = C.CurveContext(0, 1)
    ctx.session_set(0, H(v["precom"]), O.CLIENT_PREFIX, O.SERVER_PREFIX)
    payload = np.array([(i * 7 + 3) & 0xFF for i in range(1024)], np.uint8)
    b = dict(sid=np.zeros(1, np.uint32), nonce=np.ones(1, np.uint64), flags=np.zeros(1, np.uint8),
             in_off=np.zeros(1, np.uint64), lens=np.array([1024], np.uint32), inp=payload)
    out = gpu_encode(torch_cuda, ctx, b, np.zeros(1, np.uint64), 1057)
    assert out[:36].tobytes().hex() == v["reference_wire_prefix"]
    assert out.tobytes().hex() == v["wire"]


def test_golden_decode_sequences(torch_cuda, C):
    seqs = GOLDEN["decode"]
    ctx = C.CurveContext(0, len(seqs))
    sid, wires, exp = [], [], []
    for s, seq in enumerate(seqs):
        ctx.session_set(s, H(seq["precom"]), O.CLIENT_PREFIX, seq["prefix"].encode(), False, seq["peer_nonce"])
        for m in seq["msgs"]:
            sid.append(s)
            wires.append(H(m["wire"]))
            exp.append(m)
    # interleave sessions while keeping each session's order
    order = np.argsort(np.array([k * 1000 + s for s, k in zip(sid, _ranks(sid))]), kind="stable")
    sid = [sid[i] for i in order]
    wires = [wires[i] for i in order]
    exp = [exp[i] for i in order]
    rng = np.random.default_rng(2)
    inp, in_off = pack(wires, rng, max_gap=9)
    plen = [max(len(w) - 33, 0) for w in wires]
    _, out_off = pack([b"\0" * p for p in plen], rng, max_gap=7)
    size = int(out_off[-1]) + plen[-1] + 1
    out, fl, st = gpu_decode(torch_cuda, ctx, sid, in_off, [len(w) for w in wires], inp, out_off, size, fill=0xAB)
    for i, m in enumerate(exp):
        assert st[i] == m["status"], (i, hex(int(st[i])), hex(m["status"]))
        seg = out[int(out_off[i]):int(out_off[i]) + plen[i]].tobytes()
        if m["status"] == 0:
            assert fl[i] == m["flags"]
            assert seg.hex() == m["payload"]
        else:
            assert fl[i] == 0
            if len(wires[i]) >= 33:
                assert seg == b"\0" * plen[i], "failed frame must not leave plaintext"
    for s, seq in enumerate(seqs):
        assert ctx.get_peer_nonce(s) == seq["peer_nonce_after"], seq["name"]


def _ranks(sid):
    seen = {}
    out = []
    for s in sid:
        out.append(seen.get(s, 0))
        seen[s] = out[-1] + 1
    return out


@pytest.mark.parametrize("idx", range(4))
def test_golden_large(torch_cuda, C, idx):
    v = GOLDEN["large"][idx]
    ctx = C.CurveContext(0, 1)
    ctx.session_set(0, H(v["precom"]), O.CLIENT_PREFIX, O.SERVER_PREFIX)
    payload = np.frombuffer(O.splitmix_bytes(v["payload_seed"], v["payload_len"]), np.uint8)
    b = dict(sid=np.zeros(1, np.uint32), nonce=np.array([v["nonce"]], np.uint64),
             flags=np.array([v["flags"]], np.uint8), in_off=np.zeros(1, np.uint64),
             lens=np.array([v["payload_len"]], np.uint32), inp=payload)
    out = gpu_encode(torch_cuda, ctx, b, np.zeros(1, np.uint64), v["wire_len"])
    assert hashlib.sha256(out.tobytes()).hexdigest() == v["wire_sha256"]
    # and back
    ctx2 = C.CurveContext(0, 1)
    ctx2.session_set(0, H(v["precom"]), O.SERVER_PREFIX, O.CLIENT_PREFIX, False, 0)
    pl, fl, st = gpu_decode(torch_cuda, ctx2, [0], [0], [v["wire_len"]], out, [0], v["payload_len"])
    assert st[0] == 0 and fl[0] == v["flags"]
    assert np.array_equal(pl, payload)


# ------------------------------------------------------------------ random vs oracle
def _roundtrip_vs_oracle(torch, C, rng, n, sizes, n_sessions, flag_choices, max_gap, downgrade=None):
    precoms = [rng.integers(0, 256, 32, dtype=np.uint8).tobytes() for _ in range(n_sessions)]
    downgrade = downgrade or [False] * n_sessions
    enc = C.CurveContext(0, n_sessions)
    dec = C.CurveContext(0, n_sessions)
    for s in range(n_sessions):
        enc.session_set(s, precoms[s], O.CLIENT_PREFIX, O.SERVER_PREFIX, downgrade[s])
        dec.session_set(s, precoms[s], O.SERVER_PREFIX, O.CLIENT_PREFIX, downgrade[s], 2)
    b = random_batch(rng, n, sizes, n_sessions, flag_choices, max_gap=max_gap)
    out_off, wl, total = wire_layout(b["flags"], b["lens"], downgrade, b["sid"], rng, max_gap)
    gpu = gpu_encode(torch, enc, b, out_off, total)
    sess_o = np.concatenate([O.make_sessions([precoms[s]], downgrade_sub=downgrade[s]) for s in range(n_sessions)])
    ref = O.encode_batch(sess_o, b["sid"], b["nonce"], b["flags"], b["in_off"], b["lens"], b["inp"], out_off, total)
    for i in range(n):
        a, z = int(out_off[i]), int(out_off[i]) + int(wl[i])
        assert np.array_equal(gpu[a:z], ref[a:z]), f"frame {i} len {b['lens'][i]} flags {b['flags'][i]}"
    # decode the GPU wire on the GPU and on the oracle
    plen = wl.astype(np.int64) - 33
    _, pout = pack([b"\0" * int(p) for p in plen], rng, max_gap)
    psize = int(pout[-1]) + int(plen[-1]) + 1
    pl, fl, st = gpu_decode(torch, dec, b["sid"], out_off, wl, gpu, pout, psize)
    sess_d = np.concatenate([O.make_sessions([precoms[s]], dec_prefix=O.CLIENT_PREFIX, downgrade_sub=downgrade[s])
                             for s in range(n_sessions)])
    peer = np.full(n_sessions, 2, np.uint64)
    rpl, rfl, rst = O.decode_batch(sess_d, peer, b["sid"], out_off, wl, gpu, pout, psize)
    assert np.array_equal(st, rst)
    assert np.array_equal(fl, rfl)
    assert np.array_equal(pl, rpl)
    assert (st == 0).all()
    for s in range(n_sessions):
        assert dec.get_peer_nonce(s) == int(peer[s])
    return b, gpu, out_off, wl


def test_random_small_mixed(torch_cuda, C):
    rng = np.random.default_rng(10)
    sizes = list(range(0, 80)) + [127, 128, 129, 223, 224, 225, 255, 256, 257, 479, 480, 481, 1023, 1024, 1025]
    _roundtrip_vs_oracle(torch_cuda, C, rng, 700, sizes, 5, (0, 1, 2, 3, 12, 16, 13, 17), max_gap=15)


def test_random_downgrade_sub(torch_cuda, C):
    rng = np.random.default_rng(11)
    _roundtrip_vs_oracle(torch_cuda, C, rng, 200, list(range(0, 300)), 3, (0, 12, 16, 13), 7,
                         downgrade=[True, False, True])


def test_random_medium_multiwave(torch_cuda, C):
    # frames of 16..70 KiB span several 64-chunk waves: atomics + last-arriver path
    rng = np.random.default_rng(12)
    sizes = [16384 - 1, 16384, 16384 + 31, 65536 - 33, 65536, 65536 + 1, 70000]
    _roundtrip_vs_oracle(torch_cuda, C, rng, 40, sizes, 3, (0, 1), max_gap=33)


def test_config3_mixed_sessions(torch_cuda, C):
    # BASELINE config 3 shape at reduced count: {64 B, 1 KiB, 64 KiB}, 256 sessions
    rng = np.random.default_rng(13)
    _roundtrip_vs_oracle(torch_cuda, C, rng, 600, [64, 1024, 65536], 256, (0, 1), max_gap=0)


def test_config2_shape_bitexact(torch_cuda, C):
    """BASELINE config 2 at full size: 64 Ki x 1 KiB, one session."""
    torch = torch_cuda
    rng = np.random.default_rng(14)
    n, P = 65536, 1024
    precom = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    ctx = C.CurveContext(0, 1)
    ctx.session_set(0, precom, O.CLIENT_PREFIX, O.SERVER_PREFIX)
    inp = rng.integers(0, 256, n * P, dtype=np.uint8)
    flags = np.where(np.arange(n) % 16 == 15, 1, 0).astype(np.uint8)
    b = dict(sid=np.zeros(n, np.uint32), nonce=np.arange(3, 3 + n, dtype=np.uint64), flags=flags,
             in_off=np.arange(n, dtype=np.uint64) * P, lens=np.full(n, P, np.uint32), inp=inp)
    W = P + 33
    out_off = np.arange(n, dtype=np.uint64) * W
    gpu = gpu_encode(torch, ctx, b, out_off, n * W)
    sess = O.make_sessions([precom])
    ref = O.encode_batch(sess, b["sid"], b["nonce"], flags, b["in_off"], b["lens"], inp, out_off, n * W)
    assert np.array_equal(gpu, ref)
    dec = C.CurveContext(0, 1)
    dec.session_set(0, precom, O.SERVER_PREFIX, O.CLIENT_PREFIX, False, 2)
    pl, fl, st = gpu_decode(torch, dec, np.zeros(n, np.uint32), out_off, np.full(n, W, np.uint32), gpu,
                            b["in_off"], n * P)
    assert (st == 0).all() and np.array_equal(fl, flags) and np.array_equal(pl, inp)
    assert dec.get_peer_nonce(0) == 3 + n - 1


def test_jumbo_16mib_roundtrip(torch_cuda, C):
    """Config 5 frame size (16 MiB), 2 frames: bit-exact vs oracle."""
    torch = torch_cuda
    rng = np.random.default_rng(15)
    P = 16 << 20
    precom = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    ctx = C.CurveContext(0, 1)
    ctx.session_set(0, precom, O.CLIENT_PREFIX, O.SERVER_PREFIX)
    inp = rng.integers(0, 256, 2 * P, dtype=np.uint8)
    b = dict(sid=np.zeros(2, np.uint32), nonce=np.array([3, 4], np.uint64), flags=np.array([0, 1], np.uint8),
             in_off=np.array([0, P], np.uint64), lens=np.full(2, P, np.uint32), inp=inp)
    W = P + 33
    out_off = np.array([0, W + 3], np.uint64)
    gpu = gpu_encode(torch, ctx, b, out_off, 2 * W + 3)
    ref = O.encode_batch(O.make_sessions([precom]), b["sid"], b["nonce"], b["flags"], b["in_off"], b["lens"], inp,
                         out_off, 2 * W + 3)
    assert np.array_equal(gpu, ref)


# ------------------------------------------------------------------ failures
def test_tamper_every_region(torch_cuda, C):
    torch = torch_cuda
    rng = np.random.default_rng(20)
    precom = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    enc = C.CurveContext(0, 1)
    enc.session_set(0, precom, O.CLIENT_PREFIX, O.SERVER_PREFIX)
    n, P = 64, 3000
    inp = rng.integers(0, 256, n * P, dtype=np.uint8)
    b = dict(sid=np.zeros(n, np.uint32), nonce=np.arange(3, 3 + n, dtype=np.uint64), flags=np.zeros(n, np.uint8),
             in_off=np.arange(n, dtype=np.uint64) * P, lens=np.full(n, P, np.uint32), inp=inp)
    W = P + 33
    out_off = np.arange(n, dtype=np.uint64) * W
    wire = gpu_encode(torch, enc, b, out_off, n * W).copy()
    # flip one bit in frames 1, 5, 9, ... at positions across tag/ciphertext
    bad = list(range(1, n, 4))
    for k, i in enumerate(bad):
        pos = [16, 31, 32, 33, 63, 64, 100, 1000, W - 1, W - 2, 2000, 300, 17, 48, 95, 96][k % 16]
        wire[int(out_off[i]) + pos] ^= 1 << (k % 8)
    dec = C.CurveContext(0, 1)
    dec.session_set(0, precom, O.SERVER_PREFIX, O.CLIENT_PREFIX, False, 2)
    pl, fl, st = gpu_decode(torch, dec, np.zeros(n, np.uint32), out_off, np.full(n, W, np.uint32), wire,
                            b["in_off"], n * P, fill=0x5A)
    sess = O.make_sessions([precom], dec_prefix=O.CLIENT_PREFIX)
    peer = np.array([2], np.uint64)
    rpl, rfl, rst = O.decode_batch(sess, peer, np.zeros(n, np.uint32), out_off, np.full(n, W, np.uint32), wire,
                                   b["in_off"], n * P)
    assert np.array_equal(st, rst)
    assert set(np.nonzero(st)[0].tolist()) == set(bad)
    assert (st[bad] == C.ERR_CRYPTOGRAPHIC).all()
    for i in range(n):
        seg = pl[i * P:(i + 1) * P]
        if i in bad:
            assert not seg.any()
        else:
            assert np.array_equal(seg, inp[i * P:(i + 1) * P])
    assert dec.get_peer_nonce(0) == int(peer[0])


def test_replay_interleaved_sessions(torch_cuda, C):
    """Replays, reorders and MAC failures across 6 interleaved sessions: the
    per-frame statuses and final peer nonces equal the reference's
    sequential rule (oracle)."""
    torch = torch_cuda
    rng = np.random.default_rng(21)
    S = 6
    precoms = [rng.integers(0, 256, 32, dtype=np.uint8).tobytes() for _ in range(S)]
    enc = C.CurveContext(0, S)
    for s in range(S):
        enc.session_set(s, precoms[s], O.CLIENT_PREFIX, O.SERVER_PREFIX)
    b = random_batch(rng, 300, [0, 5, 40, 100, 300], S)
    out_off, wl, total = wire_layout(b["flags"], b["lens"], [False] * S, b["sid"])
    wire = gpu_encode(torch, enc, b, out_off, total)
    frames = [wire[int(out_off[i]):int(out_off[i]) + int(wl[i])].tobytes() for i in range(300)]
    sids = list(b["sid"])
    # build an adversarial stream: duplicates, swaps, tampering
    stream, ssid = [], []
    for i in range(300):
        stream.append(frames[i])
        ssid.append(sids[i])
        r = rng.random()
        if r < 0.1:  # replay an earlier frame of any session
            j = int(rng.integers(0, i + 1))
            stream.append(frames[j])
            ssid.append(sids[j])
        elif r < 0.15:  # tampered copy of a future frame
            j = min(299, i + int(rng.integers(1, 5)))
            f = bytearray(frames[j])
            f[-1] ^= 0x40
            stream.append(bytes(f))
            ssid.append(sids[j])
    inp, in_off = pack(stream, rng, 5)
    wls = np.array([len(f) for f in stream], np.uint32)
    plen = wls.astype(np.int64) - 33
    _, pout = pack([b"\0" * int(p) for p in plen])
    psize = int(pout[-1]) + int(plen[-1]) + 1
    dec = C.CurveContext(0, S)
    for s in range(S):
        dec.session_set(s, precoms[s], O.SERVER_PREFIX, O.CLIENT_PREFIX, False, 2)
    pl, fl, st = gpu_decode(torch, dec, ssid, in_off, wls, inp, pout, psize)
    sess = np.concatenate([O.make_sessions([p], dec_prefix=O.CLIENT_PREFIX) for p in precoms])
    peer = np.full(S, 2, np.uint64)
    rpl, rfl, rst = O.decode_batch(sess, peer, ssid, in_off, wls, inp, pout, psize)
    assert np.array_equal(st, rst)
    assert (st == C.ERR_INVALID_SEQUENCE).any() and (st == C.ERR_CRYPTOGRAPHIC).any()
    assert np.array_equal(fl, rfl)
    assert np.array_equal(pl, rpl)
    for s in range(S):
        assert dec.get_peer_nonce(s) == int(peer[s])


# ------------------------------------------------------------------ reference unit test, restated
def _unit_roundtrip(C, data, flags=0):
    """unittests/unittest_curve_encoding.cpp:26-71 with GPU-backed encodings."""
    rng = np.random.default_rng(len(data) + flags)
    precom = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()  # = crypto_box_beforenm output
    client = C.CurveEncoding(C.CLIENT_PREFIX, C.SERVER_PREFIX, False)
    server = C.CurveEncoding(C.SERVER_PREFIX, C.CLIENT_PREFIX, False)
    client.get_writable_precom_buffer()[:] = precom
    server.get_writable_precom_buffer()[:] = precom
    msg = C.Msg(data, flags)
    assert client.encode(msg) == 0
    server.set_peer_nonce(0)
    rc, code = server.decode(msg)
    assert rc == 0, hex(code)
    assert msg.data == bytes(data)
    return msg


def test_unit_roundtrip_empty(torch_cuda, C):
    _unit_roundtrip(C, b"")


def test_unit_roundtrip_small(torch_cuda, C):
    _unit_roundtrip(C, b"0123456789ABCDEF0123456789ABCDEF")


def test_unit_roundtrip_large(torch_cuda, C):
    _unit_roundtrip(C, b"0123456789ABCDEF0123456789ABCDEF" * 64)


def test_unit_roundtrip_empty_more(torch_cuda, C):
    msg = _unit_roundtrip(C, b"", C.MORE)
    assert msg.flags & C.MORE


def test_host_path_matches_device_path(torch_cuda, C):
    rng = np.random.default_rng(30)
    precom = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    ctx = C.CurveContext(0, 1)
    ctx.session_set(0, precom, O.CLIENT_PREFIX, O.SERVER_PREFIX)
    b = random_batch(rng, 50, [0, 1, 33, 500, 4000], 1, (0, 1, 12))
    out_off, wl, total = wire_layout(b["flags"], b["lens"], [False], b["sid"])
    a = ctx.encode_host(b["sid"], b["nonce"], b["flags"], b["in_off"], b["lens"], b["inp"], out_off, total)
    d = gpu_encode(torch_cuda, ctx, b, out_off, total)
    assert np.array_equal(a, d)


@pytest.mark.parametrize("n,sizes", [(3000, [0, 7, 64, 200, 1024, 6000]), (40000, [0, 9, 100]),
                                     (140000, [1, 30])])
def test_replay_single_session_lookback(torch_cuda, C, n, sizes):
    """One session: the replay rule runs inside the frame kernel (decoupled
    look-back over workgroup tickets) and in the body finisher for frames
    above the frame kernel's limit.  Duplicates, reorders, header and MAC
    failures scattered over many workgroups (G = 4, 2 and 1 lanes per frame
    at these batch sizes): statuses, flags, payloads and the new peer nonce
    equal the reference's sequential rule (oracle)."""
    torch = torch_cuda
    rng = np.random.default_rng(n)
    precom = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    enc = C.CurveContext(0, 1)
    enc.session_set(0, precom, O.CLIENT_PREFIX, O.SERVER_PREFIX)
    m = n - n // 20
    b = random_batch(rng, m, sizes, 1)
    out_off, wl, total = wire_layout(b["flags"], b["lens"], [False], b["sid"])
    wire = gpu_encode(torch, enc, b, out_off, total)
    frames = [wire[int(out_off[i]):int(out_off[i]) + int(wl[i])].tobytes() for i in range(m)]
    stream = []
    for i in range(m):
        r = rng.random()
        if r < 0.02 and stream:  # replay an earlier frame
            stream.append(stream[int(rng.integers(0, len(stream)))])
        elif r < 0.03:  # swap with the next frame (the later one arrives first)
            if i + 1 < m:
                stream.append(frames[i + 1])
        elif r < 0.04:  # tampered ciphertext
            f = bytearray(frames[i])
            f[-1] ^= 0x01
            stream.append(bytes(f))
        elif r < 0.045:  # not a MESSAGE command
            f = bytearray(frames[i])
            f[3] ^= 0x20
            stream.append(bytes(f))
        stream.append(frames[i])
    stream = stream[:n]
    inp, in_off = pack(stream, rng, 3)
    wls = np.array([len(f) for f in stream], np.uint32)
    plen = np.maximum(wls.astype(np.int64) - 33, 0)
    _, pout = pack([b"\0" * int(p) for p in plen])
    psize = int(pout[-1]) + int(plen[-1]) + 1
    dec = C.CurveContext(0, 1)
    dec.session_set(0, precom, O.SERVER_PREFIX, O.CLIENT_PREFIX, False, 2)
    sid = np.zeros(len(stream), np.uint32)
    pl, fl, st = gpu_decode(torch, dec, sid, in_off, wls, inp, pout, psize)
    peer = np.array([2], np.uint64)
    rpl, rfl, rst = O.decode_batch(O.make_sessions([precom], dec_prefix=O.CLIENT_PREFIX), peer, sid, in_off, wls,
                                   inp, pout, psize)
    assert (rst == C.ERR_INVALID_SEQUENCE).any() and (rst == C.ERR_CRYPTOGRAPHIC).any()
    assert np.array_equal(st, rst)
    assert np.array_equal(fl, rfl)
    assert np.array_equal(pl, rpl)
    assert dec.get_peer_nonce(0) == int(peer[0])
    # a second batch on the same context continues from the new peer nonce
    pl2, fl2, st2 = gpu_decode(torch, dec, sid[:50], in_off[:50], wls[:50], inp, pout[:50], psize)
    assert (st2 != 0).all() and (st2 == C.ERR_INVALID_SEQUENCE).sum() >= 40
