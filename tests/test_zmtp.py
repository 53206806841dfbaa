"""ZMTP framing on the device: zmqg_encode_zmtp /
zmqg_decode_zmtp against oracle/zmtp_oracle.py (the reference's ZMTP encoder
and decoder loop, src/v3_1_encoder.cpp:23-60, src/v2_decoder.cpp:35-140)
combined with the CURVE oracle.  Cases follow the decoder's branches: short
and LARGE sizes (the 255-byte boundary, LARGE with a small size), EMSGSIZE,
incomplete header / body at the buffer end, a non-MESSAGE frame, planted
"\\x07MESSAGE" signatures inside bodies, max_frames, random bytes seeded with frame-like
candidates (alone and behind valid frames)."""
import struct
import zlib

import numpy as np
import pytest

from oracle import oracle as O
from oracle import zmtp_oracle as Z
from tests.helpers import random_batch, wire_layout


def test_oracle_frame_boundary():
    assert Z.frame(b"\x07MESSAGE" + bytes(247)) [:2] == b"\x00\xff"
    f = Z.frame(b"\x07MESSAGE" + bytes(248))
    assert f[0] == Z.LARGE and struct.unpack(">Q", f[1:9])[0] == 256


def test_oracle_parse_branches():
    body = b"\x07MESSAGE" + bytes(30)
    s = Z.frame(body) + bytes([Z.LARGE]) + struct.pack(">Q", len(body)) + body  # LARGE with a small size
    r = Z.parse(s)
    assert [f[2] for f in r["frames"]] == [38, 38] and r["consumed"] == len(s) and r["error"] == 0
    assert Z.parse(s[:-1])["consumed"] == 40  # incomplete body
    assert Z.parse(s + b"\x02\x00\x00")["consumed"] == len(s)  # incomplete LARGE header
    r = Z.parse(s, max_msg_size=37)
    assert r["frames"] == [] and r["error"] == Z.EMSGSIZE
    ping = Z.frame(b"\x04PING\x00\x00")
    r = Z.parse(ping + s)
    assert len(r["frames"]) == 1 and r["consumed"] == len(ping)  # the mechanism rejects it: stop
    assert len(Z.parse(s, max_frames=1)["frames"]) == 1


@pytest.mark.gpu
def test_encode_zmtp_matches_oracle(torch_cuda, C):
    torch = torch_cuda
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(2)
    n, S = 1500, 4
    precoms = [rng.integers(0, 256, 32, dtype=np.uint8).tobytes() for _ in range(S)]
    downgrade = [False, True, False, False]
    b = random_batch(rng, n, [0, 1, 100, 221, 222, 223, 250, 300, 1024, 5000, 70000], S,
                     flag_choices=(0, 1, 2, 3, 12, 16))
    ctx = C.CurveContext(0, S)
    for s in range(S):
        ctx.session_set(s, precoms[s], C.CLIENT_PREFIX, C.SERVER_PREFIX, downgrade[s])
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a).view(dt)).to(dev)
    wires = [O.wire_size(int(f), downgrade[int(s)], int(l)) for f, s, l in zip(b["flags"], b["sid"], b["lens"])]
    total = sum(w + (9 if w > 255 else 2) for w in wires)
    out = torch.full((total + 64,), 0xEE, dtype=torch.uint8, device=dev)
    foff = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    ctx.encode_zmtp(t(b["sid"], np.int32), t(b["nonce"], np.int64), t(b["flags"], np.uint8), t(b["in_off"], np.int64),
                    t(b["lens"], np.int32), t(b["inp"], np.uint8), out, foff)
    torch.cuda.synchronize()
    got, fo = out.cpu().numpy(), foff.cpu().numpy()
    assert int(fo[n]) == total and (got[total:] == 0xEE).all()
    sessions = np.concatenate([O.make_sessions([p], downgrade_sub=d) for p, d in zip(precoms, downgrade)])
    out_off, wl, wtotal = wire_layout(b["flags"], b["lens"], downgrade, b["sid"])
    ref_wire = O.encode_batch(sessions, b["sid"], b["nonce"], b["flags"], b["in_off"], b["lens"], b["inp"], out_off,
                              wtotal)
    ref = b"".join(Z.frame(ref_wire[int(out_off[i]):int(out_off[i]) + int(wl[i])]) for i in range(n))
    assert got[:total].tobytes() == ref
    pos = 0
    for i in range(n):
        assert int(fo[i]) == pos
        pos += int(wl[i]) + (9 if wl[i] > 255 else 2)


def _stream_case(rng, case, precom, n=400):
    """A received byte stream of one connection and the decoder settings."""
    if case == "sparse":  # large frames: most 16 KiB scan lists hold no candidate
        n = 60
        b = random_batch(rng, n, [100, 40000, 70000], 1, flag_choices=(0, 1, 2))
    else:
        b = random_batch(rng, n, [0, 5, 100, 222, 223, 1024, 3000], 1, flag_choices=(0, 1, 2))
    sessions = O.make_sessions([precom])
    out_off, wl, wtotal = wire_layout(b["flags"], b["lens"], [False], b["sid"])
    wire = O.encode_batch(sessions, b["sid"], b["nonce"], b["flags"], b["in_off"], b["lens"], b["inp"], out_off, wtotal)
    bodies = [bytearray(wire[int(out_off[i]):int(out_off[i]) + int(wl[i])].tobytes()) for i in range(n)]
    frames = []
    max_msg, max_frames = -1, 1000  # the arrays below hold max_frames entries (include/zmqg_curve.h)
    for i, body in enumerate(bodies):
        if case == "planted" and rng.random() < 0.2 and len(body) > 60:
            # a frame-like header and the MESSAGE signature inside the ciphertext
            k = int(rng.integers(33, len(body) - 20))
            fake = bytes([0, int(rng.integers(8, 40))]) + b"\x07MESSAGE"
            body[k:k + len(fake)] = fake
        if case == "flood" and rng.random() < 0.3 and len(body) > 100:
            # a frame-like header + signature every 16 bytes of the ciphertext
            pat = (b"\x00\x10\x07MESSAGE" + bytes(6)) * ((len(body) - 49) // 16)
            body[33:33 + len(pat)] = pat
        if case == "large_small" and rng.random() < 0.3 and len(body) <= 255:
            frames.append(bytes([Z.LARGE]) + struct.pack(">Q", len(body)) + bytes(body))
            continue
        frames.append(Z.frame(body))
    if case == "ping":
        frames.insert(n // 2, Z.frame(b"\x04PING\x00\x00\x00"))
    stream = b"".join(frames)
    if case == "truncated":
        stream = stream[:int(rng.integers(len(stream) // 2, len(stream) - 1))]
    if case in ("garbage", "garbage_tail"):
        # random bytes (alone, or after the valid frames) seeded with
        # frame-like headers + signatures: candidates the walk must not take
        junk = bytearray(rng.bytes(40000))
        for k in rng.integers(0, len(junk) - 20, 200):
            junk[k:k + 11] = bytes([0, int(rng.integers(8, 64))]) + b"\x07MESSAGE" + b"\x00"
        stream = bytes(junk) if case == "garbage" else stream + bytes(junk)
    if case == "emsgsize":
        max_msg = 2000
    if case == "max_frames":
        max_frames = 123
    if case == "zmtp_flags":
        # MORE / COMMAND bits on some frame headers (the decoder passes them on)
        stream = bytearray(stream)
        pos = 0
        for f in frames:
            if rng.random() < 0.3:
                stream[pos] |= int(rng.choice([Z.MORE, Z.COMMAND, Z.MORE | Z.COMMAND]))
            pos += len(f)
        stream = bytes(stream)
    return stream, max_msg, max_frames


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["clean", "truncated", "planted", "flood", "large_small", "ping", "emsgsize",
                                  "max_frames", "zmtp_flags", "sparse", "planted+cub", "sparse+cub",
                                  "zmtp_flags+g0", "zmtp_flags+g8", "ping+g0", "ping+g8", "garbage",
                                  "garbage_tail"])
def test_decode_zmtp_matches_oracle(torch_cuda, C, case, monkeypatch):
    """+cub: the candidate counts scanned by hipCUB (the form for streams above
    128 MiB, ZMQG_ZMTP_CUB forces it).  +g0 / +g8: the decode's frame kernel
    forced to the one-lane-per-frame forms (k_frames_seq / k_frames_lds;
    these small streams otherwise take k_frames<4>), which OR the ZMTP flag
    bits and copy the call's result themselves."""
    torch = torch_cuda
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(zlib.crc32(case.encode()))
    if case.endswith("+cub"):
        monkeypatch.setenv("ZMQG_ZMTP_CUB", "1")
        case = case[:-4]
    elif case[-3:] in ("+g0", "+g8"):
        monkeypatch.setenv("ZMQG_FRAMES_G", case[-1])
        case = case[:-3]
    precom = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    stream, max_msg, max_frames = _stream_case(rng, case, precom)
    ref = Z.parse(stream, max_msg, max_frames)
    # CURVE decode of the frames the decoder produced, in order (peer nonce 2)
    fr = ref["frames"]
    nf = len(fr)
    f_off = np.array([f[1] for f in fr], np.uint64)
    f_len = np.array([f[2] for f in fr], np.uint32)
    plen = np.maximum(f_len.astype(np.int64) - 33, 0)
    p_off = np.concatenate([[0], np.cumsum(plen)[:-1]]).astype(np.uint64) if nf else np.zeros(0, np.uint64)
    dec = O.make_sessions([precom], dec_prefix=O.CLIENT_PREFIX)
    inp = np.frombuffer(stream, np.uint8)
    pl, fl, st = O.decode_batch(dec, np.array([2], np.uint64), np.zeros(nf, np.uint32), f_off, f_len, inp, p_off,
                                int(plen.sum()))
    fl = np.array([int(fl[i]) | (Z.msg_flags(fr[i][0]) if st[i] == 0 else 0) for i in range(nf)], np.uint8)

    ctx = C.CurveContext(0, 1)
    ctx.session_set(0, precom, C.SERVER_PREFIX, C.CLIENT_PREFIX, False, 2)
    cap = 1000
    d_in = torch.from_numpy(inp.copy()).to(dev)
    d_foff = torch.zeros(cap, dtype=torch.int64, device=dev)
    d_flen = torch.zeros(cap, dtype=torch.int32, device=dev)
    d_poff = torch.zeros(cap, dtype=torch.int64, device=dev)
    d_out = torch.full((len(stream) + 1,), 0x77, dtype=torch.uint8, device=dev)
    d_fl = torch.zeros(cap, dtype=torch.uint8, device=dev)
    d_st = torch.full((cap,), -1, dtype=torch.int32, device=dev)
    if case == "clean":  # the asynchronous form, result read once the stream is done
        res = torch.zeros(4, dtype=torch.int64, device=dev)
        ctx.decode_zmtp_async(0, d_in, len(stream), max_msg, max_frames, d_foff, d_flen, d_poff, d_out, d_fl, d_st,
                              res)
        torch.cuda.synchronize()
        r = ctx.zmtp_result(res)
    else:
        r = ctx.decode_zmtp(0, d_in, len(stream), max_msg, max_frames, d_foff, d_flen, d_poff, d_out, d_fl, d_st)
    assert r["frames"] == nf and r["consumed"] == ref["consumed"] and r["error"] == ref["error"], (r, ref["consumed"])
    assert r["out_bytes"] == int(plen.sum())
    assert (d_foff[:nf].cpu().numpy().view(np.uint64) == f_off).all()
    assert (d_flen[:nf].cpu().numpy().view(np.uint32) == f_len).all()
    # each payload is written at its body's offset (include/zmqg_curve.h)
    assert (d_poff[:nf].cpu().numpy().view(np.uint64) == f_off).all()
    got_st = d_st[:nf].cpu().numpy()
    if not (got_st == st).all():  # diagnostics for a rare first-run mismatch seen on fresh boxes
        bad = np.nonzero(got_st != st)[0]
        d_st2 = torch.full((cap,), -1, dtype=torch.int32, device=dev)
        ctx2 = C.CurveContext(0, 1)
        ctx2.session_set(0, precom, C.SERVER_PREFIX, C.CLIENT_PREFIX, False, 2)
        ctx2.decode_zmtp(0, d_in, len(stream), max_msg, max_frames, d_foff, d_flen, d_poff, d_out, d_fl, d_st2)
        again = d_st2[:nf].cpu().numpy()
        print("status mismatch at", bad[:16].tolist(), "lens", f_len[bad[:16]].tolist(), "got",
              [hex(int(x)) for x in got_st[bad[:4]]], "expected", st[bad[:4]].tolist(),
              "descriptors ok", bool((d_foff[:nf].cpu().numpy().view(np.uint64) == f_off).all()),
              "re-run mismatches", int((again != st).sum()))
    assert (got_st == st).all()
    assert (d_fl[:nf].cpu().numpy() == fl).all()
    got = d_out.cpu().numpy()
    for i in range(nf):
        a, p0, ln = int(f_off[i]), int(p_off[i]), int(plen[i])
        assert got[a:a + ln].tobytes() == pl[p0:p0 + ln].tobytes(), i
    if case == "clean":  # in place: out = in, every payload left at its body's start
        d_st3 = torch.full((cap,), -1, dtype=torch.int32, device=dev)
        ctx3 = C.CurveContext(0, 1)
        ctx3.session_set(0, precom, C.SERVER_PREFIX, C.CLIENT_PREFIX, False, 2)
        r3 = ctx3.decode_zmtp(0, d_in, len(stream), max_msg, max_frames, d_foff, d_flen, d_poff, d_in, d_fl, d_st3)
        assert r3["frames"] == nf and (d_st3[:nf].cpu().numpy() == st).all()
        got = d_in.cpu().numpy()
        for i in range(nf):
            a, p0, ln = int(f_off[i]), int(p_off[i]), int(plen[i])
            assert got[a:a + ln].tobytes() == pl[p0:p0 + ln].tobytes(), i
    if case in ("clean", "large_small", "zmtp_flags", "sparse"):
        assert (st == 0).all() and ref["consumed"] == len(stream)
    if case in ("planted", "flood"):
        assert (st == C.ERR_CRYPTOGRAPHIC).any() and ref["consumed"] == len(stream)
    if case == "ping":
        assert st[-1] != 0 and (st[:-1] == 0).all()
    if case == "emsgsize":
        assert ref["error"] == Z.EMSGSIZE


@pytest.mark.gpu
def test_zmtp_round_trip_config2(torch_cuda, C):
    """BASELINE config 2's shape (65,536 x 1 KiB, one session) through the
    framed path, checked by size-independent properties: encode_zmtp then
    decode_zmtp returns every payload, flag and frame offset; a ciphertext
    byte flipped in three frames fails exactly those three; a stream cut
    inside the last frame stops the parse before it.  The oracle checks the
    first frames' bytes."""
    torch = torch_cuda
    dev = torch.device("cuda", 0)
    n, P = 65536, 1024
    W, F = P + 33, P + 33 + 9
    rng = np.random.default_rng(11)
    precom = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    inp = torch.randint(0, 256, (n * P,), dtype=torch.uint8, device=dev, generator=g)
    sid = torch.zeros(n, dtype=torch.int32, device=dev)
    nonce = torch.arange(3, 3 + n, dtype=torch.int64, device=dev)
    flags = torch.zeros(n, dtype=torch.uint8, device=dev)
    in_off = torch.arange(n, dtype=torch.int64, device=dev) * P
    lens = torch.full((n,), P, dtype=torch.int32, device=dev)
    enc = C.CurveContext(0, 1)
    enc.session_set(0, precom, C.CLIENT_PREFIX, C.SERVER_PREFIX)
    stream = torch.empty(n * F + 64, dtype=torch.uint8, device=dev)
    foff = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    enc.encode_zmtp(sid, nonce, flags, in_off, lens, inp, stream, foff)
    torch.cuda.synchronize()
    assert int(foff[n]) == n * F
    assert torch.equal(foff[:n], torch.arange(n, dtype=torch.int64, device=dev) * F)
    # the first frames against the oracle
    k = 8
    h = inp[:k * P].cpu().numpy()
    sessions = O.make_sessions([precom])
    ref = O.encode_batch(sessions, np.zeros(k, np.uint32), np.arange(3, 3 + k, dtype=np.uint64), np.zeros(k, np.uint8),
                         np.arange(k, dtype=np.uint64) * P, np.full(k, P, np.uint32), h,
                         np.arange(k, dtype=np.uint64) * W, k * W)
    want = b"".join(Z.frame(ref[i * W:(i + 1) * W]) for i in range(k))
    assert stream[:k * F].cpu().numpy().tobytes() == want

    def decode(buf, nbytes):
        dec = C.CurveContext(0, 1)
        dec.session_set(0, precom, C.SERVER_PREFIX, C.CLIENT_PREFIX, False, 2)
        d = dict(fo=torch.zeros(n, dtype=torch.int64, device=dev), fl=torch.zeros(n, dtype=torch.int32, device=dev),
                 po=torch.zeros(n, dtype=torch.int64, device=dev), out=torch.empty(n * F, dtype=torch.uint8, device=dev),
                 mf=torch.zeros(n, dtype=torch.uint8, device=dev), st=torch.full((n,), -1, dtype=torch.int32, device=dev))
        r = dec.decode_zmtp(0, buf, nbytes, W, n, d["fo"], d["fl"], d["po"], d["out"], d["mf"], d["st"])
        dec.close()
        return r, d

    body = torch.arange(n, dtype=torch.int64, device=dev) * F + 9
    r, d = decode(stream, n * F)
    assert r == dict(frames=n, consumed=n * F, out_bytes=n * P, error=0)
    assert torch.equal(d["fo"], body) and torch.equal(d["po"], body)
    assert bool((d["fl"] == W).all()) and bool((d["st"] == 0).all()) and bool((d["mf"] == 0).all())
    got = d["out"].view(n, F)[:, 9:9 + P].reshape(-1)
    assert torch.equal(got, inp)
    # tampering: one ciphertext byte in three frames
    bad = [0, 12345, n - 1]
    t2 = stream.clone()
    for i in bad:
        t2[i * F + 9 + 33 + 100] ^= 0x40
    r, d = decode(t2, n * F)
    assert r["frames"] == n and r["consumed"] == n * F
    st = d["st"].cpu().numpy()
    assert (np.nonzero(st)[0] == bad).all() and (st[bad] == C.ERR_CRYPTOGRAPHIC).all()
    # a stream cut inside the last frame: n - 1 frames, the rest left for later
    r, d = decode(stream, n * F - 100)
    assert r == dict(frames=n - 1, consumed=(n - 1) * F, out_bytes=(n - 1) * P, error=0)
    assert bool((d["st"][:n - 1] == 0).all())
    enc.close()
