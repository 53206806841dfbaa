"""ZMQG_OPT_VERIFY_FIRST (include/zmqg_curve.h): decode writes `out` only
after each frame's verdict, as libsodium's crypto_box_open_easy_afternm
verifies before it decrypts (src/curve_mechanism_base.cpp:226-228).

* Same results as the plain decode (statuses, flags, payloads, peer nonces)
  on batches with MAC, header and replay failures, frames on both sides of
  the frame kernel's 4.5 KiB range, separate and in-place layouts.
* A second thread reading a pinned host `out` while forged batches are
  decoded never sees a plaintext byte.
* out_bytes = 0 is a valid extent for frames without payload bytes (each
  gets its own status); a frame whose payload region would end past
  out_bytes fails with ZMQG_ERR_BOUND and nothing of it is written."""
import threading

import numpy as np
import pytest

from oracle import oracle as O
from tests.helpers import pack
from tests.test_gpu_parity import dev, host

pytestmark = pytest.mark.gpu


def _batch(rng, sizes, precom, tamper_every=5):
    n = len(sizes)
    payloads = [rng.integers(0, 256, s, dtype=np.uint8).tobytes() for s in sizes]
    inp, in_off = pack(payloads)
    nonce = np.arange(3, 3 + n, dtype=np.uint64)
    nonce[n // 2] = nonce[1]  # a replay
    flags = (np.arange(n) % 3 == 0).astype(np.uint8)
    wl = np.array([s + 33 for s in sizes], np.uint32)
    wire_off = np.concatenate([[0], np.cumsum(wl)[:-1]]).astype(np.uint64)
    sess = O.make_sessions([precom])
    wire = O.encode_batch(sess, np.zeros(n, np.uint32), nonce, flags, in_off, np.array(sizes, np.uint32), inp,
                          wire_off, int(wl.sum()))
    for i in range(0, n, tamper_every):  # MAC failures
        wire[wire_off[i] + 32 + (sizes[i] // 2)] ^= 0x40
    wire[wire_off[n - 2] + 1] ^= 0x20  # broken command name
    return wire, wire_off, wl, in_off


@pytest.mark.parametrize("layout", ["separate", "inplace33", "inplace0"])
def test_verify_first_matches_plain_decode(torch_cuda, C, layout):
    torch = torch_cuda
    rng = np.random.default_rng(90)
    precom = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    sizes = [int(x) for x in rng.choice([0, 1, 31, 200, 1024, 4000, 4600, 9000, 70000], 240)]
    wire, wire_off, wl, pay_off = _batch(rng, sizes, precom)
    n = len(sizes)
    results = []
    for vf in (False, True):
        dec = C.CurveContext(0, 1)
        dec.session_set(0, precom, O.SERVER_PREFIX, O.CLIENT_PREFIX, False, 2)
        d_wire = dev(torch, wire)
        if layout == "separate":
            out = torch.full((int(pay_off[-1]) + sizes[-1] + 64,), 0x77, dtype=torch.uint8, device="cuda")
            out_off = pay_off
        else:
            out = d_wire
            out_off = wire_off + (33 if layout == "inplace33" else 0)
        fl = torch.zeros(n, dtype=torch.uint8, device="cuda")
        st = torch.zeros(n, dtype=torch.int32, device="cuda")
        dec.decode_batch(dev(torch, np.zeros(n, np.uint32)), dev(torch, wire_off), dev(torch, wl), d_wire,
                         dev(torch, out_off), out, fl, st, verify_first=vf)
        torch.cuda.synchronize()
        results.append((host(out, np.uint8).copy(), host(fl, np.uint8), host(st, np.int32), dec.get_peer_nonce(0),
                        out_off))
    (o0, f0, s0, p0, off), (o1, f1, s1, p1, _) = results
    assert (s0 != 0).sum() > n // 5
    assert np.array_equal(s0, s1) and np.array_equal(f0, f1) and p0 == p1
    for i in range(n):  # every payload region: the verified payload or zeros
        a, b = int(off[i]), int(off[i]) + sizes[i]
        if layout == "inplace0" and s0[i] != 0 and sizes[i] + 33 > 4608:
            continue  # (plain decode zeroes that frame's whole wire region; verify-first its payload region)
        assert np.array_equal(o0[a:b], o1[a:b]), (i, sizes[i], int(s0[i]))


def test_reader_thread_never_sees_forged_plaintext(torch_cuda, C):
    torch = torch_cuda
    rng = np.random.default_rng(91)
    precom = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    n, P = 16384, 1024
    inp = np.full(n * P, 0xA5, np.uint8)  # a plaintext byte the reader can recognise
    in_off = np.arange(n, dtype=np.uint64) * P
    W = P + 33
    wire_off = np.arange(n, dtype=np.uint64) * W
    sess = O.make_sessions([precom])
    wire = O.encode_batch(sess, np.zeros(n, np.uint32), np.arange(3, 3 + n, dtype=np.uint64), np.zeros(n, np.uint8),
                          in_off, np.full(n, P, np.uint32), inp, wire_off, n * W)
    wire[wire_off + 20] ^= 1  # every tag forged
    dec = C.CurveContext(0, 1)
    dec.session_set(0, precom, O.SERVER_PREFIX, O.CLIENT_PREFIX, False, 2)
    out = torch.zeros(n * P, dtype=torch.uint8).pin_memory()  # host memory the kernels write over PCIe
    view = out.numpy()
    d = [dev(torch, a) for a in (np.zeros(n, np.uint32), wire_off, np.full(n, W, np.uint32), wire, in_off)]
    fl = torch.zeros(n, dtype=torch.uint8, device="cuda")
    st = torch.zeros(n, dtype=torch.int32, device="cuda")

    def run(vf, reps=30):
        seen = [0, 0]
        stop = threading.Event()

        def reader():
            r = np.random.default_rng(5)
            while not stop.is_set():
                idx = r.integers(0, n * P, 4096)
                seen[0] += int((view[idx] == 0xA5).sum())
                seen[1] += 1

        th = threading.Thread(target=reader)
        th.start()
        try:
            for _ in range(reps):
                dec.set_peer_nonce(0, 2)  # (each rep fails on its MACs, not as replays of the last)
                dec.decode_batch(d[0], d[1], d[2], d[3], d[4], out, fl, st, verify_first=vf)
                torch.cuda.synchronize()
        finally:
            stop.set()
            th.join()
        assert (host(st, np.int32) == 0x11000001).all()  # ZMQ_PROTOCOL_ERROR_ZMTP_CRYPTOGRAPHIC
        assert not (view == 0xA5).any()  # zero-filled at completion either way
        return seen

    exposed_plain = run(False)
    exposed_vf = run(True)
    print(f"plain decode: {exposed_plain[0]} plaintext bytes seen in {exposed_plain[1]} samples; "
          f"verify-first: {exposed_vf[0]} in {exposed_vf[1]}")
    assert exposed_vf[1] > 10
    assert exposed_vf[0] == 0


def test_verify_first_extent_checks(torch_cuda, C):
    torch = torch_cuda
    rng = np.random.default_rng(91)
    precom = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    # (a) no payload bytes at all: out_bytes = 0 -- a valid empty message, a
    # frame cut below the MESSAGE minimum, an empty frame
    n = 3
    wl = np.full(n, 33, np.uint32)
    wire_off = np.arange(n, dtype=np.uint64) * 33
    wire = O.encode_batch(O.make_sessions([precom]), np.zeros(n, np.uint32), np.arange(3, 3 + n, dtype=np.uint64),
                          np.zeros(n, np.uint8), np.zeros(n, np.uint64), np.zeros(n, np.uint32),
                          np.zeros(1, np.uint8), wire_off, 33 * n)
    wl[1] = 20  # shorter than a MESSAGE
    wl[2] = 0   # empty
    dec = C.CurveContext(0, 1)
    dec.session_set(0, precom, O.SERVER_PREFIX, O.CLIENT_PREFIX, False, 2)
    out = torch.full((16,), 0x77, dtype=torch.uint8, device="cuda")
    fl = torch.zeros(3, dtype=torch.uint8, device="cuda")
    st = torch.zeros(3, dtype=torch.int32, device="cuda")
    dec.decode_batch(dev(torch, np.zeros(3, np.uint32)), dev(torch, wire_off), dev(torch, wl), dev(torch, wire),
                     dev(torch, np.zeros(3, np.uint64)), out, fl, st, verify_first=True, out_bytes=0)
    torch.cuda.synchronize()
    stt = host(st, np.int32)
    assert stt[0] == 0 and stt[1] == C.ERR_MALFORMED_MESSAGE and stt[2] == C.ERR_MALFORMED_UNSPECIFIED
    assert bool((host(out, np.uint8) == 0x77).all())
    # (b) an understated extent: the frames past it fail with ZMQG_ERR_BOUND, untouched
    sizes = [100, 3000, 100, 9000]
    wire, wire_off, wl, pay_off = _batch(rng, sizes, precom, tamper_every=100)
    wire = wire.copy()  # (_batch tampers frame 0's ciphertext and frame 2's name: undo both)
    wire[wire_off[0] + 32 + sizes[0] // 2] ^= 0x40
    wire[wire_off[2] + 1] ^= 0x20
    n = len(sizes)
    dec = C.CurveContext(0, 1)
    dec.session_set(0, precom, O.SERVER_PREFIX, O.CLIENT_PREFIX, False, 2)
    total = int(pay_off[-1]) + sizes[-1]
    out = torch.full((total + 64,), 0x77, dtype=torch.uint8, device="cuda")
    fl = torch.zeros(n, dtype=torch.uint8, device="cuda")
    st = torch.zeros(n, dtype=torch.int32, device="cuda")
    limit = int(pay_off[2]) + 50  # frame 2 (100 B) and frame 3 reach past it
    dec.decode_batch(dev(torch, np.zeros(n, np.uint32)), dev(torch, wire_off), dev(torch, wl), dev(torch, wire),
                     dev(torch, pay_off), out, fl, st, verify_first=True, out_bytes=limit)
    torch.cuda.synchronize()
    stt, o = host(st, np.int32), host(out, np.uint8)
    assert stt[0] == 0 and stt[1] == 0
    assert stt[2] == C.ERR_BOUND and stt[3] == C.ERR_BOUND
    assert bool((o[int(pay_off[2]):] == 0x77).all())


def _host_verdicts(wire, wire_off, wl, sid, peer):
    """check_basic_command_structure + check_validity in frame order
    (src/mechanism_base.cpp:14-25, src/curve_mechanism_base.cpp:80-106), the
    rule ZMQG_OPT_REPLAY_HOST's caller applies; advances `peer` per session."""
    v = np.zeros(len(wl), np.int32)
    for i in range(len(wl)):
        L, o = int(wl[i]), int(wire_off[i])
        f = wire[o:o + L].tobytes()
        if L <= 1 or L <= f[0]:
            v[i] = 0x10000011
        elif L < 8 or f[:8] != b"\x07MESSAGE":
            v[i] = 0x10000001
        elif L < 33:
            v[i] = 0x10000012
        else:
            nonce = int.from_bytes(f[8:16], "big")
            if nonce <= peer[sid[i]]:
                v[i] = 0x10000002
            else:
                peer[sid[i]] = nonce
    return v


@pytest.mark.parametrize("big", [False, True])
def test_replay_host_matches_oracle(torch_cuda, C, big):
    """ZMQG_OPT_REPLAY_HOST: eight interleaved sessions with replays,
    reordering, tampered tags, broken headers and short frames; the host's
    verdicts plus the device's open give the oracle's statuses, flags and
    payloads, and the device's peer nonces are left alone.  `big` adds
    frames above the frame kernel's 4.5 KiB (the body kernels run)."""
    torch = torch_cuda
    rng = np.random.default_rng(93)
    S = 8
    precoms = [rng.integers(0, 256, 32, dtype=np.uint8).tobytes() for _ in range(S)]
    sess = O.make_sessions(precoms, dec_prefix=O.CLIENT_PREFIX)
    choices = [0, 1, 31, 200, 1024, 4000] + ([9000, 70000] if big else [])
    n = 600
    sizes = [int(x) for x in rng.choice(choices, n)]
    sid = rng.integers(0, S, n).astype(np.uint32)
    nonce = np.zeros(n, np.uint64)
    nxt = [5] * S
    for i in range(n):
        s = int(sid[i])
        r = rng.random()
        if r < 0.06 and nxt[s] > 6:
            nonce[i] = nxt[s] - 1 - int(rng.integers(0, 2))  # a replay
        else:
            nonce[i] = nxt[s]
            nxt[s] += 1 + int(rng.integers(0, 3))  # gaps are fine
    payloads = [rng.integers(0, 256, s_, dtype=np.uint8).tobytes() for s_ in sizes]
    inp, in_off = pack(payloads)
    flags = (np.arange(n) % 3 == 0).astype(np.uint8)
    wl = np.array([s_ + 33 for s_ in sizes], np.uint32)
    wire_off = np.concatenate([[0], np.cumsum(wl)[:-1]]).astype(np.uint64)
    enc = O.make_sessions(precoms)
    wire = O.encode_batch(enc, sid, nonce, flags, in_off, np.array(sizes, np.uint32), inp, wire_off, int(wl.sum()))
    for i in range(0, n, 7):
        wire[wire_off[i] + 16 + int(rng.integers(0, 16))] ^= 0x10  # MAC failures
    wire[wire_off[n - 3] + 2] ^= 0x20  # broken command name
    wl[n - 5] = 20  # short frame (its bytes stay in place)
    peer0 = np.full(S, 2, np.uint64)
    verdict = _host_verdicts(wire, wire_off, wl, sid, [int(p) for p in peer0])
    # the oracle applies the rules itself
    opeer = peer0.copy()
    out_off = in_off
    out_bytes = int(out_off[-1]) + sizes[-1] + 16
    rpl, rfl, rst = O.decode_batch(sess, opeer, sid, wire_off, wl, wire, out_off, out_bytes)
    dec = C.CurveContext(0, S)
    for s in range(S):
        dec.session_set(s, precoms[s], O.SERVER_PREFIX, O.CLIENT_PREFIX, False, 2)
    out = torch.zeros(out_bytes, dtype=torch.uint8, device="cuda")
    fl = torch.zeros(n, dtype=torch.uint8, device="cuda")
    st = torch.zeros(n, dtype=torch.int32, device="cuda")
    dec.decode_batch(dev(torch, sid), dev(torch, wire_off), dev(torch, wl), dev(torch, wire), dev(torch, out_off),
                     out, fl, st, verify_first=True, verdict_in=dev(torch, verdict))
    torch.cuda.synchronize()
    gst = host(st, np.int32)
    assert np.array_equal(gst, rst), np.nonzero(gst != rst)[0][:10]
    assert np.array_equal(host(fl, np.uint8), rfl)
    assert (rst == 0x10000002).sum() > 10 and (rst == 0x11000001).sum() > 10
    got = host(out, np.uint8)
    for i in range(n):  # verified payloads, zeros for every failed frame's region
        if wl[i] > 33:
            a, b = int(out_off[i]), int(out_off[i]) + int(wl[i]) - 33
            assert np.array_equal(got[a:b], rpl[a:b]), (i, sizes[i], int(rst[i]))
    assert [dec.get_peer_nonce(s) for s in range(S)] == [2] * S  # the host keeps them
