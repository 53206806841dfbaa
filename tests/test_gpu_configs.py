"""GPU parity at BASELINE.json's full per-GPU sizes (configs 4 and 5).

Each test combines
  * size-independent properties over the whole batch, on the device: the
    decode of the encoded batch returns every payload byte and flag, every
    status is 0, and each session's peer nonce ends at its last nonce;
  * bit-exact oracle checks: config 4's WHOLE 16 Mi-frame wire (4.5 GiB)
    against oracle/curve_oracle.c run over 1 Mi-frame chunks on the host's
    cores (round 5; a round trip alone cannot see a keystream or MAC bug
    that encode and decode share), and a seeded sample of frames elsewhere.
Inputs are generated on the device from a seed (torch Philox), descriptors as
SURVEY.md section 8(d) specifies for the config.
"""
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _keys(n_sessions, seed):
    rng = np.random.default_rng(seed)
    return [rng.integers(0, 256, 32, dtype=np.uint8).tobytes() for _ in range(n_sessions)]


def _contexts(C, keys):
    enc = C.CurveContext(0, len(keys))
    dec = C.CurveContext(0, len(keys))
    for s, k in enumerate(keys):
        enc.session_set(s, k, O.CLIENT_PREFIX, O.SERVER_PREFIX)
        dec.session_set(s, k, O.SERVER_PREFIX, O.CLIENT_PREFIX, False, 2)
    return enc, dec


def _check_sample(torch, keys, idx, sid, nonce, flags, P, payload, wire, W):
    """Oracle encode of the sampled frames idx (sid, nonce, flags: theirs, in
    sample order) == their wire bytes on the device."""
    k = len(idx)
    ti = torch.from_numpy(idx.astype(np.int64)).to("cuda")
    pay = payload.view(-1, P)[ti].cpu().numpy().reshape(-1)
    got = wire.view(-1, W)[ti].cpu().numpy().reshape(-1)
    ref = O.encode_batch(O.make_sessions(keys), sid.astype(np.uint32), nonce.astype(np.uint64),
                         flags.astype(np.uint8), np.arange(k, dtype=np.uint64) * P, np.full(k, P, np.uint32),
                         pay, np.arange(k, dtype=np.uint64) * W, k * W)
    assert np.array_equal(got, ref)


def _host_threads():
    try:
        return max(1, min(16, len(os.sched_getaffinity(0))))
    except AttributeError:
        return max(1, min(16, os.cpu_count() or 1))


def _check_all_uniform(torch, sessions, n, P, ns, payload, wire, W, chunk=1 << 20):
    """Every frame of a uniform batch (frame i: sid i mod ns, nonce 3 + i // ns,
    MORE on one in 16) bit-exact against the oracle: the device wire is copied
    back a chunk at a time and the oracle (a ctypes call, which releases the
    GIL) encodes the chunk's frames in slices on the host's cores."""
    pw = payload.view(-1, P)
    ww = wire.view(-1, W)
    nt = _host_threads()

    def oracle_slice(a, b, pay):
        i = np.arange(a, b, dtype=np.int64)
        k = b - a
        return O.encode_batch(sessions, (i % ns).astype(np.uint32), (3 + i // ns).astype(np.uint64),
                              (i % 16 == 15).astype(np.uint8), np.arange(k, dtype=np.uint64) * P,
                              np.full(k, P, np.uint32), pay, np.arange(k, dtype=np.uint64) * W, k * W)

    with ThreadPoolExecutor(nt) as ex:
        for a in range(0, n, chunk):
            b = min(n, a + chunk)
            pay = pw[a:b].cpu().numpy().reshape(-1)
            got = ww[a:b].cpu().numpy().reshape(-1)
            cuts = np.linspace(a, b, nt + 1).astype(np.int64)
            futs = [ex.submit(oracle_slice, int(x), int(y), pay[(x - a) * P:(y - a) * P])
                    for x, y in zip(cuts[:-1], cuts[1:]) if y > x]
            ref = np.concatenate([f.result() for f in futs])
            if not np.array_equal(got, ref):
                bad = int(np.flatnonzero(got != ref)[0])
                raise AssertionError(f"frame {a + bad // W} differs from the oracle (byte {bad % W})")


def test_config4_full_size_flood(torch_cuda, C):
    """Config 4 at the size of one GPU's whole batch: 16 Mi x 256 B frames over
    1024 sessions (sid = i mod 1024), per-session sequential nonces from 3,
    MORE on one frame in 16."""
    torch = torch_cuda
    n, P, ns = 16 << 20, 256, 1024
    W = P + 33
    keys = _keys(ns, 40)
    enc, dec = _contexts(C, keys)
    i = torch.arange(n, device="cuda", dtype=torch.int64)
    sid = (i % ns).to(torch.int32)
    nonce = 3 + i // ns
    flags = (i % 16 == 15).to(torch.uint8)
    in_off = i * P
    lens = torch.full((n,), P, dtype=torch.int32, device="cuda")
    out_off = i * W
    g = torch.Generator(device="cuda")
    g.manual_seed(41)
    payload = torch.randint(0, 256, (n * P,), dtype=torch.uint8, device="cuda", generator=g)
    wire = torch.zeros(n * W, dtype=torch.uint8, device="cuda")
    enc.encode_batch(sid, nonce, flags, in_off, lens, payload, out_off, wire)
    back = torch.zeros(n * P, dtype=torch.uint8, device="cuda")
    fl = torch.zeros(n, dtype=torch.uint8, device="cuda")
    st = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    wl = torch.full((n,), W, dtype=torch.int32, device="cuda")
    dec.decode_batch(sid, out_off, wl, wire, in_off, back, fl, st)
    torch.cuda.synchronize()
    assert int((st != 0).sum()) == 0
    assert torch.equal(fl, flags)
    assert torch.equal(back, payload)
    last = 3 + (n // ns) - 1
    for s in (0, 1, 511, 1023):
        assert dec.get_peer_nonce(s) == last
    rng = np.random.default_rng(42)
    idx = np.sort(rng.choice(n, 4096, replace=False))
    idx[:2] = [0, 1]
    idx[-1] = n - 1
    ii = idx.astype(np.int64)
    _check_sample(torch, keys, idx, (ii % ns), 3 + ii // ns, (ii % 16 == 15), P, payload, wire, W)
    # and every frame of the batch
    _check_all_uniform(torch, O.make_sessions(keys), n, P, ns, payload, wire, W)


def test_config4_replay_of_a_flood_slice(torch_cuda, C):
    """Re-decoding any frame of an accepted batch is a replay (nonce not above
    the session's peer nonce): every frame is rejected with
    ZMQ_PROTOCOL_ERROR_ZMTP_INVALID_SEQUENCE and its payload region zeroed."""
    torch = torch_cuda
    n, P, ns = 1 << 20, 256, 1024
    W = P + 33
    keys = _keys(ns, 43)
    enc, dec = _contexts(C, keys)
    i = torch.arange(n, device="cuda", dtype=torch.int64)
    sid = (i % ns).to(torch.int32)
    nonce = 3 + i // ns
    flags = torch.zeros(n, dtype=torch.uint8, device="cuda")
    lens = torch.full((n,), P, dtype=torch.int32, device="cuda")
    payload = torch.randint(0, 256, (n * P,), dtype=torch.uint8, device="cuda")
    wire = torch.zeros(n * W, dtype=torch.uint8, device="cuda")
    enc.encode_batch(sid, nonce, flags, i * P, lens, payload, i * W, wire)
    wl = torch.full((n,), W, dtype=torch.int32, device="cuda")
    back = torch.zeros(n * P, dtype=torch.uint8, device="cuda")
    fl = torch.zeros(n, dtype=torch.uint8, device="cuda")
    st = torch.zeros(n, dtype=torch.int32, device="cuda")
    dec.decode_batch(sid, i * W, wl, wire, i * P, back, fl, st)
    torch.cuda.synchronize()
    assert int((st != 0).sum()) == 0 and torch.equal(back, payload)
    back.fill_(0x5a)
    dec.decode_batch(sid, i * W, wl, wire, i * P, back, fl, st)
    torch.cuda.synchronize()
    assert int((st != C.ERR_INVALID_SEQUENCE).sum()) == 0
    assert int(back.count_nonzero()) == 0


def test_config5_jumbo_per_gpu_share(torch_cuda, C):
    """Config 5's per-GPU share at 8 GPUs: 128 x 16 MiB frames (2 GiB), 16
    sessions; round trip over the whole batch, oracle on three frames."""
    torch = torch_cuda
    n, P, ns = 128, 16 << 20, 16
    W = P + 33
    keys = _keys(ns, 44)
    enc, dec = _contexts(C, keys)
    i = torch.arange(n, device="cuda", dtype=torch.int64)
    sid = (i % ns).to(torch.int32)
    nonce = 3 + i // ns
    flags = (i % 16 == 15).to(torch.uint8)
    lens = torch.full((n,), P, dtype=torch.int32, device="cuda")
    g = torch.Generator(device="cuda")
    g.manual_seed(45)
    payload = torch.randint(0, 256, (n * P,), dtype=torch.uint8, device="cuda", generator=g)
    wire = torch.zeros(n * W, dtype=torch.uint8, device="cuda")
    enc.encode_batch(sid, nonce, flags, i * P, lens, payload, i * W, wire)
    back = torch.zeros(n * P, dtype=torch.uint8, device="cuda")
    fl = torch.zeros(n, dtype=torch.uint8, device="cuda")
    st = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    wl = torch.full((n,), W, dtype=torch.int32, device="cuda")
    dec.decode_batch(sid, i * W, wl, wire, i * P, back, fl, st)
    torch.cuda.synchronize()
    assert int((st != 0).sum()) == 0
    assert torch.equal(fl, flags) and torch.equal(back, payload)
    idx = np.array([0, 77, n - 1])
    _check_sample(torch, keys, idx, idx % ns, 3 + idx // ns, (idx % 16 == 15), P, payload, wire, W)


def test_big_frame_failures_zero_filled(torch_cuda, C):
    """Frames spanning many body tiles that fail (flipped ciphertext bit, flipped
    tag bit, replayed nonce) get their status and a zero-filled payload region,
    while the frames around them decode intact (the decode body kernel's
    end-of-kernel zero-fill after every workgroup's release)."""
    torch = torch_cuda
    sizes = [65536, 70000, 1 << 20, 65536, 200000, 65536, 1 << 20, 12288, 65536, 300000]
    n = len(sizes)
    keys = _keys(1, 46)
    enc, dec = _contexts(C, keys)
    rng = np.random.default_rng(47)
    pay = [rng.integers(0, 256, s, dtype=np.uint8) for s in sizes]
    in_off = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64)
    W = np.array(sizes, np.uint64) + 33
    out_off = np.concatenate([[0], np.cumsum(W)[:-1]]).astype(np.uint64)
    nonce = np.arange(3, 3 + n, dtype=np.uint64)
    nonce[6] = nonce[4]  # frame 6 replays frame 4's nonce
    t = lambda a, d: torch.from_numpy(np.ascontiguousarray(a).view(d)).to("cuda")
    sid = torch.zeros(n, dtype=torch.int32, device="cuda")
    flags = torch.zeros(n, dtype=torch.uint8, device="cuda")
    payload = t(np.concatenate(pay), np.uint8)
    wire = torch.zeros(int(W.sum()), dtype=torch.uint8, device="cuda")
    enc.encode_batch(sid, t(nonce, np.int64), flags, t(in_off, np.int64), t(np.array(sizes, np.uint32), np.int32),
                     payload, t(out_off, np.int64), wire)
    torch.cuda.synchronize()
    w = wire.cpu().numpy()
    w[int(out_off[1]) + 33 + 50000] ^= 4          # ciphertext bit, frame 1 (70 KB)
    w[int(out_off[2]) + 20] ^= 1                  # tag bit, frame 2 (1 MiB)
    w[int(out_off[9]) + int(W[9]) - 1] ^= 0x80    # last ciphertext byte, frame 9
    back = torch.full((int(sum(sizes)),), 0x5A, dtype=torch.uint8, device="cuda")
    fl = torch.zeros(n, dtype=torch.uint8, device="cuda")
    st = torch.zeros(n, dtype=torch.int32, device="cuda")
    dec.decode_batch(sid, t(out_off, np.int64), t(W.astype(np.uint32), np.int32), t(w, np.uint8),
                     t(in_off, np.int64), back, fl, st)
    torch.cuda.synchronize()
    got = back.cpu().numpy()
    status = st.cpu().numpy()
    expect = {1: C.ERR_CRYPTOGRAPHIC, 2: C.ERR_CRYPTOGRAPHIC, 6: C.ERR_INVALID_SEQUENCE, 9: C.ERR_CRYPTOGRAPHIC}
    for i in range(n):
        region = got[int(in_off[i]):int(in_off[i]) + sizes[i]]
        assert status[i] == expect.get(i, 0), (i, status[i])
        if i in expect:
            assert not region.any(), i
        else:
            assert np.array_equal(region, pay[i]), i
    assert dec.get_peer_nonce(0) == int(nonce.max())
