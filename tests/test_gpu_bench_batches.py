"""The exact batches bench.py times for BASELINE configs 3 and 5 (built by
bench.config_inputs, stepped by bench.config_step: encode with
device-assigned nonces, then decode), checked against the oracle at full
size rather than only round-tripped:

  config 3  49,152 frames of {64 B, 1 KiB, 64 KiB}, 256 sessions: every
            64 KiB frame's wire bytes (header, nonce, tag, ciphertext) and a
            3,000-frame sample of the others equal the oracle's
            curve_encoding_t::encode; the decode returns every payload with
            status 0 and leaves each session's peer nonce at its last nonce.
  config 5  1,024 x 16 MiB frames, 8 sessions, on one GPU: 16 spread frames'
            wire bytes equal the oracle's; the whole batch round-trips.

A symmetric keystream or MAC bug (one the round trip cannot see) shows in
the encode comparison; the decode is then checked by the round trip plus
its tag verdicts on oracle-exact wire.  Reference: src/curve_mechanism_base.cpp:111-284."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _setup(torch, C, w):
    import bench
    b = bench.config_inputs(C, torch, torch.device("cuda", 0), 0, 0, w)
    bench.config_step(b)
    torch.cuda.synchronize()
    return b


def _nonces(sid):
    """NONCE_AUTO from a send counter of 3: each session's frames in batch order."""
    n = len(sid)
    nonce = np.zeros(n, np.uint64)
    first = {}
    for i, s in enumerate(sid.tolist()):
        first.setdefault(s, i)
        nonce[i] = 3 + i - first[s]
    return nonce


def _oracle_check(torch, b, idx, nonce):
    """Oracle encode of frames idx (their sessions, nonces, payloads) == the
    device's wire bytes of those frames."""
    sizes, W, in_off, out_off, sid = b["sizes"], b["W"], b["in_off"], b["out_off"], b["sid"]
    pay_h = []
    wire_h = []
    for i in idx.tolist():
        a, L = int(in_off[i]), int(sizes[i])
        pay_h.append(b["payload"][a:a + L].cpu().numpy())
        o, wl = int(out_off[i]), int(W[i])
        wire_h.append(b["wire"][o:o + wl].cpu().numpy())
    k = len(idx)
    lens = np.array([len(p) for p in pay_h], np.uint32)
    p_off = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    wls = lens.astype(np.uint64) + 33
    w_off = np.concatenate([[0], np.cumsum(wls)[:-1]]).astype(np.uint64)
    ref = O.encode_batch(O.make_sessions(b["keys"]), sid[idx], nonce[idx], np.zeros(k, np.uint8), p_off, lens,
                         np.concatenate(pay_h), w_off, int(wls.sum()))
    got = np.concatenate(wire_h)
    if not np.array_equal(got, ref):
        for j in range(k):
            a, e = int(w_off[j]), int(w_off[j] + wls[j])
            assert np.array_equal(got[a:e], ref[a:e]), ("frame", int(idx[j]), "size", int(lens[j]))


def _roundtrip(torch, b, nonce):
    assert int((b["st"] != 0).sum()) == 0
    assert torch.equal(b["back"], b["payload"])
    sid = b["sid"]
    last = {}
    for i, s in enumerate(sid.tolist()):
        last[s] = int(nonce[i])
    for s in sorted(set([0, 1, b["S"] // 2, b["S"] - 1]) & set(last)):
        assert b["dec"].get_peer_nonce(s) == last[s]
        assert b["enc"].get_nonce(s) == last[s] + 1


def test_config3_bench_batch_vs_oracle(torch_cuda, C):
    torch = torch_cuda
    b = _setup(torch, C, "3")
    assert b["n"] == 49152 and b["S"] == 256
    nonce = _nonces(b["sid"])
    big = np.nonzero(b["sizes"] == 65536)[0]
    assert len(big) > 15000
    rng = np.random.default_rng(33)
    small = np.nonzero(b["sizes"] != 65536)[0]
    sample = np.sort(rng.choice(small, 3000, replace=False))
    # every 64 KiB frame, in chunks (bounded host memory per oracle call)
    for c in range(0, len(big), 2048):
        _oracle_check(torch, b, big[c:c + 2048], nonce)
    _oracle_check(torch, b, sample, nonce)
    _roundtrip(torch, b, nonce)


def test_config5_bench_batch_vs_oracle(torch_cuda, C):
    torch = torch_cuda
    b = _setup(torch, C, "5")
    assert b["n"] == 1024 and int(b["sizes"][0]) == 16 << 20 and b["S"] == 8
    nonce = _nonces(b["sid"])
    idx = np.linspace(0, b["n"] - 1, 16).astype(np.int64)
    for c in range(0, 16, 4):
        _oracle_check(torch, b, idx[c:c + 4], nonce)
    _roundtrip(torch, b, nonce)
