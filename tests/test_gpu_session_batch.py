"""zmqg_session_set_batch (the mass handshake):
4,096 sessions derived on the device by zmqg_box_beforenm_batch and installed
in one asynchronous launch from its device output, then one frame encoded and
decoded per session, every byte against the oracle's sequential
curve_encoding_t (keys from the oracle's own crypto_box_beforenm).
Reference: the precom derivations at src/curve_server.cpp:382-383 and
src/curve_client_tools.hpp:105; the codec at src/curve_mechanism_base.cpp:111-284."""
import numpy as np
import pytest

from oracle import oracle as O
from tests.helpers import pack, wire_layout

pytestmark = pytest.mark.gpu

S = 4096


def _dev(torch, a, dt=None):
    a = np.ascontiguousarray(a)
    if a.dtype == np.uint64:
        a = a.view(np.int64)
    elif a.dtype == np.uint32:
        a = a.view(np.int32)
    return torch.from_numpy(a.copy()).to("cuda")


def _oracle_sessions(precoms, enc_prefix, dec_prefix, downgrade):
    s = np.zeros(len(precoms), O.SESSION_DTYPE)
    for i, p in enumerate(precoms):
        s[i]["precom"] = np.frombuffer(p, np.uint8)
        s[i]["enc_prefix"] = np.frombuffer(enc_prefix, np.uint8)
        s[i]["dec_prefix"] = np.frombuffer(dec_prefix, np.uint8)
        s[i]["downgrade_sub"] = int(downgrade[i])
    return s


def test_batch_install_4096_sessions_encode_decode(torch_cuda, C):
    torch = torch_cuda
    rng = np.random.default_rng(4096)
    sk = [rng.integers(0, 256, 32, dtype=np.uint8).tobytes() for _ in range(S)]
    pk = [rng.integers(0, 256, 32, dtype=np.uint8).tobytes() for _ in range(S)]
    # the oracle's keys, indexed by session id below
    ref = [O.box_beforenm(p, s) for p, s in zip(pk, sk)]
    assert all(rc == 0 for rc, _ in ref)

    keyctx = C.CurveContext(0, 1)
    k_out = torch.zeros(32 * S, dtype=torch.uint8, device="cuda")
    st = torch.zeros(S, dtype=torch.int32, device="cuda")
    keyctx.box_beforenm_batch(_dev(torch, np.frombuffer(b"".join(pk), np.uint8)),
                              _dev(torch, np.frombuffer(b"".join(sk), np.uint8)), k_out, st)
    # key j goes to session perm[j] (installs are unordered); half the
    # sessions downgraded, peer nonces spread
    perm = rng.permutation(S).astype(np.uint32)
    down_j = (rng.integers(0, 2, S) == 1).astype(np.uint8)
    peer_j = rng.integers(1, 1 << 40, S).astype(np.uint64)
    stream = torch.cuda.current_stream()
    cli = C.CurveContext(0, S)
    srv = C.CurveContext(0, S)
    cli.session_set_batch(perm, k_out, C.CLIENT_PREFIX, C.SERVER_PREFIX, down_j, None, stream)
    srv.session_set_batch(perm, k_out, C.SERVER_PREFIX, C.CLIENT_PREFIX, down_j, peer_j, stream)
    # by session id
    precom_s = [None] * S
    down_s = np.zeros(S, np.uint8)
    peer_s = np.zeros(S, np.uint64)
    for j in range(S):
        precom_s[perm[j]] = ref[j][1]
        down_s[perm[j]] = down_j[j]
        peer_s[perm[j]] = peer_j[j]
    assert cli.get_nonce(int(perm[5])) == 1 and cli.get_peer_nonce(int(perm[5])) == 1
    assert srv.get_peer_nonce(int(perm[7])) == int(peer_j[7])

    # one frame per session, in a shuffled order; every flag kind
    n = S
    sid = rng.permutation(S).astype(np.uint32)
    lens = rng.integers(0, 300, n).astype(np.uint32)
    flags = rng.choice(np.array([0, 1, 2, 3, 12, 16], np.uint8), n)
    nonce = (peer_s[sid] + rng.integers(1, 5, n).astype(np.uint64)).astype(np.uint64)
    payloads = [rng.integers(0, 256, int(l), dtype=np.uint8).tobytes() for l in lens]
    inp, in_off = pack(payloads, rng, 7)
    w_off, w_len, w_total = wire_layout(flags, lens, down_s, sid, rng, 5)
    wire = torch.zeros(max(w_total, 1), dtype=torch.uint8, device="cuda")
    cli.encode_batch(_dev(torch, sid), _dev(torch, nonce), _dev(torch, flags), _dev(torch, in_off),
                     _dev(torch, lens), _dev(torch, inp), _dev(torch, w_off), wire, stream)
    torch.cuda.synchronize()
    got = wire.cpu().numpy()[:w_total]
    osess_c = _oracle_sessions(precom_s, O.CLIENT_PREFIX, O.SERVER_PREFIX, down_s)
    want = O.encode_batch(osess_c, sid, nonce, flags, in_off, lens, inp, w_off, w_total)
    assert np.array_equal(got, want)

    # decode on the server side; a few frames tampered
    tam = rng.choice(n, 40, replace=False)
    wire_np = want.copy()
    for i in tam:
        wire_np[int(w_off[i]) + 16 + int(rng.integers(0, 16))] ^= 0x20  # the tag
    p_out = np.zeros(n, np.uint64)
    pos = 0
    for i in range(n):
        p_out[i] = pos
        pos += max(int(w_len[i]) - 33, 0) + 3
    out = torch.zeros(max(pos, 1), dtype=torch.uint8, device="cuda")
    fl = torch.zeros(n, dtype=torch.uint8, device="cuda")
    stt = torch.zeros(n, dtype=torch.int32, device="cuda")
    srv.decode_batch(_dev(torch, sid), _dev(torch, w_off), _dev(torch, w_len), _dev(torch, wire_np),
                     _dev(torch, p_out), out, fl, stt, stream)
    torch.cuda.synchronize()
    osess_s = _oracle_sessions(precom_s, O.SERVER_PREFIX, O.CLIENT_PREFIX, down_s)
    peer_o = peer_s.copy()
    o_out, o_fl, o_st = O.decode_batch(osess_s, peer_o, sid, w_off, w_len, wire_np, p_out, pos)
    assert np.array_equal(stt.cpu().numpy(), o_st)
    assert set(np.nonzero(o_st)[0].tolist()) == set(int(i) for i in tam)
    assert np.array_equal(fl.cpu().numpy(), o_fl)
    assert np.array_equal(out.cpu().numpy()[:pos], o_out)
    for s_ in (0, 17, S - 1):
        assert srv.get_peer_nonce(s_) == int(peer_o[s_])


def test_batch_install_rejects_bad_sids(torch_cuda, C):
    torch = torch_cuda
    ctx = C.CurveContext(0, 8)
    k = torch.zeros(32 * 3, dtype=torch.uint8, device="cuda")
    with pytest.raises(C.ZmqgError):
        ctx.session_set_batch([1, 2, 1], k, C.CLIENT_PREFIX, C.SERVER_PREFIX)
    with pytest.raises(C.ZmqgError):
        ctx.session_set_batch([1, 2, 8], k, C.CLIENT_PREFIX, C.SERVER_PREFIX)
    ctx.session_set_batch([1, 2, 3], k, C.CLIENT_PREFIX, C.SERVER_PREFIX)
    torch.cuda.synchronize()
    assert ctx.get_nonce(2) == 1 and ctx.get_peer_nonce(3) == 1


def test_batch_install_send_nonces(torch_cuda, C):
    """zmqg_session_set_batch_ex: each session's send nonce as installed (a
    client connection continues from 3 after HELLO and INITIATE), and the
    first nonce-auto encode takes it, against the oracle."""
    torch = torch_cuda
    rng = np.random.default_rng(77)
    keys = [rng.integers(0, 256, 32, dtype=np.uint8).tobytes() for _ in range(4)]
    k = torch.from_numpy(np.frombuffer(b"".join(keys), np.uint8).copy()).to("cuda")
    ctx = C.CurveContext(0, 4)
    sn = np.array([3, 10, 1 << 33, 7], np.uint64)
    ctx.session_set_batch([2, 0, 3, 1], k, C.CLIENT_PREFIX, C.SERVER_PREFIX, peer_nonce=[5, 6, 7, 8],
                          send_nonce=sn)
    torch.cuda.synchronize()
    assert [ctx.get_nonce(s) for s in (2, 0, 3, 1)] == [int(x) for x in sn]
    assert [ctx.get_peer_nonce(s) for s in (2, 0, 3, 1)] == [5, 6, 7, 8]
    # one 100-byte frame per session, nonces assigned on the device
    sid = np.array([0, 1, 2, 3], np.uint32)
    lens = np.full(4, 100, np.uint32)
    flags = np.zeros(4, np.uint8)
    payloads = [rng.integers(0, 256, 100, dtype=np.uint8).tobytes() for _ in range(4)]
    inp, in_off = pack(payloads, rng, 3)
    w_off, w_len, w_total = wire_layout(flags, lens, np.zeros(4, np.uint8), sid, rng, 3)
    wire = torch.zeros(w_total, dtype=torch.uint8, device="cuda")
    ctx.encode_batch(_dev(torch, sid), None, _dev(torch, flags), _dev(torch, in_off), _dev(torch, lens),
                     _dev(torch, inp), _dev(torch, w_off), wire, nonce_auto=True)
    torch.cuda.synchronize()
    by_sid = {2: keys[0], 0: keys[1], 3: keys[2], 1: keys[3]}
    nonce_by_sid = {2: 3, 0: 10, 3: 1 << 33, 1: 7}
    osess = _oracle_sessions([by_sid[s] for s in range(4)], O.CLIENT_PREFIX, O.SERVER_PREFIX, np.zeros(4, np.uint8))
    nonce = np.array([nonce_by_sid[int(s)] for s in sid], np.uint64)
    want = O.encode_batch(osess, sid, nonce, flags, in_off, lens, inp, w_off, w_total)
    assert np.array_equal(wire.cpu().numpy(), want)
    assert [ctx.get_nonce(s) for s in (2, 0, 3, 1)] == [int(x) + 1 for x in sn]
