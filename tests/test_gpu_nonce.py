"""GPU tests of ZMQG_OPT_NONCE_AUTO: encode nonces taken from each session's
send counter on the device, in batch order, as curve_encoding_t's
get_and_inc_nonce assigns them per message (src/curve_mechanism_base.hpp:41,
called at src/curve_mechanism_base.cpp:116).  The wire must equal the
oracle's encode with the nonces the reference would have used, and the
counters must advance by each session's frame count across calls."""
import numpy as np
import pytest

from oracle import oracle as O
from tests.helpers import pack

pytestmark = pytest.mark.gpu


def _t(torch, a):
    a = np.ascontiguousarray(a)
    if a.dtype == np.uint64:
        a = a.view(np.int64)
    elif a.dtype == np.uint32:
        a = a.view(np.int32)
    return torch.from_numpy(a.copy()).to("cuda")


@pytest.mark.parametrize("n_sessions,n,big", [(1, 300, True), (1, 70000, False), (7, 2000, True),
                                              (1024, 70000, False)])
def test_nonce_auto_matches_get_and_inc(torch_cuda, C, n_sessions, n, big):
    torch = torch_cuda
    rng = np.random.default_rng(n_sessions * 1000 + n)
    keys = [rng.integers(0, 256, 32, dtype=np.uint8).tobytes() for _ in range(n_sessions)]
    ctx = C.CurveContext(0, n_sessions)
    for s, k in enumerate(keys):
        ctx.session_set(s, k, O.CLIENT_PREFIX, O.SERVER_PREFIX)
    assert all(ctx.get_nonce(s) == 1 for s in range(min(n_sessions, 4)))  # _cn_nonce (1)
    start = rng.integers(1, 1 << 40, n_sessions, dtype=np.uint64)
    start[0] = (1 << 32) - 5  # crosses the 32-bit boundary inside the batch
    for s in range(n_sessions):
        ctx.set_nonce(s, int(start[s]))
    sess = np.concatenate([O.make_sessions([k]) for k in keys])
    ctr = start.copy()
    for call in range(2):
        if n_sessions == 1:
            sid = np.zeros(n, np.uint32)
        elif call == 0:
            sid = rng.integers(0, n_sessions, n).astype(np.uint32)
        else:  # runs of one session, as a batcher per connection produces them
            sid = np.sort(rng.integers(0, n_sessions, n)).astype(np.uint32)
        sizes = rng.choice([0, 1, 31, 200, 1024], n).astype(np.uint32)
        if big:
            sizes[n // 3] = 70000  # the chunked (body) path's head takes the nonce too
        flags = rng.choice([0, 1], n).astype(np.uint8)
        pays = [rng.integers(0, 256, int(s), dtype=np.uint8).tobytes() for s in sizes]
        inp, in_off = pack(pays)
        wl = np.array([O.wire_size(int(f), 0, int(s)) for f, s in zip(flags, sizes)], np.uint32)
        _, woff = pack([b"\0" * int(w) for w in wl])
        total = int(woff[-1]) + int(wl[-1]) + 16
        # the reference's nonces: one get_and_inc_nonce per message, per session, in batch order
        nonce = np.zeros(n, np.uint64)
        for i in range(n):
            nonce[i] = ctr[sid[i]]
            ctr[sid[i]] += 1
        ref = O.encode_batch(sess, sid, nonce, flags, in_off, sizes, inp, woff, total)
        out = torch.zeros(total, dtype=torch.uint8, device="cuda")
        ctx.encode_batch(_t(torch, sid), None, _t(torch, flags), _t(torch, in_off), _t(torch, sizes),
                         _t(torch, inp), _t(torch, woff), out, nonce_auto=True)
        torch.cuda.synchronize()
        got = out.cpu().numpy()
        bad = np.flatnonzero(got != ref)
        assert bad.size == 0, f"call {call}: first mismatch at byte {bad[:4]}"
        for s in set(int(x) for x in rng.choice(n_sessions, min(n_sessions, 16), replace=False)) | {0}:
            assert ctx.get_nonce(s) == int(ctr[s]), s


def test_nonce_auto_rejects_too_many_sessions(torch_cuda, C):
    torch = torch_cuda
    ctx = C.CurveContext(0, 8193)
    z = torch.zeros(4, dtype=torch.int32, device="cuda")
    with pytest.raises(C.ZmqgError):
        ctx.encode_batch(z, None, z.to(torch.uint8), z.to(torch.int64), z, z.to(torch.uint8), z.to(torch.int64),
                         torch.zeros(256, dtype=torch.uint8, device="cuda"), nonce_auto=True)
