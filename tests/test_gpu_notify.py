"""GPU tests of the completion wake-up (zmqg_fence_record_notify,
include/zmqg_curve.h) and of the ctx's stream ordering on the null stream.

The reference I/O thread sleeps in epoll_wait (src/epoll.cpp:157-158) and
wakes only for a descriptor it watches; the batched codec's completion must
therefore arrive as a readable descriptor.  Checked: an eventfd becomes
readable once a config-2-sized decode batch has finished (never before the
fence is reached: zmqg_fence_query is 1 as soon as the fd is readable), the
counter sums several fences, and zmqg_notify_quiesce returns once every
notification has run.  Ordering: a session install on the null stream
(handle 0, which orders nothing against the ctx's non-blocking own stream)
is seen by a per-message call issued right after it with no
synchronisation, and by the session accessors.
"""
import ctypes
import os
import select

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _batch(torch, C, n=65536, P=1024, seed=3):
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(seed)
    key = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    enc = C.CurveContext(0, 1)
    enc.session_set(0, key, O.CLIENT_PREFIX, O.SERVER_PREFIX)
    dec = C.CurveContext(0, 1)
    dec.session_set(0, key, O.SERVER_PREFIX, O.CLIENT_PREFIX, False, 2)
    W = C.wire_size(0, 0, P)
    t = lambda a, d: torch.from_numpy(np.ascontiguousarray(a).view(d)).to(dev)
    b = dict(sid=torch.zeros(n, dtype=torch.int32, device=dev),
             pay=torch.randint(0, 256, (n * P,), dtype=torch.uint8, device=dev),
             in_off=t(np.arange(n, dtype=np.uint64) * P, np.int64),
             lens=t(np.full(n, P, np.uint32), np.int32),
             w_off=t(np.arange(n, dtype=np.uint64) * W, np.int64),
             wl=t(np.full(n, W, np.uint32), np.int32),
             wire=torch.zeros(n * W, dtype=torch.uint8, device=dev),
             flags=torch.zeros(n, dtype=torch.uint8, device=dev),
             back=torch.zeros(n * P, dtype=torch.uint8, device=dev),
             fl=torch.zeros(n, dtype=torch.uint8, device=dev),
             st=torch.full((n,), -1, dtype=torch.int32, device=dev))
    enc.encode_batch(b["sid"], t(np.arange(3, 3 + n, dtype=np.uint64), np.int64), b["flags"], b["in_off"],
                     b["lens"], b["pay"], b["w_off"], b["wire"])
    torch.cuda.synchronize()
    return enc, dec, b


def test_notify_fd_readable_when_the_batch_is_done(torch_cuda, C):
    torch = torch_cuda
    enc, dec, b = _batch(torch, C)
    L = C.lib()
    fd = os.eventfd(0, os.EFD_NONBLOCK | os.EFD_CLOEXEC)
    try:
        s = torch.cuda.Stream()
        fences = []
        with torch.cuda.stream(s):
            for k in range(3):
                if k == 0:
                    dec.decode_batch(b["sid"], b["w_off"], b["wl"], b["wire"], b["in_off"], b["back"], b["fl"],
                                     b["st"], stream=s.cuda_stream)
                f = ctypes.c_uint64()
                assert L.zmqg_fence_record_notify(dec._ctx, ctypes.c_void_p(s.cuda_stream), fd,
                                                  ctypes.byref(f)) == 0
                fences.append(f.value)
        assert fences == sorted(fences) and len(set(fences)) == 3
        # the I/O thread's wait: block on the descriptor alone
        total = 0
        while total < 3:
            r, _, _ = select.select([fd], [], [], 10.0)
            assert r == [fd], "no wake-up within 10 s"
            total += os.eventfd_read(fd)
            # readable => the fences it stands for are reached
            assert L.zmqg_fence_query(dec._ctx, fences[total - 1]) == 1
        assert total == 3
        assert L.zmqg_notify_quiesce(dec._ctx) == 0
        # the batch really is finished: its results are final on the host
        assert int((b["st"] != 0).sum()) == 0 and torch.equal(b["back"], b["pay"])
        for f in fences:
            assert L.zmqg_fence_query(dec._ctx, f) == 1
    finally:
        os.close(fd)


def test_notify_rejects_a_bad_fd(torch_cuda, C):
    ctx = C.CurveContext(0, 1)
    f = ctypes.c_uint64()
    assert C.lib().zmqg_fence_record_notify(ctx._ctx, None, -1, ctypes.byref(f)) == -22


def test_null_stream_install_is_seen_by_the_next_message_call(torch_cuda, C):
    """zmqg_session_set_batch on the null stream, then zmqg_encode_msg and
    zmqg_session_get_nonce with no synchronisation: the message is encoded
    under the installed key (bit-exact with the oracle) and the accessor
    sees the install's send counter."""
    torch = torch_cuda
    rng = np.random.default_rng(77)
    S = 64
    keys = rng.integers(0, 256, (S, 32), dtype=np.uint8)
    ctx = C.CurveContext(0, S)
    for rep in range(3):
        keys = rng.integers(0, 256, (S, 32), dtype=np.uint8)
        precom = torch.from_numpy(keys.reshape(-1).copy()).to("cuda")
        ctx.session_set_batch(np.arange(S, dtype=np.uint32), precom, O.CLIENT_PREFIX, O.SERVER_PREFIX, stream=0)
        sid = int(rng.integers(0, S))
        pay = rng.integers(0, 256, 700, dtype=np.uint8).tobytes()
        got = ctx.encode_msg(sid, 5, 0, pay)
        sess = O.make_sessions([keys[sid].tobytes()])
        ws = O.wire_size(0, 0, len(pay))
        ref = O.encode_batch(sess, np.zeros(1, np.uint32), np.array([5], np.uint64), np.zeros(1, np.uint8),
                             np.zeros(1, np.uint64), np.array([len(pay)], np.uint32),
                             np.frombuffer(pay, np.uint8), np.zeros(1, np.uint64), ws)
        assert got == bytes(ref[:ws]), rep
        # a fresh install leaves the send counter at 1 (zmqg_session_set_batch)
        ctx.session_set_batch(np.arange(S, dtype=np.uint32), precom, O.CLIENT_PREFIX, O.SERVER_PREFIX, stream=0)
        assert ctx.get_nonce(sid) == 1
