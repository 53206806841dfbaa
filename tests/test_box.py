"""Handshake boxes: zmqg_box_afternm_batch /
zmqg_box_open_afternm_batch against the oracle and libsodium 1.0.18 vectors
of the CURVE handshake's shapes (tests/golden/box_vectors.json, made by
tests/golden/make_box_vectors.py): HELLO, WELCOME, cookie, vouch, INITIATE,
READY (reference src/curve_client_tools.hpp:36-180,
src/curve_server.cpp:198-444) and edge sizes."""
import json
import os

import numpy as np
import pytest

from oracle import oracle as O
from tests.helpers import pack

VEC = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "box_vectors.json")))["items"]
H = bytes.fromhex


def test_oracle_pinned_by_box_vectors():
    for v in VEC:
        k, n, m, c = H(v["key"]), H(v["nonce"]), H(v["m"]), H(v["c"])
        assert O.box_easy_afternm(m, n, k) == c, v["kind"]
        rc, back = O.box_open_easy_afternm(c, n, k)
        assert rc == 0 and back == m
        if "pk" in v:
            rc, kk = O.box_beforenm(H(v["pk"]), H(v["sk"]))
            assert rc == 0 and kk == k


def _dev(torch, a):
    a = np.ascontiguousarray(a)
    if a.dtype == np.uint64:
        a = a.view(np.int64)
    elif a.dtype == np.uint32:
        a = a.view(np.int32)
    return torch.from_numpy(a.copy()).to("cuda")


def _seal(torch, C, keys, nonces, msgs, rng=None, gap=0):
    ctx = C.CurveContext(0, 1)
    inp, in_off = pack(msgs, rng, gap)
    outs = [bytes(len(m) + 16) for m in msgs]
    _, out_off = pack(outs, rng, gap)
    total = int(out_off[-1]) + len(outs[-1]) if msgs else 1
    out = torch.zeros(max(total, 1), dtype=torch.uint8, device="cuda")
    ctx.box_afternm_batch(_dev(torch, np.frombuffer(b"".join(keys), np.uint8)),
                          _dev(torch, np.frombuffer(b"".join(nonces), np.uint8)), _dev(torch, in_off),
                          _dev(torch, np.array([len(m) for m in msgs], np.uint32)), _dev(torch, inp),
                          _dev(torch, out_off), out)
    torch.cuda.synchronize()
    o = out.cpu().numpy().tobytes()
    return [o[int(a):int(a) + len(m) + 16] for a, m in zip(out_off, msgs)]


def _open(torch, C, keys, nonces, boxes, rng=None, gap=0, fill=0x77):
    ctx = C.CurveContext(0, 1)
    inp, in_off = pack(boxes, rng, gap)
    plain = [bytes(max(len(b) - 16, 0)) for b in boxes]
    _, out_off = pack(plain, rng, gap)
    total = int(out_off[-1]) + len(plain[-1])
    out = torch.full((max(total, 1),), fill, dtype=torch.uint8, device="cuda")
    st = torch.full((len(boxes),), 7, dtype=torch.int32, device="cuda")
    ctx.box_open_afternm_batch(_dev(torch, np.frombuffer(b"".join(keys), np.uint8)),
                               _dev(torch, np.frombuffer(b"".join(nonces), np.uint8)), _dev(torch, in_off),
                               _dev(torch, np.array([len(b) for b in boxes], np.uint32)), _dev(torch, inp),
                               _dev(torch, out_off), out, st)
    torch.cuda.synchronize()
    o = out.cpu().numpy().tobytes()
    return [o[int(a):int(a) + len(p)] for a, p in zip(out_off, plain)], st.cpu().numpy()


@pytest.mark.gpu
def test_box_vectors_seal_and_open(torch_cuda, C):
    keys = [H(v["key"]) for v in VEC]
    nonces = [H(v["nonce"]) for v in VEC]
    msgs = [H(v["m"]) for v in VEC]
    got = _seal(torch_cuda, C, keys, nonces, msgs, np.random.default_rng(1), 5)
    for g, v in zip(got, VEC):
        assert g == H(v["c"]), v["kind"]
    back, st = _open(torch_cuda, C, keys, nonces, [H(v["c"]) for v in VEC], np.random.default_rng(2), 7)
    assert (st == 0).all()
    assert back == msgs


@pytest.mark.gpu
def test_box_chain_from_key_pairs(torch_cuda, C):
    """crypto_box(pk, sk) = zmqg_box_beforenm_batch then zmqg_box_afternm_batch."""
    torch = torch_cuda
    items = [v for v in VEC if "pk" in v]
    pk = _dev(torch, np.frombuffer(b"".join(H(v["pk"]) for v in items), np.uint8))
    sk = _dev(torch, np.frombuffer(b"".join(H(v["sk"]) for v in items), np.uint8))
    k = torch.zeros(32 * len(items), dtype=torch.uint8, device="cuda")
    st = torch.zeros(len(items), dtype=torch.int32, device="cuda")
    C.CurveContext(0, 1).box_beforenm_batch(pk, sk, k, st)
    torch.cuda.synchronize()
    assert (st.cpu().numpy() == 0).all()
    kb = k.cpu().numpy().tobytes()
    keys = [kb[32 * i:32 * i + 32] for i in range(len(items))]
    assert keys == [H(v["key"]) for v in items]
    got = _seal(torch, C, keys, [H(v["nonce"]) for v in items], [H(v["m"]) for v in items])
    assert got == [H(v["c"]) for v in items]


@pytest.mark.gpu
def test_box_random_vs_oracle(torch_cuda, C):
    rng = np.random.default_rng(3)
    n = 700
    sizes = [int(x) for x in rng.choice([0, 1, 16, 31, 32, 33, 64, 96, 200, 511, 600, 4100], n)]
    keys = [rng.integers(0, 256, 32, dtype=np.uint8).tobytes() for _ in range(n)]
    nonces = [rng.integers(0, 256, 24, dtype=np.uint8).tobytes() for _ in range(n)]
    msgs = [rng.integers(0, 256, s, dtype=np.uint8).tobytes() for s in sizes]
    got = _seal(torch_cuda, C, keys, nonces, msgs, rng, 9)
    assert got == [O.box_easy_afternm(m, nn, k) for m, nn, k in zip(msgs, nonces, keys)]
    back, st = _open(torch_cuda, C, keys, nonces, got, rng, 3)
    assert (st == 0).all() and back == msgs


@pytest.mark.gpu
def test_box_open_rejects(torch_cuda, C):
    """A flipped bit anywhere (tag or ciphertext), a wrong key, a wrong nonce
    or a box shorter than the tag: status -1 and a zero-filled plaintext."""
    rng = np.random.default_rng(4)
    base = [v for v in VEC if v["kind"] in ("hello", "welcome", "initiate", "ready", "size1", "size0")]
    keys, nonces, boxes, expect = [], [], [], []
    for v in base:
        k, nn, c = H(v["key"]), H(v["nonce"]), bytearray(H(v["c"]))
        for pos in sorted({0, 15, 16, len(c) - 1}):
            if pos < len(c):
                t = bytearray(c)
                t[pos] ^= 1 << int(rng.integers(0, 8))
                keys.append(k), nonces.append(nn), boxes.append(bytes(t)), expect.append(-1)
        keys.append(bytes(31) + b"\x01"), nonces.append(nn), boxes.append(bytes(c)), expect.append(-1)
        keys.append(k), nonces.append(nn[:-1] + bytes([nn[-1] ^ 0x80])), boxes.append(bytes(c)), expect.append(-1)
        keys.append(k), nonces.append(nn), boxes.append(bytes(c)), expect.append(0)
    for short in (0, 1, 15):
        keys.append(bytes(32)), nonces.append(bytes(24)), boxes.append(bytes(short)), expect.append(-1)
    back, st = _open(torch_cuda, C, keys, nonces, boxes, rng, 4)
    assert list(st) == expect
    for b, e, box, k, nn in zip(back, expect, boxes, keys, nonces):
        if e != 0:
            assert b == bytes(len(b))
        else:
            assert b == O.box_open_easy_afternm(box, nn, k)[1]
