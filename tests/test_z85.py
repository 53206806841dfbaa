"""Batched Z85 key codec: zmq_z85_encode /
zmq_z85_decode, reference src/zmq_utils.cpp:100-180.

CPU: the oracle's restatement against the reference's own vectors
(tests/golden/z85_vectors.json, from tests/test_base85.cpp and the CURVE key
pairs of tests/test_sodium.cpp / test_heartbeats.cpp).  GPU: the device batch
kernels against the oracle, item by item, including what a failed decode
leaves in its destination."""
import json
import os

import numpy as np
import pytest

from oracle import oracle as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "z85_vectors.json")
V = json.load(open(GOLDEN))


def test_oracle_encode_vectors():
    for v in V["encode"]:
        got = O.z85_encode(bytes.fromhex(v["hex"]))
        assert got == (v["z85"].encode() if v["z85"] is not None else None)


def test_oracle_decode_vectors():
    for v in V["decode"]:
        rc, out = O.z85_decode(bytes.fromhex(v["z85_hex"]))
        assert rc == v["rc"]
        if rc == 0:
            assert out == bytes.fromhex(v["hex"])


def test_oracle_roundtrips():
    for h in V["encode_decode_roundtrip_hex"]:
        s = O.z85_encode(bytes.fromhex(h))
        assert O.z85_decode(s) == (0, bytes.fromhex(h))
    for s in V["decode_encode_roundtrip"]:
        rc, key = O.z85_decode(s.encode())
        assert rc == 0 and len(key) == 32
        assert O.z85_encode(key) == s.encode()


def _items(rng, n):
    """Encode inputs (lengths around multiples of 4) and decode strings
    (valid, wrong length, invalid characters, overflowing groups)."""
    alphabet = b"0123456789abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ.-:+=^!/*?&<>()[]{}@%$#"
    enc = [bytes(rng.integers(0, 256, int(rng.choice([0, 1, 3, 4, 8, 31, 32, 33, 64, 100])), dtype=np.uint8))
           for _ in range(n)]
    dec = []
    for k in range(n):
        r = rng.random()
        if r < 0.5:
            src = bytes(rng.integers(0, 256, 4 * int(rng.integers(1, 12)), dtype=np.uint8))
            s = bytearray(O.z85_encode(src))
            if r < 0.15:  # one invalid byte somewhere (groups before it still decode)
                s[int(rng.integers(0, len(s)))] = int(rng.choice([0, 3, 0x20, 0x22, 0x27, 0x2c, 0x7f, 0x80, 0xff]))
        elif r < 0.65:
            s = bytearray(alphabet[int(i)] for i in rng.integers(0, 85, int(rng.choice([0, 1, 4, 6, 9, 11]))))
        elif r < 0.8:  # groups near and above 0xffffffff
            s = bytearray(b"%nSc0" if rng.random() < 0.5 else b"%nSc1") + bytearray(b"HelloWorld")
            if rng.random() < 0.5:
                s = bytearray(b"HelloWorld") + bytearray(b"#####")
        else:
            s = bytearray(alphabet[int(i)] for i in rng.integers(0, 85, 5 * int(rng.integers(1, 10))))
        dec.append(bytes(s))
    dec += [bytes.fromhex(v["z85_hex"]) for v in V["decode"]] + [s.encode() for s in V["decode_encode_roundtrip"]]
    enc += [bytes.fromhex(v["hex"]) for v in V["encode"]]
    return enc, dec


def _pack(items):
    off = np.zeros(len(items), np.uint64)
    pos = 0
    for i, b in enumerate(items):
        off[i] = pos
        pos += len(b) + 8
    buf = np.zeros(max(pos, 1), np.uint8)
    for i, b in enumerate(items):
        buf[int(off[i]):int(off[i]) + len(b)] = np.frombuffer(b, np.uint8) if b else []
    return buf, off, np.array([len(b) for b in items], np.uint32)


@pytest.mark.gpu
def test_device_z85_matches_oracle(torch_cuda, C):
    torch = torch_cuda
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(85)
    enc, dec = _items(rng, 3000)
    ctx = C.CurveContext(0, 1)
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a).view(dt)).to(dev)

    # encode
    buf, off, ln = _pack(enc)
    ooff = np.zeros(len(enc), np.uint64)
    pos = 0
    for i, b in enumerate(enc):
        ooff[i] = pos
        pos += len(b) * 5 // 4 + 1 + 3
    out = torch.full((pos,), 0xAA, dtype=torch.uint8, device=dev)
    st = torch.full((len(enc),), -1, dtype=torch.int32, device=dev)
    ctx.z85_encode_batch(t(off, np.int64), t(ln, np.int32), t(buf, np.uint8), t(ooff, np.int64), out, st)
    torch.cuda.synchronize()
    out_h, st_h = out.cpu().numpy(), st.cpu().numpy()
    for i, b in enumerate(enc):
        ref = O.z85_encode(b)
        o = int(ooff[i])
        if ref is None:
            assert st_h[i] == 22 and (out_h[o:o + len(b) * 5 // 4 + 1] == 0xAA).all()
        else:
            assert st_h[i] == 0
            assert out_h[o:o + len(ref)].tobytes() == ref and out_h[o + len(ref)] == 0

    # decode
    buf, off, ln = _pack(dec)
    ooff = np.zeros(len(dec), np.uint64)
    pos = 0
    for i, s in enumerate(dec):
        ooff[i] = pos
        pos += len(s) * 4 // 5 + 4
    out = torch.full((max(pos, 1),), 0x5C, dtype=torch.uint8, device=dev)
    st = torch.full((len(dec),), -1, dtype=torch.int32, device=dev)
    ctx.z85_decode_batch(t(off, np.int64), t(ln, np.int32), t(buf, np.uint8), t(ooff, np.int64), out, st)
    torch.cuda.synchronize()
    out_h, st_h = out.cpu().numpy(), st.cpu().numpy()
    fails = 0
    for i, s in enumerate(dec):
        rc, ref = O.z85_decode(s, fill=0x5C)
        o = int(ooff[i])
        assert st_h[i] == rc, (i, s)
        assert out_h[o:o + len(ref)].tobytes() == ref, (i, s)
        fails += rc != 0
    assert 0 < fails < len(dec)
