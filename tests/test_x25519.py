"""Handshake key derivation in batches:
crypto_box_beforenm and crypto_scalarmult(_base) as the reference's handshake
calls them (src/curve_client_tools.hpp:105, src/curve_server.cpp:382-383,
src/zmq_utils.cpp:222-245).  CPU: the oracle (radix 2^51) against
tests/golden/x25519_vectors.json (libsodium 1.0.18 outputs for RFC 7748
vectors, the NaCl box keys, the reference's CURVE key pairs, small-order
points, random keys).  GPU: the device kernels against the fixture and the
oracle on a larger seeded batch."""
import json
import os

import numpy as np
import pytest

from oracle import oracle as O

V = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "x25519_vectors.json")))
H = bytes.fromhex


def test_oracle_scalarmult_vectors():
    for v in V["scalarmult"]:
        rc, out = O.x25519(H(v["scalar"]), H(v["point"]))
        assert rc == v["rc"] and out.hex() == v["out"]


def test_oracle_base_and_reference_key_pairs():
    nine = b"\x09" + bytes(31)
    for v in V["base"]:
        assert O.x25519(H(v["scalar"]), nine) == (0, H(v["out"]))
    for p in V["z85_pairs"]:  # zmq_curve_public(secret) == public (tests/test_sodium.cpp)
        rc, sk = O.z85_decode(p["secret"].encode())
        assert rc == 0
        rc, pk = O.x25519(sk, nine)
        assert rc == 0 and pk.hex() == p["public_hex"] and O.z85_encode(pk) == p["public"].encode()


def test_oracle_beforenm_vectors():
    nacl = "1b27556473e985d462cd51197a9a46c76009549eac6474f206c4ee0844f68389"  # SURVEY.md section 8c KAT
    assert any(v["k"] == nacl for v in V["beforenm"])
    for v in V["beforenm"]:
        rc, k = O.box_beforenm(H(v["pk"]), H(v["sk"]))
        assert rc == v["rc"]
        assert (k.hex() if k else None) == v["k"]


def _dev(torch, b):
    return torch.from_numpy(np.frombuffer(b, np.uint8).copy()).to("cuda")


@pytest.mark.gpu
def test_device_scalarmult_and_beforenm(torch_cuda, C):
    torch = torch_cuda
    rng = np.random.default_rng(7)
    ctx = C.CurveContext(0, 1)
    # fixture items plus random ones (checked against the oracle)
    sm = [(H(v["scalar"]), H(v["point"])) for v in V["scalarmult"]]
    sm += [(rng.integers(0, 256, 32, dtype=np.uint8).tobytes(), rng.integers(0, 256, 32, dtype=np.uint8).tobytes())
           for _ in range(200)]
    n = len(sm)
    out = torch.zeros(32 * n, dtype=torch.uint8, device="cuda")
    st = torch.full((n,), 7, dtype=torch.int32, device="cuda")
    ctx.scalarmult_batch(_dev(torch, b"".join(s for s, _ in sm)), _dev(torch, b"".join(p for _, p in sm)), out, st)
    torch.cuda.synchronize()
    o, s = out.cpu().numpy().tobytes(), st.cpu().numpy()
    for i, (sc, pt) in enumerate(sm):
        rc, ref = O.x25519(sc, pt)
        assert s[i] == rc and o[32 * i:32 * i + 32] == ref, i
    for i, v in enumerate(V["scalarmult"]):
        assert s[i] == v["rc"] and o[32 * i:32 * i + 32].hex() == v["out"]

    # base point (zmq_curve_public)
    bs = [H(v["scalar"]) for v in V["base"]] + [H(p["secret_hex"]) for p in V["z85_pairs"]]
    n = len(bs)
    out = torch.zeros(32 * n, dtype=torch.uint8, device="cuda")
    st = torch.full((n,), 7, dtype=torch.int32, device="cuda")
    ctx.scalarmult_batch(_dev(torch, b"".join(bs)), None, out, st)
    torch.cuda.synchronize()
    o = out.cpu().numpy().tobytes()
    assert (st.cpu().numpy() == 0).all()
    exp = [v["out"] for v in V["base"]] + [p["public_hex"] for p in V["z85_pairs"]]
    assert [o[32 * i:32 * i + 32].hex() for i in range(n)] == exp

    # beforenm: fixture + random, k untouched where it fails
    bf = [(H(v["pk"]), H(v["sk"])) for v in V["beforenm"]]
    bf += [(rng.integers(0, 256, 32, dtype=np.uint8).tobytes(), rng.integers(0, 256, 32, dtype=np.uint8).tobytes())
           for _ in range(200)]
    n = len(bf)
    k = torch.full((32 * n,), 0x5A, dtype=torch.uint8, device="cuda")
    st = torch.full((n,), 7, dtype=torch.int32, device="cuda")
    ctx.box_beforenm_batch(_dev(torch, b"".join(p for p, _ in bf)), _dev(torch, b"".join(s for _, s in bf)), k, st)
    torch.cuda.synchronize()
    o, s = k.cpu().numpy().tobytes(), st.cpu().numpy()
    fails = 0
    for i, (pk, sk) in enumerate(bf):
        rc, ref = O.box_beforenm(pk, sk)
        assert s[i] == rc, i
        assert o[32 * i:32 * i + 32] == (ref if rc == 0 else b"\x5a" * 32), i
        fails += rc != 0
    assert fails == 7  # the seven small-order points
