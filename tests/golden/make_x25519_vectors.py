#!/usr/bin/env python3
"""Generates tests/golden/x25519_vectors.json (run in the build container,
not on the GPU box): expected outputs from libsodium 1.0.18 -- the
third-party library the reference calls for crypto_scalarmult /
crypto_box_beforenm (src/curve_client_tools.hpp:105,
src/curve_server.cpp:382-383, src/zmq_utils.cpp:222-245) -- loaded with
ctypes from the image's conda environment.  Inputs: the RFC 7748 section
5.2 / 6.1 vectors, the NaCl crypto_box key pair, the CURVE key pairs of the
reference's tests (tests/test_sodium.cpp, tests/test_heartbeats.cpp, as Z85),
the small-order points libsodium rejects, and seeded random keys."""
import ctypes
import json
import os
import random

L = ctypes.CDLL("/opt/conda/lib/libsodium.so.23")
assert L.sodium_init() >= 0
L.sodium_version_string.restype = ctypes.c_char_p


def scalarmult(n, p):
    q = ctypes.create_string_buffer(32)
    rc = L.crypto_scalarmult_curve25519(q, bytes(n), bytes(p))
    return rc, q.raw


def scalarmult_base(n):
    q = ctypes.create_string_buffer(32)
    rc = L.crypto_scalarmult_curve25519_base(q, bytes(n))
    return rc, q.raw


def beforenm(pk, sk):
    k = ctypes.create_string_buffer(b"\xaa" * 32, 32)
    rc = L.crypto_box_beforenm(k, bytes(pk), bytes(sk))
    return rc, k.raw


def z85_decode(s):
    out = ctypes.create_string_buffer(32)
    # the reference's zmq_z85_decode is restated by the oracle; libsodium has no Z85
    from oracle import oracle as O
    rc, key = O.z85_decode(s.encode())
    assert rc == 0
    return key


H = bytes.fromhex
rfc = [("a546e36bf0527c9d3b16154b82465edd62144c0ac1fc5a18506a2244ba449ac4",
        "e6db6867583030db3594c1a424b15f7c726624ec26b3353b10a903a6d0ab1c4c"),
       ("4b66e9d4d1b4673c5ad22691957d6af5c11b6421e0ea01d42ca4169e7918ba0d",
        "e5210f12786811d3f4b7959d0538ae2c31dbe7106fc03c3efc4cd549c715a493"),
       ("09" + "00" * 31, "09" + "00" * 31)]
alice_sk = "77076d0a7318a57d3c16c17251b26645df4c2f87ebc0992ab177fba51db92c2a"
bob_sk = "5dab087e624a8a4b79e17f8b83800ee66f3bb1292618b6fd1c2f8b27ff88e0eb"
small_order = ["00" * 32, "01" + "00" * 31,
               "e0eb7a7c3b41b8ae1656e3faf19fc46ada098deb9c32b1fd866205165f49b800",
               "5f9c95bca3508c24b1d0b1559c83ef5b04445cc4581c8e86d8224eddd09f1157",
               "ec" + "ff" * 30 + "7f", "ed" + "ff" * 30 + "7f", "ee" + "ff" * 30 + "7f"]
ref_pairs = [("D:)Q[IlAW!ahhC2ac:9*A}h:p?([4%wOTJ%JR%cs", "Yne@$w-vo<fVvi]a<NY6T1ed:M$fCG*[IaLV{hID"),
             ("JTKVSB%%)wK0E.X)V>+}o?pNmC{O&4W4b!Ni{Lh6", "rq:rM>}U?@Lns47E1%kR.o@n%FcmmsL/@{H8]yf7")]

v = {"source": "libsodium " + L.sodium_version_string().decode() + " (ctypes, build container); inputs: RFC 7748, "
               "NaCl crypto_box test keys, reference tests/test_sodium.cpp + tests/test_heartbeats.cpp key pairs",
     "scalarmult": [], "base": [], "beforenm": [], "z85_pairs": []}
for n, p in rfc:
    rc, q = scalarmult(H(n), H(p))
    v["scalarmult"].append({"scalar": n, "point": p, "rc": rc, "out": q.hex()})
for p in small_order:
    rc, q = scalarmult(H(alice_sk), H(p))
    v["scalarmult"].append({"scalar": alice_sk, "point": p, "rc": rc, "out": q.hex()})
    rc, k = beforenm(H(p), H(alice_sk))
    v["beforenm"].append({"pk": p, "sk": alice_sk, "rc": rc, "k": k.hex() if rc == 0 else None})
for sk in (alice_sk, bob_sk):
    rc, q = scalarmult_base(H(sk))
    v["base"].append({"scalar": sk, "rc": rc, "out": q.hex()})
rc, bob_pk = scalarmult_base(H(bob_sk))
rc, k = beforenm(bob_pk, H(alice_sk))
v["beforenm"].append({"pk": bob_pk.hex(), "sk": alice_sk, "rc": rc, "k": k.hex()})
for sec, pub in ref_pairs:
    sk = z85_decode(sec)
    rc, q = scalarmult_base(sk)
    v["z85_pairs"].append({"secret": sec, "public": pub, "public_hex": q.hex(), "secret_hex": sk.hex()})
rng = random.Random(0x25519)
for _ in range(48):
    sk = bytes(rng.randrange(256) for _ in range(32))
    pk = bytes(rng.randrange(256) for _ in range(32))  # any 32 bytes (bit 255 set half the time)
    rc, q = scalarmult(sk, pk)
    v["scalarmult"].append({"scalar": sk.hex(), "point": pk.hex(), "rc": rc, "out": q.hex()})
    rc, k = beforenm(pk, sk)
    v["beforenm"].append({"pk": pk.hex(), "sk": sk.hex(), "rc": rc, "k": k.hex() if rc == 0 else None})
    rc, q = scalarmult_base(sk)
    v["base"].append({"scalar": sk.hex(), "rc": rc, "out": q.hex()})
out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "x25519_vectors.json")
json.dump(v, open(out, "w"), indent=1)
print("wrote", out)
