#!/usr/bin/env python3
"""Generate tests/golden/box_vectors.json: the CURVE handshake boxes.

Test infrastructure only (runs in the build container, never on the GPU box).
Every box of the CURVE handshake is one libsodium 1.0.18 crypto_box or
crypto_secretbox call with its own key and 24-byte nonce; the vectors below
have the reference's shapes (nonce prefixes and plaintext sizes):

  HELLO     crypto_box(C', S), 64 zero bytes,        "CurveZMQHELLO---" || short nonce
            reference src/curve_client_tools.hpp:36-48
  WELCOME   crypto_box(S', C'), S' || cookie (128 B), "WELCOME-" || 16 random
            src/curve_server.cpp:222-236
  cookie    crypto_secretbox(K), C' || s' (64 B),     "COOKIE--" || 16 random
            src/curve_server.cpp:198-211
  vouch     crypto_box(C, S'), C' || S (64 B),        "VOUCH---" || 16 random
            src/curve_client_tools.hpp:130-143
  INITIATE  crypto_box(C', S'), C || vouch box || metadata, "CurveZMQINITIATE" || short
            src/curve_client_tools.hpp:160-180
  READY     crypto_box_afternm(precom), metadata,     "CurveZMQREADY---" || short
            src/curve_server.cpp:430-444

Bytes come from the container's libsodium (/opt/conda/lib/libsodium.so.23,
the library the reference links), loaded with ctypes.  Key pairs are the
reference tests' CURVE pairs (tests/test_sodium.cpp, tests/test_heartbeats.cpp,
taken from x25519_vectors.json) plus seeded random ones;
crypto_box_beforenm, crypto_box_easy_afternm and crypto_secretbox_easy give
the precomputed key and the box.  Output fields per item: kind, key (the
32-byte key the afternm form uses), nonce, m, c = tag || ciphertext, and for
crypto_box items pk/sk with key = crypto_box_beforenm(pk, sk).
"""
import ctypes
import json
import os
import random

HERE = os.path.dirname(os.path.abspath(__file__))
SODIUM_PATH = "/opt/conda/lib/libsodium.so.23"


def main():
    so = ctypes.CDLL(SODIUM_PATH)
    assert so.sodium_init() >= 0
    so.sodium_version_string.restype = ctypes.c_char_p
    ver = so.sodium_version_string().decode()
    assert ver == "1.0.18", ver

    def beforenm(pk, sk):
        k = ctypes.create_string_buffer(32)
        assert so.crypto_box_beforenm(k, pk, sk) == 0
        return k.raw

    def box_afternm(m, n, k):
        c = ctypes.create_string_buffer(len(m) + 16)
        assert so.crypto_box_easy_afternm(c, m, ctypes.c_ulonglong(len(m)), n, k) == 0
        return c.raw

    def box(m, n, pk, sk):
        c = ctypes.create_string_buffer(len(m) + 16)
        assert so.crypto_box_easy(c, m, ctypes.c_ulonglong(len(m)), n, pk, sk) == 0
        return c.raw

    def secretbox(m, n, k):
        c = ctypes.create_string_buffer(len(m) + 16)
        assert so.crypto_secretbox_easy(c, m, ctypes.c_ulonglong(len(m)), n, k) == 0
        return c.raw

    def public(sk):
        pk = ctypes.create_string_buffer(32)
        assert so.crypto_scalarmult_curve25519_base(pk, sk) == 0
        return pk.raw

    rnd = random.Random(0x5EED)
    rb = lambda n: bytes(rnd.getrandbits(8) for _ in range(n))
    # the reference tests' CURVE key pairs (tests/test_sodium.cpp,
    # tests/test_heartbeats.cpp), as decoded in x25519_vectors.json
    zp = json.load(open(os.path.join(HERE, "x25519_vectors.json")))["z85_pairs"]
    pairs = [(bytes.fromhex(p["public_hex"]), bytes.fromhex(p["secret_hex"])) for p in zp]
    for _ in range(4):
        sk = rb(32)
        pairs.append((public(sk), sk))
    short = lambda v: v.to_bytes(8, "big")  # src/wire.hpp put_uint64

    items = []

    def add_box(kind, m, n, pk, sk):
        k = beforenm(pk, sk)
        c = box(m, n, pk, sk)
        assert c == box_afternm(m, n, k)  # crypto_box = afternm(beforenm)
        items.append(dict(kind=kind, pk=pk.hex(), sk=sk.hex(), key=k.hex(), nonce=n.hex(), m=m.hex(), c=c.hex()))

    def add_secretbox(kind, m, n, k):
        c = secretbox(m, n, k)
        assert c == box_afternm(m, n, k)  # crypto_secretbox = crypto_box_afternm
        items.append(dict(kind=kind, key=k.hex(), nonce=n.hex(), m=m.hex(), c=c.hex()))

    for j in range(len(pairs)):
        client_pk, client_sk = pairs[j]
        server_pk, server_sk = pairs[(j + 1) % len(pairs)]
        cn_sk = rb(32)
        cn_pk = public(cn_sk)
        sn_sk = rb(32)
        sn_pk = public(sn_sk)
        cookie_key = rb(32)
        nonce = 1 + j
        add_box("hello", bytes(64), b"CurveZMQHELLO---" + short(nonce), server_pk, cn_sk)
        cookie_nonce = rb(16)
        cookie_pt = cn_pk + sn_sk
        add_secretbox("cookie", cookie_pt, b"COOKIE--" + cookie_nonce, cookie_key)
        cookie = cookie_nonce + secretbox(cookie_pt, b"COOKIE--" + cookie_nonce, cookie_key)
        add_box("welcome", sn_pk + cookie, b"WELCOME-" + rb(16), cn_pk, server_sk)
        vouch_nonce = rb(16)
        add_box("vouch", cn_pk + server_pk, b"VOUCH---" + vouch_nonce, sn_pk, client_sk)
        vouch = vouch_nonce + box(cn_pk + server_pk, b"VOUCH---" + vouch_nonce, sn_pk, client_sk)
        meta = b"\x0bSocket-Type\x00\x00\x00\x06DEALER" + b"\x08Identity\x00\x00\x00" + bytes([j * 7]) + rb(j * 7)
        add_box("initiate", client_pk + vouch + meta, b"CurveZMQINITIATE" + short(nonce + 1), sn_pk, cn_sk)
        precom = beforenm(cn_pk, sn_sk)
        c = box_afternm(meta, b"CurveZMQREADY---" + short(nonce), precom)
        items.append(dict(kind="ready", key=precom.hex(), nonce=(b"CurveZMQREADY---" + short(nonce)).hex(),
                          m=meta.hex(), c=c.hex()))
    # sizes around the window edges of the kernel (32 / 64-byte steps) and empty
    for L in (0, 1, 15, 16, 17, 31, 32, 33, 63, 64, 65, 95, 96, 97, 127, 128, 129, 255, 256, 257, 1000):
        add_secretbox("size%d" % L, rb(L), rb(24), rb(32))

    json.dump(dict(source="libsodium " + ver + " via ctypes (tests/golden/make_box_vectors.py)", items=items),
              open(os.path.join(HERE, "box_vectors.json"), "w"), indent=0)
    print(len(items), "items")


if __name__ == "__main__":
    main()
