#!/usr/bin/env python3
"""Generate the golden CURVE MESSAGE vectors committed under tests/golden/.

Test infrastructure only: this script runs in the build container, never on the
GPU box, and nothing in the product imports it.

Where the bytes come from
-------------------------
* Crypto: libsodium 1.0.18 (conda package ``libsodium-1.0.18-h7b6447c_0``,
  ``/opt/conda/lib/libsodium.so.23``), the exact library the reference links
  for ``crypto_box_easy_afternm`` / ``crypto_box_open_easy_afternm``
  (reference ``src/curve_mechanism_base.cpp:172-174, 226-228``).  It is loaded
  with ctypes; no reference source is compiled or copied.
* Framing: ``curve_encoding_t::encode/decode/check_validity`` and
  ``mechanism_base_t::check_basic_command_structure`` restated below from
  reference ``src/curve_mechanism_base.cpp:80-284`` and
  ``src/mechanism_base.cpp:14-25``.  The framing restatement is pinned by the
  wire prefix the survey recorded from the compiled reference
  (checked in ``tests/test_golden.py``).

Output: ``curve_golden.json``: small cases as hex; large cases (64 KiB .. 3 MiB)
as a splitmix64 payload seed plus the wire's sha256, head and tail.
"""
import ctypes
import hashlib
import json
import os
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SODIUM_PATH = "/opt/conda/lib/libsodium.so.23"

# include/zmq.h:424-437
ERR_UNEXPECTED_COMMAND = 0x10000001
ERR_INVALID_SEQUENCE = 0x10000002
ERR_MALFORMED_UNSPECIFIED = 0x10000011
ERR_MALFORMED_MESSAGE = 0x10000012
ERR_CRYPTOGRAPHIC = 0x11000001

# src/msg.hpp:55-62, 16, 30-31
MORE, COMMAND, SUBSCRIBE, CANCEL, CMD_TYPE_MASK = 1, 2, 12, 16, 0x1C
SUB_CMD = b"\x09SUBSCRIBE"
CANCEL_CMD = b"\x06CANCEL"
MESSAGE_CMD = b"\x07MESSAGE"
CLIENT_PREFIX = b"CurveZMQMESSAGEC"  # src/curve_client.cpp:22-23
SERVER_PREFIX = b"CurveZMQMESSAGES"


def load_sodium():
    lib = ctypes.CDLL(SODIUM_PATH)
    assert lib.sodium_init() >= 0
    lib.sodium_version_string.restype = ctypes.c_char_p
    assert lib.sodium_version_string() == b"1.0.18", lib.sodium_version_string()
    return lib


S = load_sodium()
ull = ctypes.c_ulonglong


def buf(n):
    return (ctypes.c_ubyte * max(n, 1))()


def box_easy_afternm(m, n, k):
    out = buf(len(m) + 16)
    rc = S.crypto_box_easy_afternm(out, bytes(m), ull(len(m)), bytes(n), bytes(k))
    assert rc == 0
    return bytes(out)[: len(m) + 16]


def box_open_easy_afternm(c, n, k):
    out = buf(len(c))
    rc = S.crypto_box_open_easy_afternm(out, bytes(c), ull(len(c)), bytes(n), bytes(k))
    return rc, bytes(out)[: max(len(c) - 16, 0)]


def hsalsa20(inp16, k):
    out = buf(32)
    assert S.crypto_core_hsalsa20(out, bytes(inp16), bytes(k), None) == 0
    return bytes(out)


def salsa20_stream(nbytes, n8, k):
    out = buf(nbytes)
    assert S.crypto_stream_salsa20(out, ull(nbytes), bytes(n8), bytes(k)) == 0
    return bytes(out)[:nbytes]


def poly1305(m, k):
    out = buf(16)
    assert S.crypto_onetimeauth_poly1305(out, bytes(m), ull(len(m)), bytes(k)) == 0
    return bytes(out)


def beforenm(pk, sk):
    out = buf(32)
    assert S.crypto_box_beforenm(out, bytes(pk), bytes(sk)) == 0
    return bytes(out)


def scalarmult_base(sk):
    out = buf(32)
    assert S.crypto_scalarmult_curve25519_base(out, bytes(sk)) == 0
    return bytes(out)


# ---- deterministic bytes (splitmix64), mirrored by oracle/curve_oracle.c ----
def splitmix_bytes(seed, n):
    out = bytearray()
    x = seed & 0xFFFFFFFFFFFFFFFF
    while len(out) < n:
        x = (x + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
        z = x
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
        z ^= z >> 31
        out += struct.pack("<Q", z)
    return bytes(out[:n])


# ---- framing restatement: src/curve_mechanism_base.cpp:111-205 ----
def curve_encode(precom, enc_prefix, nonce, msg_flags, downgrade_sub, payload):
    is_sub = (msg_flags & CMD_TYPE_MASK) == SUBSCRIBE
    is_cancel = (msg_flags & CMD_TYPE_MASK) == CANCEL
    pt = bytearray([msg_flags & (MORE | COMMAND)])
    if is_sub or is_cancel:
        if downgrade_sub:
            pt.append(1 if is_sub else 0)
        else:
            pt[0] |= COMMAND
            pt += CANCEL_CMD if is_cancel else SUB_CMD
    pt += payload
    n24 = enc_prefix + struct.pack(">Q", nonce)
    box = box_easy_afternm(bytes(pt), n24, precom)
    return MESSAGE_CMD + struct.pack(">Q", nonce) + box


# ---- src/mechanism_base.cpp:14-25 + src/curve_mechanism_base.cpp:80-109, 207-284 ----
def curve_decode(precom, dec_prefix, peer_nonce, wire):
    """Returns (status, flags, payload, new_peer_nonce). status 0 = ok."""
    if len(wire) <= 1 or len(wire) <= wire[0]:
        return ERR_MALFORMED_UNSPECIFIED, 0, b"", peer_nonce
    if len(wire) < 8 or wire[:8] != MESSAGE_CMD:
        return ERR_UNEXPECTED_COMMAND, 0, b"", peer_nonce
    if len(wire) < 16 + 16 + 1:
        return ERR_MALFORMED_MESSAGE, 0, b"", peer_nonce
    nonce = struct.unpack(">Q", wire[8:16])[0]
    if nonce <= peer_nonce:
        return ERR_INVALID_SEQUENCE, 0, b"", peer_nonce
    peer_nonce = nonce  # set before the MAC check (:105)
    rc, pt = box_open_easy_afternm(wire[16:], dec_prefix + wire[8:16], precom)
    if rc != 0:
        return ERR_CRYPTOGRAPHIC, 0, b"", peer_nonce
    return 0, pt[0] & (MORE | COMMAND), pt[1:], peer_nonce


def main():
    H = lambda b: bytes(b).hex()
    doc = {
        "about": "golden CURVE MESSAGE vectors; crypto from libsodium 1.0.18 via ctypes, "
        "framing restated from reference src/curve_mechanism_base.cpp:80-284",
        "libsodium": "1.0.18",
    }

    # --- primitive-level vectors ---
    prim = {"hsalsa20": [], "salsa20": [], "poly1305": [], "box_afternm": []}
    for i in range(4):
        k = splitmix_bytes(100 + i, 32)
        inp = splitmix_bytes(200 + i, 16)
        prim["hsalsa20"].append({"k": H(k), "in": H(inp), "out": H(hsalsa20(inp, k))})
    for i, ln in enumerate([64, 130, 1000]):
        k = splitmix_bytes(300 + i, 32)
        n8 = splitmix_bytes(400 + i, 8)
        prim["salsa20"].append({"k": H(k), "n": H(n8), "len": ln, "out": H(salsa20_stream(ln, n8, k))})
    # Poly1305: lengths straddling the 16-byte block boundaries, plus the
    # carry-heavy all-0xff message / key corner cases.
    for i, ln in enumerate([0, 1, 15, 16, 17, 31, 32, 33, 63, 64, 65, 255, 256, 1000]):
        k = splitmix_bytes(500 + i, 32)
        m = splitmix_bytes(600 + i, ln)
        prim["poly1305"].append({"k": H(k), "m": H(m), "tag": H(poly1305(m, k))})
    for ln in [16, 17, 64, 1025]:
        k = b"\xff" * 32
        m = b"\xff" * ln
        prim["poly1305"].append({"k": H(k), "m": H(m), "tag": H(poly1305(m, k))})
        k = b"\x00" * 16 + b"\xff" * 16
        prim["poly1305"].append({"k": H(k), "m": H(m), "tag": H(poly1305(m, k))})
    # NaCl crypto_box KAT (tests/box.c of NaCl), re-derived from libsodium here.
    alicesk = bytes.fromhex("77076d0a7318a57d3c16c17251b26645df4c2f87ebc0992ab177fba51db92c2a")
    bobpk = bytes.fromhex("de9edb7d7b7dc1b4d35b61c2ece435373f8343c85b78674dadfc7e146f882b4f")
    nacl_k = beforenm(bobpk, alicesk)
    assert nacl_k.hex() == "1b27556473e985d462cd51197a9a46c76009549eac6474f206c4ee0844f68389"
    nacl_n = bytes.fromhex("69696ee955b62b73cd62bda875fc73d68219e0036b7a0b37")
    nacl_m = bytes.fromhex(
        "be075fc53c81f2d5cf141316ebeb0c7b5228c52a4c62cbd44b66849b64244ffc"
        "e5ecbaaf33bd751a1ac728d45e6c61296cdc3c01233561f41db66cce314adb31"
        "0e3be8250c46f06dceea3a7fa1348057e2f6556ad6b1318a024a838f21af1fde"
        "048977eb48f59ffd4924ca1c60902e52f0a089bc76897040e082f93776384864"
        "5e0705")
    nacl_c = box_easy_afternm(nacl_m, nacl_n, nacl_k)
    assert nacl_c[:16].hex() == "f3ffc7703f9400e52a7dfb4b3d3305d9"
    prim["box_afternm"].append({"k": H(nacl_k), "n": H(nacl_n), "m": H(nacl_m), "c": H(nacl_c), "name": "nacl_box_kat"})
    for i, ln in enumerate([1, 31, 32, 33, 64, 1025, 4097]):
        k = splitmix_bytes(700 + i, 32)
        n = splitmix_bytes(800 + i, 24)
        m = splitmix_bytes(900 + i, ln)
        prim["box_afternm"].append({"k": H(k), "n": H(n), "m": H(m), "c": H(box_easy_afternm(m, n, k))})
    # subkey hoist: box(m, prefix||n8, k) == secretbox under HSalsa20(k, prefix)
    doc["primitives"] = prim

    # --- survey pin: wire prefix recorded from the compiled reference ---
    precom = bytes(range(32))
    payload = bytes((i * 7 + 3) & 0xFF for i in range(1024))
    wire = curve_encode(precom, CLIENT_PREFIX, 1, 0, False, payload)
    assert wire[:36].hex() == ("074d455353414745" "0000000000000001"
                               "211ac25d7ffe5201b43880d3fb29fb06" "94b72981"), wire[:36].hex()
    doc["survey_pin"] = {"precom": H(precom), "prefix": CLIENT_PREFIX.decode(), "nonce": 1, "flags": 0,
                         "payload_rule": "(i*7+3)&0xff, 1024 bytes",
                         "reference_wire_prefix": wire[:36].hex(), "wire": H(wire)}

    # --- encode vectors: a1 (src/curve_mechanism_base.cpp:111-205) ---
    enc = []
    sizes = [0, 1, 15, 16, 17, 31, 32, 33, 63, 64, 65, 127, 128, 129, 255, 256, 257,
             1023, 1024, 1025, 2048, 4096]
    flag_cases = [(0, False), (MORE, False), (COMMAND, False), (MORE | COMMAND, False),
                  (SUBSCRIBE, False), (CANCEL, False), (SUBSCRIBE, True), (CANCEL, True),
                  (SUBSCRIBE | MORE, False), (4 | MORE, False), (0x80 | MORE, False)]
    case = 0
    for direction, pre in (("client", CLIENT_PREFIX), ("server", SERVER_PREFIX)):
        for si, sz in enumerate(sizes):
            fl, dg = flag_cases[(si + (direction == "server")) % len(flag_cases)]
            precom = splitmix_bytes(1000 + case, 32)
            nonce = [3, 2, 1, 0xFFFFFFFF, 0x100000000, 0xFFFFFFFFFFFFFFFF, 12345][case % 7]
            payload = splitmix_bytes(2000 + case, sz)
            w = curve_encode(precom, pre, nonce, fl, dg, payload)
            enc.append({"precom": H(precom), "prefix": pre.decode(), "nonce": nonce, "flags": fl,
                        "downgrade_sub": dg, "payload": H(payload), "wire": H(w)})
            case += 1
    for fl, dg in flag_cases:  # every flag case at one small size
        precom = splitmix_bytes(1000 + case, 32)
        payload = splitmix_bytes(2000 + case, 40)
        w = curve_encode(precom, CLIENT_PREFIX, 7, fl, dg, payload)
        enc.append({"precom": H(precom), "prefix": CLIENT_PREFIX.decode(), "nonce": 7, "flags": fl,
                    "downgrade_sub": dg, "payload": H(payload), "wire": H(w)})
        case += 1
    doc["encode"] = enc

    # --- decode sequences: a2-a4, including every failure path ---
    dec = []

    def seq(name, precom, prefix, peer0, wires):
        peer = peer0
        out = []
        for w in wires:
            st, fl, pl, peer = curve_decode(precom, prefix, peer, w)
            out.append({"wire": H(w), "status": st, "flags": fl, "payload": H(pl)})
        dec.append({"name": name, "precom": H(precom), "prefix": prefix.decode(), "peer_nonce": peer0,
                    "msgs": out, "peer_nonce_after": peer})

    pk = splitmix_bytes(5000, 32)
    good = [curve_encode(pk, CLIENT_PREFIX, 3 + i, [0, MORE, 0, COMMAND][i % 4], False,
                         splitmix_bytes(5100 + i, [0, 1, 31, 32, 33, 1024, 17, 64][i % 8]))
            for i in range(8)]
    seq("in_order", pk, CLIENT_PREFIX, 2, good)
    seq("unit_test_peer0", pk, CLIENT_PREFIX, 0, good[:2])  # unittest_curve_encoding.cpp:58
    seq("wrong_key", splitmix_bytes(5001, 32), CLIENT_PREFIX, 2, good[:3])
    seq("wrong_prefix", pk, SERVER_PREFIX, 2, good[:2])
    seq("replay", pk, CLIENT_PREFIX, 2, [good[0], good[1], good[1], good[0], good[2]])
    seq("reorder", pk, CLIENT_PREFIX, 2, [good[2], good[1], good[3], good[0], good[4]])
    seq("below_peer", pk, CLIENT_PREFIX, 4, good[:4])
    bad = []
    w = bytearray(good[5]); w[16] ^= 1; bad.append(bytes(w))            # tag bit flip
    w = bytearray(good[5]); w[40] ^= 0x80; bad.append(bytes(w))         # ciphertext bit flip
    w = bytearray(good[5]); w[-1] ^= 0x01; bad.append(bytes(w))         # last byte
    w = bytearray(good[5]); w[15] ^= 0x01; bad.append(bytes(w))         # nonce (still > peer)
    bad.append(good[5][:-1])                                             # truncated
    bad.append(good[5] + b"\x00")                                        # extended
    seq("mac_failures", pk, CLIENT_PREFIX, 2, bad)
    # MAC failure advances the peer nonce before the check (:105): a good
    # message with a lower nonce after it is then a sequence error.
    w = bytearray(good[4]); w[20] ^= 4
    seq("mac_fail_advances_peer", pk, CLIENT_PREFIX, 2, [bytes(w), good[3], good[5]])
    short = [b"", b"\x07", b"\x07MESS", b"\x07MESSAGE", b"\x07MESSAGE" + b"\x00" * 8,
             good[0][:32], good[0][:33], b"\x06MESSAGE" + good[0][8:], b"\x07MESSAGF" + good[0][8:],
             b"\x02ab", b"\x00\x00", b"\xff" * 40, b"\x08MESSAGES" + b"\x00" * 40]
    seq("malformed", pk, CLIENT_PREFIX, 2, short)
    # minimum valid: empty payload -> W = 33
    seq("empty_payload", pk, CLIENT_PREFIX, 2, [good[0]])
    doc["decode"] = dec

    # --- large cases: payload regenerated from splitmix64(seed); wire pinned by sha256 + tag ---
    large = []
    for i, (sz, fl) in enumerate([(65536, 0), (65536 + 13, MORE), (1 << 20, 0), (3 * (1 << 20) + 5, MORE)]):
        precom = splitmix_bytes(9000 + i, 32)
        payload = splitmix_bytes(9100 + i, sz)
        w = curve_encode(precom, CLIENT_PREFIX, 3 + i, fl, False, payload)
        large.append({"precom": H(precom), "prefix": CLIENT_PREFIX.decode(), "nonce": 3 + i, "flags": fl,
                      "payload_seed": 9100 + i, "payload_len": sz, "wire_len": len(w),
                      "wire_head": H(w[:64]), "wire_tail": H(w[-64:]),
                      "wire_sha256": hashlib.sha256(w).hexdigest()})
    doc["large"] = large

    with open(os.path.join(HERE, "curve_golden.json"), "w") as f:
        json.dump(doc, f, indent=0)
    print("wrote", len(enc), "encode vectors,", len(dec), "decode sequences")


if __name__ == "__main__":
    sys.exit(main())
