"""Pin the CPU oracle against the golden vectors (tests/golden/curve_golden.json).

The vectors come from libsodium 1.0.18 (the library the reference links) and
the framing of reference src/curve_mechanism_base.cpp:80-284; the survey pin
is the wire prefix recorded from the compiled reference itself.
"""
import hashlib
import json
import os
import struct

import numpy as np
import pytest

from oracle import oracle as O

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "curve_golden.json")))
H = bytes.fromhex


def test_splitmix_matches_generator():
    # tests/golden/make_golden.py::splitmix_bytes, first 16 bytes of seed 0
    x = 0
    out = b""
    for _ in range(2):
        x = (x + 0x9E3779B97F4A7C15) & (2**64 - 1)
        z = x
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & (2**64 - 1)
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & (2**64 - 1)
        z ^= z >> 31
        out += struct.pack("<Q", z)
    assert O.splitmix_bytes(0, 16) == out
    assert O.splitmix_bytes(0, 13) == out[:13]


@pytest.mark.parametrize("v", GOLDEN["primitives"]["hsalsa20"])
def test_hsalsa20(v):
    assert O.hsalsa20(H(v["in"]), H(v["k"])).hex() == v["out"]


@pytest.mark.parametrize("v", GOLDEN["primitives"]["salsa20"])
def test_salsa20(v):
    assert O.salsa20_stream(v["len"], H(v["n"]), H(v["k"])).hex() == v["out"]


@pytest.mark.parametrize("v", GOLDEN["primitives"]["poly1305"])
def test_poly1305(v):
    assert O.poly1305(H(v["m"]), H(v["k"])).hex() == v["tag"]


@pytest.mark.parametrize("v", GOLDEN["primitives"]["box_afternm"])
def test_box_afternm(v):
    c = O.box_easy_afternm(H(v["m"]), H(v["n"]), H(v["k"]))
    assert c.hex() == v["c"]
    rc, m = O.box_open_easy_afternm(c, H(v["n"]), H(v["k"]))
    assert rc == 0 and m.hex() == v["m"]
    bad = bytearray(c)
    bad[-1] ^= 1
    assert O.box_open_easy_afternm(bytes(bad), H(v["n"]), H(v["k"]))[0] == -1


def test_nacl_kat_present():
    kat = [v for v in GOLDEN["primitives"]["box_afternm"] if v.get("name") == "nacl_box_kat"][0]
    # NaCl tests/box.c expected output (tag then first ciphertext bytes)
    assert kat["c"].startswith("f3ffc7703f9400e52a7dfb4b3d3305d9" "8e993b9f48681273c29650ba32fc76ce")


def _encode_one(v, out_align=0):
    sess = O.make_sessions([H(v["precom"])], enc_prefix=v["prefix"].encode(), downgrade_sub=v["downgrade_sub"])
    payload = np.frombuffer(H(v["payload"]), np.uint8)
    wl = O.wire_size(v["flags"], v["downgrade_sub"], len(payload))
    return O.encode_batch(sess, [0], [v["nonce"]], [v["flags"]], [0], [len(payload)], payload if len(payload) else
                          np.zeros(1, np.uint8), [out_align], wl + out_align)[out_align:].tobytes()


def test_survey_pin_reference_wire_prefix():
    v = GOLDEN["survey_pin"]
    payload = bytes((i * 7 + 3) & 0xFF for i in range(1024))
    vv = dict(precom=v["precom"], prefix=v["prefix"], nonce=1, flags=0, downgrade_sub=False, payload=payload.hex())
    wire = _encode_one(vv)
    assert wire[:36].hex() == v["reference_wire_prefix"]
    assert wire.hex() == v["wire"]


@pytest.mark.parametrize("idx", range(len(GOLDEN["encode"])))
def test_encode_vectors(idx):
    v = GOLDEN["encode"][idx]
    assert _encode_one(v).hex() == v["wire"]
    assert _encode_one(v, out_align=5).hex() == v["wire"]


@pytest.mark.parametrize("seq", GOLDEN["decode"], ids=[s["name"] for s in GOLDEN["decode"]])
def test_decode_sequences(seq):
    msgs = seq["msgs"]
    sess = O.make_sessions([H(seq["precom"])], dec_prefix=seq["prefix"].encode())
    wires = [H(m["wire"]) for m in msgs]
    in_off = np.cumsum([0] + [len(w) for w in wires])[:-1]
    inp = np.frombuffer(b"".join(wires) + b"\0", np.uint8)
    plen = [max(len(w) - 33, 0) for w in wires]
    out_off = np.cumsum([0] + plen)[:-1]
    peer = np.array([seq["peer_nonce"]], np.uint64)
    out, fl, st = O.decode_batch(sess, peer, [0] * len(wires), in_off, [len(w) for w in wires], inp, out_off,
                                 sum(plen))
    for i, m in enumerate(msgs):
        assert st[i] == m["status"], (i, hex(st[i]), hex(m["status"]))
        if m["status"] == 0:
            assert fl[i] == m["flags"]
            assert out[out_off[i]:out_off[i] + plen[i]].tobytes().hex() == m["payload"]
    assert int(peer[0]) == seq["peer_nonce_after"]


@pytest.mark.parametrize("v", GOLDEN["large"][:3], ids=lambda v: str(v["payload_len"]))
def test_large_vectors(v):
    payload = np.frombuffer(O.splitmix_bytes(v["payload_seed"], v["payload_len"]), np.uint8)
    sess = O.make_sessions([H(v["precom"])], enc_prefix=v["prefix"].encode())
    wire = O.encode_batch(sess, [0], [v["nonce"]], [v["flags"]], [0], [len(payload)], payload, [0],
                          v["wire_len"]).tobytes()
    assert wire[:64].hex() == v["wire_head"] and wire[-64:].hex() == v["wire_tail"]
    assert hashlib.sha256(wire).hexdigest() == v["wire_sha256"]
