"""ctypes view of the CPU oracle (oracle/curve_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, as the checker.  The product never imports it.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libcurve_oracle.so")

CLIENT_PREFIX = b"CurveZMQMESSAGEC"  # reference src/curve_client.cpp:22-23
SERVER_PREFIX = b"CurveZMQMESSAGES"

_lib = None
_P = ctypes.c_void_p
_U64 = ctypes.c_uint64


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.oracle_splitmix_bytes.argtypes = [_U64, _P, _U64]
        L.oracle_hsalsa20.argtypes = [_P, _P, _P]
        L.oracle_salsa20_stream.argtypes = [_P, _U64, _P, _P]
        L.oracle_poly1305.argtypes = [_P, _P, _U64, _P]
        L.oracle_box_easy_afternm.argtypes = [_P, _P, _U64, _P, _P]
        L.oracle_box_open_easy_afternm.argtypes = [_P, _P, _U64, _P, _P]
        L.oracle_plaintext_header.argtypes = [_P, ctypes.c_uint8, ctypes.c_int]
        L.oracle_plaintext_header.restype = ctypes.c_uint32
        L.oracle_wire_size.argtypes = [ctypes.c_uint8, ctypes.c_int, _U64]
        L.oracle_wire_size.restype = _U64
        L.oracle_session_size.restype = _U64
        L.oracle_encode_batch.argtypes = [_P, _U64] + [_P] * 8
        L.oracle_decode_batch.argtypes = [_P, _P, _U64] + [_P] * 8
        L.oracle_bench_roundtrip.argtypes = [ctypes.c_int, ctypes.c_uint32, _P, _U64] + [_P] * 10
        L.oracle_bench_roundtrip.restype = ctypes.c_double
        L.oracle_x25519.argtypes = [_P, _P, _P]
        L.oracle_box_beforenm.argtypes = [_P, _P, _P]
        L.oracle_z85_encode.argtypes = [_P, _P, _U64]
        L.oracle_z85_decode.argtypes = [_P, _P, _U64]
        assert L.oracle_session_size() == 68
        _lib = L
    return _lib


def _buf(b):
    return ctypes.create_string_buffer(bytes(b), max(len(b), 1))


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


def splitmix_bytes(seed, n):
    out = ctypes.create_string_buffer(max(n, 1))
    lib().oracle_splitmix_bytes(seed, out, n)
    return out.raw[:n]


def hsalsa20(inp16, k):
    out = ctypes.create_string_buffer(32)
    lib().oracle_hsalsa20(out, _buf(inp16), _buf(k))
    return out.raw


def salsa20_stream(n, n8, k):
    out = ctypes.create_string_buffer(max(n, 1))
    lib().oracle_salsa20_stream(out, n, _buf(n8), _buf(k))
    return out.raw[:n]


def poly1305(m, k):
    out = ctypes.create_string_buffer(16)
    lib().oracle_poly1305(out, _buf(m), len(m), _buf(k))
    return out.raw


def box_easy_afternm(m, n, k):
    out = ctypes.create_string_buffer(len(m) + 16)
    lib().oracle_box_easy_afternm(out, _buf(m), len(m), _buf(n), _buf(k))
    return out.raw


def box_open_easy_afternm(c, n, k):
    out = ctypes.create_string_buffer(max(len(c), 1))
    rc = lib().oracle_box_open_easy_afternm(out, _buf(c), len(c), _buf(n), _buf(k))
    return rc, out.raw[: max(len(c) - 16, 0)]


def wire_size(flags, downgrade_sub, payload_len):
    return int(lib().oracle_wire_size(flags, int(downgrade_sub), payload_len))


SESSION_DTYPE = np.dtype([("precom", np.uint8, 32), ("enc_prefix", np.uint8, 16),
                          ("dec_prefix", np.uint8, 16), ("downgrade_sub", np.int32)])


def make_sessions(precoms, enc_prefix=CLIENT_PREFIX, dec_prefix=SERVER_PREFIX, downgrade_sub=False):
    s = np.zeros(len(precoms), SESSION_DTYPE)
    for i, p in enumerate(precoms):
        s[i]["precom"] = np.frombuffer(p, np.uint8)
        s[i]["enc_prefix"] = np.frombuffer(enc_prefix, np.uint8)
        s[i]["dec_prefix"] = np.frombuffer(dec_prefix, np.uint8)
        s[i]["downgrade_sub"] = int(downgrade_sub)
    return s


def encode_batch(sessions, sid, nonce, flags, in_off, length, inp, out_off, out_size):
    """Sequential curve_encoding_t::encode over a batch; returns the out buffer."""
    out = np.zeros(max(out_size, 1), np.uint8)
    sid = np.ascontiguousarray(sid, np.uint32)
    nonce = np.ascontiguousarray(nonce, np.uint64)
    flags = np.ascontiguousarray(flags, np.uint8)
    in_off = np.ascontiguousarray(in_off, np.uint64)
    length = np.ascontiguousarray(length, np.uint32)
    inp = np.ascontiguousarray(inp, np.uint8)
    out_off = np.ascontiguousarray(out_off, np.uint64)
    rc = lib().oracle_encode_batch(_ptr(sessions), len(sid), _ptr(sid), _ptr(nonce), _ptr(flags), _ptr(in_off),
                                   _ptr(length), _ptr(inp), _ptr(out_off), _ptr(out))
    assert rc == 0
    return out[:out_size]


def decode_batch(sessions, peer_nonce, sid, in_off, wire_len, inp, out_off, out_size):
    """Sequential curve_mechanism_base_t::decode over a batch (batch order).
    Returns (out, flags_out, status_out); peer_nonce (np.uint64) is updated."""
    n = len(sid)
    out = np.zeros(max(out_size, 1), np.uint8)
    flags_out = np.zeros(max(n, 1), np.uint8)
    status = np.zeros(max(n, 1), np.int32)
    sid = np.ascontiguousarray(sid, np.uint32)
    in_off = np.ascontiguousarray(in_off, np.uint64)
    wire_len = np.ascontiguousarray(wire_len, np.uint32)
    inp = np.ascontiguousarray(inp, np.uint8)
    out_off = np.ascontiguousarray(out_off, np.uint64)
    assert peer_nonce.dtype == np.uint64 and peer_nonce.flags["C_CONTIGUOUS"]
    rc = lib().oracle_decode_batch(_ptr(sessions), _ptr(peer_nonce), n, _ptr(sid), _ptr(in_off), _ptr(wire_len),
                                   _ptr(inp), _ptr(out_off), _ptr(out), _ptr(flags_out), _ptr(status))
    assert rc == 0
    return out[:out_size], flags_out[:n], status[:n]


def bench_roundtrip(use_sodium, nthreads, sessions, sid, nonce, flags, in_off, length, inp, wire_off, wire_size_total):
    """Timed CPU baseline; returns (seconds, ok_count) or (None, 0) when
    libsodium was requested but is not loadable."""
    sid = np.ascontiguousarray(sid, np.uint32)
    nonce = np.ascontiguousarray(nonce, np.uint64)
    flags = np.ascontiguousarray(flags, np.uint8)
    in_off = np.ascontiguousarray(in_off, np.uint64)
    length = np.ascontiguousarray(length, np.uint32)
    wire_off = np.ascontiguousarray(wire_off, np.uint64)
    wire = np.zeros(wire_size_total, np.uint8)
    back = np.zeros(len(inp), np.uint8)
    ok = ctypes.c_uint64(0)
    secs = lib().oracle_bench_roundtrip(int(use_sodium), nthreads, _ptr(sessions), len(sid), _ptr(sid), _ptr(nonce),
                                        _ptr(flags), _ptr(in_off), _ptr(length), _ptr(inp), _ptr(wire_off),
                                        _ptr(wire), _ptr(back), ctypes.byref(ok))
    if secs < 0:
        return None, 0
    return secs, ok.value


def z85_encode(data):
    """zmq_z85_encode (src/zmq_utils.cpp:100-124): the string, or None (EINVAL)."""
    data = bytes(data)
    out = ctypes.create_string_buffer(len(data) * 5 // 4 + 1)
    if lib().oracle_z85_encode(out, _buf(data), len(data)) != 0:
        return None
    return out.raw[:len(data) * 5 // 4]


def z85_decode(string, fill=0):
    """zmq_z85_decode (src/zmq_utils.cpp:131-180) of `string` (bytes, its
    length standing for strlen): (rc, out) with rc 0 or 22 (EINVAL) and out the
    len*4//5-byte destination, pre-filled with `fill`, as the call left it."""
    string = bytes(string)
    out = ctypes.create_string_buffer(bytes([fill]) * max(len(string) * 4 // 5, 1), max(len(string) * 4 // 5, 1))
    rc = lib().oracle_z85_decode(out, _buf(string), len(string))
    return rc, out.raw[:len(string) * 4 // 5]


def x25519(scalar, point):
    """crypto_scalarmult_curve25519 (libsodium 1.0.18 semantics): (rc, out)."""
    out = ctypes.create_string_buffer(32)
    rc = lib().oracle_x25519(out, _buf(bytes(scalar)), _buf(bytes(point)))
    return rc, out.raw


def box_beforenm(pk, sk):
    """crypto_box_beforenm(k, pk, sk): (rc, k or None)."""
    k = ctypes.create_string_buffer(32)
    rc = lib().oracle_box_beforenm(k, _buf(bytes(pk)), _buf(bytes(sk)))
    return rc, (k.raw if rc == 0 else None)
