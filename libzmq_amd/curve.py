"""Host-side mirror of libzmq's CURVE message codec over the MI355X C ABI.

Python view of include/zmqg_curve.h (libzmq_amd/libzmqg_curve.so).  Two
layers:

* ``CurveContext`` -- the batch API: one call encodes or decodes many frames
  held in device memory (torch tensors on the ctx's device) or host memory.
* ``CurveEncoding`` -- the single-message interface of the reference's
  ``curve_encoding_t`` (src/curve_mechanism_base.hpp:26-59): ``encode(msg)``,
  ``decode(msg) -> (rc, error_event_code)``, ``get_writable_precom_buffer``,
  ``set_peer_nonce``, ``get_and_inc_nonce``, with the reference's return /
  errno / error-event conventions (src/curve_mechanism_base.cpp:80-284).

There is no CPU fallback: if the HIP library is missing, importing this module
raises.  Build it with ``python -c "import __graft_entry__ as g; g.build()"``.
"""
import ctypes
import errno
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ZMQG_CURVE_LIB") or os.path.join(HERE, "libzmqg_curve.so")  # override: experiments

# include/zmq.h:424-437 (= ZMQG_ERR_* of include/zmqg_curve.h)
ERR_UNEXPECTED_COMMAND = 0x10000001
ERR_INVALID_SEQUENCE = 0x10000002
ERR_MALFORMED_UNSPECIFIED = 0x10000011
ERR_MALFORMED_MESSAGE = 0x10000012
ERR_CRYPTOGRAPHIC = 0x11000001
# library codes (zmqg_curve.h): unknown session; frame above the caller's max_len
ERR_SESSION = 0x7A000001
ERR_BOUND = 0x7A000002
# the largest max_len for which a call skips the large-frame kernels
MAX_LEN_FRAME_KERNEL_DECODE = 4608
MAX_LEN_FRAME_KERNEL_ENCODE = 4565

# src/msg.hpp:55-62
MORE, COMMAND, SUBSCRIBE, CANCEL = 1, 2, 12, 16
CLIENT_PREFIX = b"CurveZMQMESSAGEC"  # src/curve_client.cpp:22-23
SERVER_PREFIX = b"CurveZMQMESSAGES"

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"{LIB_PATH} is missing: the MI355X CURVE path has no CPU fallback. "
        "Build it with `make -C libzmq_amd/csrc` (hipcc --offload-arch=gfx950).")

_P = ctypes.c_void_p
_U64 = ctypes.c_uint64
_U32 = ctypes.c_uint32
_lib = ctypes.CDLL(LIB_PATH)
_lib.zmqg_abi_version.restype = ctypes.c_int
_lib.zmqg_ctx_create.argtypes = [ctypes.c_int, _U32, ctypes.POINTER(_P)]
_lib.zmqg_ctx_destroy.argtypes = [_P]
_lib.zmqg_session_set.argtypes = [_P, _U32, _P, _P, _P, ctypes.c_int, _U64]
_lib.zmqg_session_set_batch.argtypes = [_P, _U64, _P, _P, _P, _P, _P, _P, _P]
_lib.zmqg_session_set_batch_ex.argtypes = [_P, _U64, _P, _P, _P, _P, _P, _P, _P, _P]
_lib.zmqg_session_set_peer_nonce.argtypes = [_P, _U32, _U64]
_lib.zmqg_session_get_peer_nonce.argtypes = [_P, _U32, ctypes.POINTER(_U64)]
_lib.zmqg_session_set_nonce.argtypes = [_P, _U32, _U64]
_lib.zmqg_session_get_nonce.argtypes = [_P, _U32, ctypes.POINTER(_U64)]
_lib.zmqg_wire_size.argtypes = [ctypes.c_uint8, ctypes.c_int, _U64]
_lib.zmqg_wire_size.restype = _U64
_lib.zmqg_encode_batch.argtypes = [_P, _U64] + [_P] * 9
_lib.zmqg_decode_batch.argtypes = [_P, _U64] + [_P] * 9
OPT_NONCE_AUTO = 1  # zmqg_batch_opts.flags: encode nonces from the sessions' send counters
OPT_VERIFY_FIRST = 2  # zmqg_batch_opts.flags: decode writes out only after each frame's verdict
OPT_REPLAY_HOST = 4  # zmqg_batch_opts.flags: the caller applied the header / replay rules (verdict_in)
OPT_STREAM_OUT = 8  # zmqg_batch_opts.flags: decode output not cache-resident (whole-segment stores; a hint)


class BatchOpts(ctypes.Structure):  # zmqg_batch_opts
    _fields_ = [("size", _U32), ("flags", _U32), ("max_len", _U64), ("status_out", _P),
                ("session_max_out", _P), ("out_bytes", _U64), ("verdict_in", _P)]


_lib.zmqg_encode_batch_ex.argtypes = [_P, _U64] + [_P] * 8 + [ctypes.POINTER(BatchOpts), _P]
_lib.zmqg_decode_batch_ex.argtypes = [_P, _U64] + [_P] * 8 + [ctypes.POINTER(BatchOpts), _P]
_lib.zmqg_session_max_batch.argtypes = [_P, _U64] + [_P] * 6
_lib.zmqg_encode_host.argtypes = [_P, _U64, _P, _P, _P, _P, _P, _P, _U64, _P, _P, _U64]
_lib.zmqg_decode_host.argtypes = [_P, _U64, _P, _P, _P, _P, _U64, _P, _P, _U64, _P, _P]
_lib.zmqg_encode_msg.argtypes = [_P, _U32, _U64, ctypes.c_uint8, _P, _U32, _P]
_lib.zmqg_decode_msg.argtypes = [_P, _U32, _P, _U32, _P, _P, _P]
class ZmtpResult(ctypes.Structure):  # zmqg_zmtp_result
    _fields_ = [("frames", _U64), ("consumed", _U64), ("out_bytes", _U64), ("error", ctypes.c_int32),
                ("pad", ctypes.c_int32)]


_lib.zmqg_encode_zmtp.argtypes = [_P, _U64] + [_P] * 9
_lib.zmqg_decode_zmtp.argtypes = [_P, _U32, _P, _U64, ctypes.c_int64, _U64] + [_P] * 6 + [ctypes.POINTER(ZmtpResult),
                                                                                       _P]
_lib.zmqg_decode_zmtp_async.argtypes = [_P, _U32, _P, _U64, ctypes.c_int64, _U64] + [_P] * 8
_lib.zmqg_scalarmult_batch.argtypes = [_P, _U64] + [_P] * 5
_lib.zmqg_box_beforenm_batch.argtypes = [_P, _U64] + [_P] * 5
_lib.zmqg_box_afternm_batch.argtypes = [_P, _U64] + [_P] * 8
_lib.zmqg_box_open_afternm_batch.argtypes = [_P, _U64] + [_P] * 9
_lib.zmqg_z85_encode_batch.argtypes = [_P, _U64] + [_P] * 7
_lib.zmqg_z85_decode_batch.argtypes = [_P, _U64] + [_P] * 7
_lib.zmqg_host_alloc.argtypes = [_P, _U64, ctypes.POINTER(_P)]
_lib.zmqg_host_free.argtypes = [_P, _P]
_lib.zmqg_ctx_stream.argtypes = [_P, ctypes.POINTER(_P)]
_lib.zmqg_fence_record.argtypes = [_P, _P, ctypes.POINTER(_U64)]
_lib.zmqg_fence_query.argtypes = [_P, _U64]
_lib.zmqg_fence_wait.argtypes = [_P, _U64]
_lib.zmqg_ctx_set_profiling.argtypes = [_P, ctypes.c_int]
_lib.zmqg_ctx_get_profile.argtypes = [_P, ctypes.c_int, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_U64)]
_lib.zmqg_last_error.argtypes = [_P]
_lib.zmqg_last_error.restype = ctypes.c_char_p
_lib.zmqg_fence_record_notify.argtypes = [_P, _P, ctypes.c_int, ctypes.POINTER(_U64)]
_lib.zmqg_notify_quiesce.argtypes = [_P]
_lib.zmqg_build_id.restype = ctypes.c_char_p
assert _lib.zmqg_abi_version() == 5


def build_id():
    """(source id, commit) the loaded library was built from (zmqg_build_id)."""
    sid, _, commit = _lib.zmqg_build_id().decode().partition(" ")
    return sid, commit


def lib():
    return _lib


def wire_size(msg_flags, downgrade_sub, payload_len):
    """Encoded frame size (src/curve_mechanism_base.cpp:113-128, 169)."""
    return int(_lib.zmqg_wire_size(msg_flags & 0xFF, int(bool(downgrade_sub)), payload_len))


class ZmqgError(RuntimeError):
    pass


def _ptr(x):
    """Device/host address of a torch tensor or numpy array."""
    if x is None:
        return None
    if isinstance(x, np.ndarray):
        return ctypes.c_void_p(x.ctypes.data)
    return ctypes.c_void_p(x.data_ptr())


def _stream_handle(stream):
    if stream is None:
        import torch
        stream = torch.cuda.current_stream()
    if isinstance(stream, int):
        return ctypes.c_void_p(stream)
    return ctypes.c_void_p(stream.cuda_stream)


class CurveContext:
    """A zmqg_ctx: a session table on one GPU plus batch encode/decode."""

    def __init__(self, device=0, max_sessions=1):
        self._ctx = _P()
        self.device = device
        self.max_sessions = max_sessions
        self.downgrade = [False] * max_sessions
        rc = _lib.zmqg_ctx_create(device, max_sessions, ctypes.byref(self._ctx))
        if rc != 0:
            raise ZmqgError(f"zmqg_ctx_create failed: {rc}")

    def close(self):
        if self._ctx:
            _lib.zmqg_ctx_destroy(self._ctx)
            self._ctx = _P()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if rc != 0:
            raise ZmqgError(f"{what} failed: {rc} ({_lib.zmqg_last_error(self._ctx).decode()})")

    def session_set(self, sid, precom, enc_prefix, dec_prefix, downgrade_sub=False, peer_nonce=1):
        precom, enc_prefix, dec_prefix = bytes(precom), bytes(enc_prefix), bytes(dec_prefix)
        if len(precom) != 32 or len(enc_prefix) != 16 or len(dec_prefix) != 16:
            raise ValueError("precom must be 32 bytes and prefixes 16 bytes")
        self.downgrade[sid] = bool(downgrade_sub)
        self._check(_lib.zmqg_session_set(self._ctx, sid, precom, enc_prefix, dec_prefix, int(bool(downgrade_sub)),
                                          peer_nonce), "zmqg_session_set")

    def session_set_batch(self, sid, precom, enc_prefix, dec_prefix, downgrade=None, peer_nonce=None, stream=None,
                          send_nonce=None):
        """zmqg_session_set_batch(_ex): sid / downgrade / peer_nonce /
        send_nonce are host sequences (numpy-convertible), precom a device
        tensor of n x 32 bytes (e.g. box_beforenm_batch's k_out); asynchronous
        on `stream`."""
        sid = np.ascontiguousarray(sid, dtype=np.uint32)
        n = len(sid)
        enc_prefix, dec_prefix = bytes(enc_prefix), bytes(dec_prefix)
        if len(enc_prefix) != 16 or len(dec_prefix) != 16:
            raise ValueError("prefixes must be 16 bytes")
        dg = None if downgrade is None else np.ascontiguousarray(downgrade, dtype=np.uint8)
        pn = None if peer_nonce is None else np.ascontiguousarray(peer_nonce, dtype=np.uint64)
        sn = None if send_nonce is None else np.ascontiguousarray(send_nonce, dtype=np.uint64)
        if (dg is not None and len(dg) != n) or (pn is not None and len(pn) != n) or (sn is not None and len(sn) != n):
            raise ValueError("downgrade / peer_nonce / send_nonce must have one entry per session")
        self._check(_lib.zmqg_session_set_batch_ex(self._ctx, n, sid.ctypes.data, _ptr(precom), enc_prefix,
                                                   dec_prefix, None if dg is None else dg.ctypes.data,
                                                   None if pn is None else pn.ctypes.data,
                                                   None if sn is None else sn.ctypes.data, _stream_handle(stream)),
                    "zmqg_session_set_batch_ex")
        for i, s in enumerate(sid.tolist()):
            self.downgrade[s] = bool(dg[i]) if dg is not None else False

    def set_peer_nonce(self, sid, nonce):
        self._check(_lib.zmqg_session_set_peer_nonce(self._ctx, sid, nonce), "zmqg_session_set_peer_nonce")

    def get_peer_nonce(self, sid):
        v = _U64(0)
        self._check(_lib.zmqg_session_get_peer_nonce(self._ctx, sid, ctypes.byref(v)), "zmqg_session_get_peer_nonce")
        return v.value

    def set_nonce(self, sid, nonce):
        """The session's send counter (_cn_nonce) used by nonce_auto encodes."""
        self._check(_lib.zmqg_session_set_nonce(self._ctx, sid, nonce), "zmqg_session_set_nonce")

    def get_nonce(self, sid):
        v = _U64(0)
        self._check(_lib.zmqg_session_get_nonce(self._ctx, sid, ctypes.byref(v)), "zmqg_session_get_nonce")
        return v.value

    # ---- profiling hooks (HIP events around the body kernels) ----
    # zmqg_curve.h ZMQG_PROF_*: MAIN = the frame kernel (dominant kernel),
    # CALL = the whole batch call, BODY = the chunked body kernel (big frames)
    PROF_ENCODE_MAIN, PROF_DECODE_MAIN, PROF_ENCODE_CALL, PROF_DECODE_CALL = 0, 1, 2, 3
    PROF_ENCODE_BODY, PROF_DECODE_BODY = 4, 5

    def set_profiling(self, enable):
        self._check(_lib.zmqg_ctx_set_profiling(self._ctx, int(bool(enable))), "zmqg_ctx_set_profiling")

    def get_profile(self, kind):
        """(total_ms, launches) for `kind` since the last call; resets."""
        ms = ctypes.c_double(0)
        cnt = _U64(0)
        self._check(_lib.zmqg_ctx_get_profile(self._ctx, kind, ctypes.byref(ms), ctypes.byref(cnt)),
                    "zmqg_ctx_get_profile")
        return ms.value, cnt.value

    # ---- device-resident batches (torch tensors on self.device) ----
    # max_len / status_out / session_max_out: zmqg_batch_opts (the _ex calls)
    # nonce_auto: encode takes nonces from the sessions' send counters (nonce may be None)
    @staticmethod
    def _opts(max_len, status_out, session_max_out, nonce_auto=False, verify_first=False, out_bytes=0,
              verdict_in=None, stream_out=False):
        if (not max_len and status_out is None and session_max_out is None and not nonce_auto and not verify_first
                and verdict_in is None and not stream_out):
            return None
        fl = ((OPT_NONCE_AUTO if nonce_auto else 0) | (OPT_VERIFY_FIRST if verify_first else 0)
              | (OPT_REPLAY_HOST if verdict_in is not None else 0) | (OPT_STREAM_OUT if stream_out else 0))
        o = BatchOpts(ctypes.sizeof(BatchOpts), fl, int(max_len or 0), _ptr(status_out), _ptr(session_max_out),
                      int(out_bytes), _ptr(verdict_in))
        return ctypes.byref(o), o

    def encode_batch(self, sid, nonce, flags, in_off, length, inp, out_off, out, stream=None, max_len=0,
                     status_out=None, nonce_auto=False, stream_out=False):
        """stream_out: ZMQG_OPT_STREAM_OUT, the cache hint for outputs the
        device's caches do not hold."""
        n = int(sid.numel())
        o = self._opts(max_len, status_out, None, nonce_auto, stream_out=stream_out)
        self._check(_lib.zmqg_encode_batch_ex(self._ctx, n, _ptr(sid), _ptr(nonce), _ptr(flags), _ptr(in_off),
                                              _ptr(length), _ptr(inp), _ptr(out_off), _ptr(out),
                                              o[0] if o else None, _stream_handle(stream)), "zmqg_encode_batch")

    def decode_batch(self, sid, in_off, wire_len, inp, out_off, out, flags_out, status_out, stream=None, max_len=0,
                     session_max_out=None, verify_first=False, out_bytes=None, verdict_in=None, stream_out=False):
        """session_max_out: int64 tensor of max_sessions entries (device),
        receives each session's largest header-valid nonce of the batch.
        verify_first: ZMQG_OPT_VERIFY_FIRST (out receives only verified
        payloads and zeros; out's extent is taken from the tensor unless
        out_bytes is given).  verdict_in: int32 tensor (device) of the host's
        header / replay verdicts, ZMQG_OPT_REPLAY_HOST (with verify_first).
        stream_out: ZMQG_OPT_STREAM_OUT, the cache hint for outputs the device's
        caches do not hold."""
        n = int(sid.numel())
        if out_bytes is None:
            out_bytes = out.numel() * out.element_size() if verify_first else 0
        o = self._opts(max_len, None, session_max_out, verify_first=verify_first, out_bytes=out_bytes,
                       verdict_in=verdict_in, stream_out=stream_out)
        self._check(_lib.zmqg_decode_batch_ex(self._ctx, n, _ptr(sid), _ptr(in_off), _ptr(wire_len), _ptr(inp),
                                              _ptr(out_off), _ptr(out), _ptr(flags_out), _ptr(status_out),
                                              o[0] if o else None, _stream_handle(stream)), "zmqg_decode_batch")

    def session_max_batch(self, sid, in_off, wire_len, inp, session_max_out, stream=None):
        """Header pass: session_max_out (int64, max_sessions entries) = each
        session's largest header-valid nonce among the frames (sharded decode)."""
        n = int(sid.numel())
        self._check(_lib.zmqg_session_max_batch(self._ctx, n, _ptr(sid), _ptr(in_off), _ptr(wire_len), _ptr(inp),
                                                _ptr(session_max_out), _stream_handle(stream)),
                    "zmqg_session_max_batch")

    # ---- ZMTP framing on the device (device tensors) ----
    def encode_zmtp(self, sid, nonce, flags, in_off, length, inp, out, frame_off, stream=None):
        """Encode and frame n messages back to back in `out`; frame_off (n + 1
        int64) receives the frame offsets and the total."""
        n = int(sid.numel())
        self._check(_lib.zmqg_encode_zmtp(self._ctx, n, _ptr(sid), _ptr(nonce), _ptr(flags), _ptr(in_off),
                                          _ptr(length), _ptr(inp), _ptr(out), _ptr(frame_off),
                                          _stream_handle(stream)), "zmqg_encode_zmtp")

    def decode_zmtp(self, sid, inp, in_bytes, max_msg_size, max_frames, frame_in_off, frame_len, out_off, out,
                    flags_out, status_out, stream=None):
        """Parse and decode a received stream of one connection; returns
        dict(frames, consumed, out_bytes, error)."""
        r = ZmtpResult()
        self._check(_lib.zmqg_decode_zmtp(self._ctx, sid, _ptr(inp), in_bytes, max_msg_size, max_frames,
                                          _ptr(frame_in_off), _ptr(frame_len), _ptr(out_off), _ptr(out),
                                          _ptr(flags_out), _ptr(status_out), ctypes.byref(r),
                                          _stream_handle(stream)), "zmqg_decode_zmtp")
        return dict(frames=r.frames, consumed=r.consumed, out_bytes=r.out_bytes, error=r.error)

    def decode_zmtp_async(self, sid, inp, in_bytes, max_msg_size, max_frames, frame_in_off, frame_len, out_off, out,
                          flags_out, status_out, result, stream=None):
        """The same without synchronising: `result` is a device int64 tensor of
        4 entries (zmqg_zmtp_result: frames, consumed, out_bytes, error | pad)
        filled when the stream gets there; read it with zmtp_result()."""
        self._check(_lib.zmqg_decode_zmtp_async(self._ctx, sid, _ptr(inp), in_bytes, max_msg_size, max_frames,
                                                _ptr(frame_in_off), _ptr(frame_len), _ptr(out_off), _ptr(out),
                                                _ptr(flags_out), _ptr(status_out), _ptr(result),
                                                _stream_handle(stream)), "zmqg_decode_zmtp_async")

    @staticmethod
    def zmtp_result(result):
        r = result.cpu().numpy().view(np.uint64)
        return dict(frames=int(r[0]), consumed=int(r[1]), out_bytes=int(r[2]),
                    error=int(np.int32(r[3] & np.uint64(0xffffffff))))

    # ---- handshake key derivation (device tensors of n x 32 bytes) ----
    def scalarmult_batch(self, scalar, point, out, status_out, stream=None):
        """crypto_scalarmult_curve25519 per item; point None = the base point."""
        n = int(status_out.numel())
        self._check(_lib.zmqg_scalarmult_batch(self._ctx, n, _ptr(scalar), _ptr(point), _ptr(out), _ptr(status_out),
                                               _stream_handle(stream)), "zmqg_scalarmult_batch")

    def box_beforenm_batch(self, pk, sk, k_out, status_out, stream=None):
        """crypto_box_beforenm(k, pk, sk) per item."""
        n = int(status_out.numel())
        self._check(_lib.zmqg_box_beforenm_batch(self._ctx, n, _ptr(pk), _ptr(sk), _ptr(k_out), _ptr(status_out),
                                                 _stream_handle(stream)), "zmqg_box_beforenm_batch")

    # ---- handshake boxes: crypto_box_easy_afternm / _open_ per item ----
    def box_afternm_batch(self, key, nonce, in_off, length, inp, out_off, out, stream=None):
        """Seal: out[out_off[i]] = tag || ciphertext of in[in_off[i] .. +length[i]]
        under key[i] (32 B) and nonce[i] (24 B)."""
        n = int(in_off.numel())
        self._check(_lib.zmqg_box_afternm_batch(self._ctx, n, _ptr(key), _ptr(nonce), _ptr(in_off), _ptr(length),
                                                _ptr(inp), _ptr(out_off), _ptr(out), _stream_handle(stream)),
                    "zmqg_box_afternm_batch")

    def box_open_afternm_batch(self, key, nonce, in_off, length, inp, out_off, out, status_out, stream=None):
        """Open: length[i] = 16 + plaintext bytes; status 0 or -1."""
        n = int(in_off.numel())
        self._check(_lib.zmqg_box_open_afternm_batch(self._ctx, n, _ptr(key), _ptr(nonce), _ptr(in_off),
                                                     _ptr(length), _ptr(inp), _ptr(out_off), _ptr(out),
                                                     _ptr(status_out), _stream_handle(stream)),
                    "zmqg_box_open_afternm_batch")

    # ---- batched Z85 (zmq_z85_encode / zmq_z85_decode), device tensors ----
    def z85_encode_batch(self, in_off, length, inp, out_off, out, status_out, stream=None):
        n = int(in_off.numel())
        self._check(_lib.zmqg_z85_encode_batch(self._ctx, n, _ptr(in_off), _ptr(length), _ptr(inp), _ptr(out_off),
                                               _ptr(out), _ptr(status_out), _stream_handle(stream)),
                    "zmqg_z85_encode_batch")

    def z85_decode_batch(self, in_off, length, inp, out_off, out, status_out, stream=None):
        n = int(in_off.numel())
        self._check(_lib.zmqg_z85_decode_batch(self._ctx, n, _ptr(in_off), _ptr(length), _ptr(inp), _ptr(out_off),
                                               _ptr(out), _ptr(status_out), _stream_handle(stream)),
                    "zmqg_z85_decode_batch")

    # ---- host-memory batches (numpy), staged through pinned buffers ----
    def encode_host(self, sid, nonce, flags, in_off, length, inp, out_off, out_size):
        sid = np.ascontiguousarray(sid, np.uint32)
        nonce = np.ascontiguousarray(nonce, np.uint64)
        flags = np.ascontiguousarray(flags, np.uint8)
        in_off = np.ascontiguousarray(in_off, np.uint64)
        length = np.ascontiguousarray(length, np.uint32)
        inp = np.ascontiguousarray(inp, np.uint8)
        out_off = np.ascontiguousarray(out_off, np.uint64)
        out = np.zeros(max(out_size, 1), np.uint8)
        self._check(_lib.zmqg_encode_host(self._ctx, len(sid), _ptr(sid), _ptr(nonce), _ptr(flags), _ptr(in_off),
                                          _ptr(length), _ptr(inp), inp.nbytes, _ptr(out_off), _ptr(out), out.nbytes),
                    "zmqg_encode_host")
        return out[:out_size]

    def decode_host(self, sid, in_off, wire_len, inp, out_off, out_size):
        sid = np.ascontiguousarray(sid, np.uint32)
        in_off = np.ascontiguousarray(in_off, np.uint64)
        wire_len = np.ascontiguousarray(wire_len, np.uint32)
        inp = np.ascontiguousarray(inp, np.uint8)
        out_off = np.ascontiguousarray(out_off, np.uint64)
        n = len(sid)
        out = np.zeros(max(out_size, 1), np.uint8)
        fl = np.zeros(max(n, 1), np.uint8)
        st = np.zeros(max(n, 1), np.int32)
        self._check(_lib.zmqg_decode_host(self._ctx, n, _ptr(sid), _ptr(in_off), _ptr(wire_len), _ptr(inp),
                                          inp.nbytes, _ptr(out_off), _ptr(out), out.nbytes, _ptr(fl), _ptr(st)),
                    "zmqg_decode_host")
        return out[:out_size], fl[:n], st[:n]


    # ---- one message, host bytes (zmqg_encode_msg / zmqg_decode_msg) ----
    def encode_msg(self, sid, nonce, flags, payload):
        """The MESSAGE command for one message (bytes) on session sid."""
        p = np.frombuffer(bytes(payload), np.uint8)
        out = np.zeros(wire_size(flags, 1 if self.downgrade[sid] else 0, len(p)), np.uint8)
        self._check(_lib.zmqg_encode_msg(self._ctx, sid, nonce, flags, _ptr(p) if len(p) else None, len(p),
                                         _ptr(out)), "zmqg_encode_msg")
        return out.tobytes()

    def decode_msg(self, sid, wire):
        """(payload bytes or None, flags, status) of one received frame."""
        w = np.frombuffer(bytes(wire), np.uint8)
        out = np.zeros(max(len(w) - 33, 1), np.uint8)
        fl = np.zeros(1, np.uint8)
        st = np.zeros(1, np.int32)
        self._check(_lib.zmqg_decode_msg(self._ctx, sid, _ptr(w) if len(w) else None, len(w), _ptr(out), _ptr(fl),
                                         _ptr(st)), "zmqg_decode_msg")
        if st[0] != 0:
            return None, 0, int(st[0])
        return out[:len(w) - 33].tobytes(), int(fl[0]), 0


class Msg:
    """Minimal stand-in for zmq::msg_t on this path: bytes + flags byte
    (src/msg.hpp:55-62).  ``set_flags`` ORs, as msg_t::set_flags does."""

    def __init__(self, data=b"", flags=0):
        self.data = bytes(data)
        self.flags = flags

    def size(self):
        return len(self.data)

    def set_flags(self, f):
        self.flags |= f


class CurveEncoding:
    """curve_encoding_t (src/curve_mechanism_base.hpp:26-59) backed by the GPU.

    Each instance owns one session of a shared CurveContext (or its own)."""

    def __init__(self, encode_nonce_prefix, decode_nonce_prefix, downgrade_sub, ctx=None, sid=0):
        self._enc_prefix = bytes(encode_nonce_prefix)
        self._dec_prefix = bytes(decode_nonce_prefix)
        self._downgrade_sub = bool(downgrade_sub)
        self._ctx = ctx if ctx is not None else CurveContext(0, 1)
        self._sid = sid
        self._cn_nonce = 1  # src/curve_mechanism_base.cpp:59-60
        self._precom = bytearray(32)
        self._installed = None

    def get_writable_precom_buffer(self):
        self._installed = None
        return self._precom

    def _install(self, peer_nonce=None):
        key = bytes(self._precom)
        if self._installed != key:
            cur = 1 if peer_nonce is None else peer_nonce
            self._ctx.session_set(self._sid, key, self._enc_prefix, self._dec_prefix, self._downgrade_sub, cur)
            self._installed = key

    def get_and_inc_nonce(self):
        n = self._cn_nonce
        self._cn_nonce += 1
        return n

    def set_peer_nonce(self, nonce):
        self._install()
        self._ctx.set_peer_nonce(self._sid, nonce)

    def get_peer_nonce(self):
        self._install()
        return self._ctx.get_peer_nonce(self._sid)

    def encode(self, msg):
        """Replaces msg's content with the MESSAGE frame; returns 0."""
        self._install()
        nonce = self.get_and_inc_nonce()
        payload = np.frombuffer(msg.data, np.uint8) if msg.size() else np.zeros(1, np.uint8)
        ws = wire_size(msg.flags, self._downgrade_sub, msg.size())
        out = self._ctx.encode_host([self._sid], [nonce], [msg.flags], [0], [msg.size()], payload, [0], ws)
        msg.data = out.tobytes()
        msg.flags = 0  # the encoder output is a fresh msg_t (src/curve_mechanism_base.cpp:167-177)
        return 0

    def decode(self, msg):
        """Returns (rc, error_event_code): (0, None) and msg holds the payload
        with the decoded flags ORed in, or (-1, code) with errno EPROTO."""
        self._install()
        wire = np.frombuffer(msg.data, np.uint8) if msg.size() else np.zeros(1, np.uint8)
        plen = max(msg.size() - 33, 0)
        out, fl, st = self._ctx.decode_host([self._sid], [0], [msg.size()], wire, [0], plen)
        if st[0] != 0:
            return -1, int(st[0])
        msg.data = out[:plen].tobytes()
        msg.set_flags(int(fl[0]))
        return 0, None


EPROTO = errno.EPROTO
