"""ZMTP framing restatement for CURVE MESSAGE commands (SURVEY.md section 8f
row 2).  TEST INFRASTRUCTURE ONLY: the checker for zmqg_encode_zmtp /
zmqg_decode_zmtp; the product never imports it.  Pure-Python loops over
frames (small cases).

  frame(body)   the engine's ZMTP encoder on a boxed CURVE message, a msg_t
                with no MORE / COMMAND / sub-cancel flag
                (src/curve_mechanism_base.cpp:166-177): flags byte 0, or
                LARGE (2) when the body is longer than 255 bytes, then the
                size as one byte or a big-endian uint64 (src/v3_1_encoder.cpp:
                23-60, src/v2_encoder.cpp:23-60).
  parse(buf)    the ZMTP decoder loop (src/v2_decoder.cpp:35-140): flags
                byte, size (LARGE -> 8 bytes big endian), EMSGSIZE above
                maxmsgsize (:74-84), body; frame flags MORE -> msg_t more,
                COMMAND -> msg_t command.  It stops, as the engine does, after
                the first complete frame that is not a MESSAGE command (body
                shorter than 8 bytes or not starting with "\\x07MESSAGE"):
                the mechanism rejects it (src/curve_mechanism_base.cpp:80-97)
                and the engine drops the connection.
"""
import struct

MORE, LARGE, COMMAND = 1, 2, 4  # src/v2_protocol.hpp:14-19
EMSGSIZE = 90
MESSAGE = b"\x07MESSAGE"


def frame(body):
    body = bytes(body)
    if len(body) > 255:
        return bytes([LARGE]) + struct.pack(">Q", len(body)) + body
    return bytes([0, len(body)]) + body


def parse(buf, max_msg_size=-1, max_frames=None):
    """dict(frames=[(zmtp_flags, body_off, body_len)], consumed, error)."""
    buf = bytes(buf)
    n = len(buf)
    pos, frames, error = 0, [], 0
    while pos < n and (max_frames is None or len(frames) < max_frames):
        if pos + 2 > n:
            break
        f = buf[pos]
        if f & LARGE:
            if pos + 9 > n:
                break
            size, hdr = struct.unpack(">Q", buf[pos + 1:pos + 9])[0], 9
        else:
            size, hdr = buf[pos + 1], 2
        # max_msg_size: src/v2_decoder.cpp:74-84.  The 2^32 - 1 bound is this
        # library's restriction (32-bit frame lengths, include/zmqg_curve.h),
        # not the reference's: on LP64 its size_t check (:78) never fires.
        if (max_msg_size >= 0 and size > max_msg_size) or size > 0xFFFFFFFF:
            error = EMSGSIZE
            break
        if pos + hdr + size > n:
            break  # incomplete: wait for more bytes
        frames.append((f, pos + hdr, size))
        body = buf[pos + hdr:pos + hdr + size]
        pos += hdr + size
        if size < 8 or body[:8] != MESSAGE:
            break  # the mechanism rejects it; the connection ends here
    return dict(frames=frames, consumed=pos, error=error)


def msg_flags(zmtp_flags):
    """msg_t flags the decoder gives a frame (src/v2_decoder.cpp:35-41)."""
    return (1 if zmtp_flags & MORE else 0) | (2 if zmtp_flags & COMMAND else 0)
