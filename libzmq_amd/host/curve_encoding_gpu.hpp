// curve_encoding_gpu.hpp -- host-side mirror of libzmq's zmq::curve_encoding_t
// (reference src/curve_mechanism_base.hpp:26-59) running its MESSAGE AEAD on
// an MI355X through the C ABI in include/zmqg_curve.h.
//
// This is the piece a libzmq maintainer compiles into curve_mechanism_base_t
// (INTEGRATION.md): same constructor arguments, same encode/decode/nonce
// methods, same error convention (return -1, errno = EPROTO and the
// ZMQ_PROTOCOL_ERROR_ZMTP_* code in *error_event_code).  One object is one
// CURVE connection = one session slot of a shared zmqg_ctx.
//
// Messages are a minimal msg_t stand-in (bytes + msg_t flag bits), because
// zmq::msg_t is not part of this repository; the adapter only uses what the
// reference codec uses: data(), size(), flags() and, on encode, the
// subscribe/cancel/command bits (src/curve_mechanism_base.cpp:118-164).
//
// Batching: encode_many / decode_many submit the
// messages of many connections on one ctx as ONE batch call, which is how an
// I/O thread should drive the GPU; encode/decode are the n = 1 forms with
// the reference's per-message semantics.
#ifndef ZMQG_CURVE_ENCODING_GPU_HPP_INCLUDED
#define ZMQG_CURVE_ENCODING_GPU_HPP_INCLUDED

#include <stddef.h>
#include <stdint.h>

#include <vector>

#include "../../include/zmqg_curve.h"

namespace zmqg
{
// msg_t flag bits used on this path (reference src/msg.hpp:55-62)
enum
{
    msg_more = ZMQG_MSG_MORE,
    msg_command = ZMQG_MSG_COMMAND,
    msg_subscribe = ZMQG_MSG_SUBSCRIBE,
    msg_cancel = ZMQG_MSG_CANCEL,
};

struct msg_buf_t
{
    std::vector<uint8_t> bytes;
    uint8_t flags = 0;

    uint8_t *data () { return bytes.empty () ? nullptr : &bytes[0]; }
    size_t size () const { return bytes.size (); }
};

//  Per-I/O-thread device context and session slots for the drop-in
//  zmq::curve_encoding_t (zmq_curve_encoding.hpp).  libzmq runs each engine,
//  and so each curve_encoding_t, on one I/O thread for its whole life
//  (src/io_thread.hpp); a zmqg_ctx is externally synchronised, so each I/O
//  thread gets its own, created on first use on device ZMQG_DEVICE (default
//  0) with thread_sessions slots (or ZMQG_THREAD_SESSIONS, up to 2^24: each
//  slot is 64 bytes of device session table plus two 8-byte nonces).
//  acquire_session returns 0 and a free slot of the calling thread's ctx, or
//  -1 (errno ENOMEM: all slots in use, or EIO: the ctx could not be
//  created); release_session returns the slot.  The drop-in
//  zmq::curve_encoding_t turns a failure into a rejected connection, never an
//  abort (zmq_curve_encoding.hpp).
enum
{
    thread_sessions = 4096
};
zmqg_ctx *thread_ctx ();
int acquire_session (uint32_t *sid_);
void release_session (uint32_t sid_);

class curve_encoding_gpu_t
{
  public:
    typedef uint64_t nonce_t;

    //  ctx_: a context created with zmqg_ctx_create; sid_: this connection's
    //  session slot in it (< max_sessions).  Prefixes are the 16-byte
    //  "CurveZMQMESSAGEC"/"CurveZMQMESSAGES" strings
    //  (src/curve_client.cpp:22-23, src/curve_server.cpp:24-25).
    curve_encoding_gpu_t (zmqg_ctx *ctx_,
                          uint32_t sid_,
                          const char *encode_nonce_prefix_,
                          const char *decode_nonce_prefix_,
                          bool downgrade_sub_);

    //  src/curve_mechanism_base.cpp:111-205.  Replaces msg_'s bytes with the
    //  MESSAGE command and clears its flags, as msg_->move (msg_box) does.
    int encode (msg_buf_t *msg_);
    //  src/curve_mechanism_base.cpp:207-284.  On success msg_ holds the
    //  payload and the plaintext MORE/COMMAND bits are ORed into its flags.
    int decode (msg_buf_t *msg_, int *error_event_code_);

    //  The same on raw bytes, one message per device call with no
    //  intermediate buffers (zmqg_encode_msg / zmqg_decode_msg): encode_msg
    //  writes wire_size (flags_, len_) bytes to out_; decode_msg writes the
    //  wire_len_ - 33 payload bytes to out_ (which may be in_) and sets
    //  *flags_out_ to the plaintext MORE / COMMAND bits.  The MESSAGE path
    //  of zmq::curve_encoding_t (zmq_curve_encoding.hpp).
    size_t wire_size (uint8_t flags_, size_t len_) const
    {
        return zmqg_wire_size (flags_, _downgrade_sub ? 1 : 0, len_);
    }
    int encode_msg (const uint8_t *in_, size_t len_, uint8_t flags_, uint8_t *out_);
    int decode_msg (const uint8_t *in_,
                    size_t wire_len_,
                    uint8_t *out_,
                    uint8_t *flags_out_,
                    int *error_event_code_);

    //  Batched forms: one device submission for all messages, each message on
    //  its own connection's session.  Return 0, or -1 with errno set when the
    //  call itself failed; per-message results of decode_many are in
    //  status_out (0 or a ZMQ_PROTOCOL_ERROR_ZMTP_* code).
    static int encode_many (curve_encoding_gpu_t *const *enc_,
                            msg_buf_t *const *msgs_,
                            size_t n_);
    static int decode_many (curve_encoding_gpu_t *const *dec_,
                            msg_buf_t *const *msgs_,
                            size_t n_,
                            int32_t *status_out_);

    //  src/curve_mechanism_base.hpp:36-42
    uint8_t *get_writable_precom_buffer () { return _cn_precom; }
    const uint8_t *get_precom_buffer () const { return _cn_precom; }
    nonce_t get_and_inc_nonce () { return _cn_nonce++; }
    void set_peer_nonce (nonce_t peer_nonce_);
    nonce_t get_peer_nonce () const;

    //  The header rules and the replay rule of one received frame, in
    //  order, on the host: check_basic_command_structure
    //  (src/mechanism_base.cpp:14-25) and check_validity
    //  (src/curve_mechanism_base.cpp:80-106).  0, or the
    //  ZMQ_PROTOCOL_ERROR_ZMTP_* code; *peer_ advances before the MAC, as
    //  set_peer_nonce does there.
    static int32_t frame_verdict (const uint8_t *wire_,
                                  size_t size_,
                                  uint64_t *peer_);

  private:
    friend class curve_batcher_t;

    //  installs the session on the device when the precom buffer changed
    int sync_session ();

    //  The connection's peer nonce.  The device's copy is advanced by the
    //  calls that apply the replay rule there (decode_msg, decode_many); a
    //  batch under ZMQG_OPT_REPLAY_HOST (curve_batcher_t) advances the host's
    //  copy instead.  Each side catches up from the other before it is used.
    enum peer_state_t
    {
        peer_synced,      //  _peer == the device's
        peer_host_ahead,  //  _peer is newer: set the device's before use
        peer_device_ahead //  the device's is newer: read it before use
    };
    //  the host copy, current (reads the device's when that is ahead);
    //  -1 when the device cannot be read
    int host_peer (uint64_t **peer_);
    //  the device copy, current (writes _peer when the host is ahead)
    int device_peer ();

    zmqg_ctx *const _ctx;
    const uint32_t _sid;
    uint8_t _encode_nonce_prefix[16];
    uint8_t _decode_nonce_prefix[16];
    nonce_t _cn_nonce;
    uint8_t _cn_precom[32];
    uint8_t _installed_precom[32];
    bool _installed;
    const bool _downgrade_sub;
    uint64_t _peer;
    peer_state_t _peer_state;

    curve_encoding_gpu_t (const curve_encoding_gpu_t &);
    curve_encoding_gpu_t &operator= (const curve_encoding_gpu_t &);
};
}

#endif
