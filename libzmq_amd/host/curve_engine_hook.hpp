// curve_engine_hook.hpp -- the stream-engine side of the batched CURVE
// codec: what src/stream_engine_base.cpp's two
// codec call sites and the I/O thread's poller loop become when the
// MESSAGE AEAD runs on the GPU in batches.
//
// The reference engine calls its mechanism synchronously, one message at a
// time, inside its event handlers:
//   out_event (src/stream_engine_base.cpp:331-348): _next_msg =
//     pull_and_encode (:607-616) pulls a message from the session and
//     encodes it, until out_batch_size bytes are queued for the socket;
//   in_event_internal (:281-291): for every frame the ZMTP decoder
//     completes, _process_msg = decode_and_push (:618-647) decodes it and
//     pushes it to the session.
// With curve_batcher_t (one per I/O thread) the codec becomes asynchronous.
// The two objects here carry the rest of the change:
//
//   curve_io_hook_t       one per I/O thread: owns the batcher, routes every
//                         result back to its connection (the sink), and is
//                         driven once per poller iteration (iteration(): the
//                         batches the engines queued are launched, finished
//                         ones delivered -- io_thread_t::in_event's place).
//   curve_engine_link_t   one per engine (connection): replaces the two
//                         mechanism calls.
//     out side   submit_send()   where pull_and_encode called encode ();
//                next_encoded()  where the encoder's load_msg took the
//                                encoded msg_t: the MESSAGE commands come
//                                back in submission order, so the engine
//                                keeps restarting output while any are
//                                ready (restart_output in the reference);
//     in side    submit_received()  where decode_and_push called decode ();
//                next_decoded()     the session push: decoded messages in
//                                   receive order, flags ORed as set_flags
//                                   does (src/msg.cpp:433-436);
//                failed ()          the first failure's error_event_code:
//                                   the engine's error (protocol_error) path,
//                                   as curve_mechanism_base_t::decode's -1.
// A connection's messages keep the reference's per-connection order in both
// directions; its failure stops its own delivery (the reference tears the
// connection down on the first decode failure) and no one else's.
// Single-threaded, like the I/O thread it serves.
#ifndef ZMQG_CURVE_ENGINE_HOOK_HPP_INCLUDED
#define ZMQG_CURVE_ENGINE_HOOK_HPP_INCLUDED

#include <stddef.h>
#include <stdint.h>

#include <deque>
#include <set>
#include <vector>

#include "curve_batcher.hpp"

namespace zmqg
{
class curve_engine_link_t;

class curve_io_hook_t : private curve_sink_t
{
  public:
    curve_io_hook_t (zmqg_ctx *ctx_,
                     const curve_batcher_t::config_t &config_ =
                       curve_batcher_t::config_t (),
                     void *stream_ = NULL);
    //  0, or -1 (errno) when the batcher's slots cannot be allocated
    int init ();
    //  once per poller iteration: launch what the engines queued, deliver
    //  what finished (never blocks).  Messages delivered, or -1 (errno).
    int iteration ();
    //  launch and wait for everything queued (shutdown, tests)
    int drain ();
    size_t outstanding () const;

  private:
    friend class curve_engine_link_t;
    void on_encoded (uint64_t tag_, const uint8_t *wire_, size_t size_);
    void on_decoded (uint64_t tag_,
                     int status_,
                     const uint8_t *payload_,
                     size_t size_,
                     uint8_t flags_);

    curve_batcher_t _batcher;
    std::set<curve_engine_link_t *> _links; //  live links (results of a closed one are dropped)
};

class curve_engine_link_t
{
  public:
    //  codec_: this connection's session (its ctx must be the hook's)
    curve_engine_link_t (curve_io_hook_t *hook_, curve_encoding_gpu_t *codec_);
    ~curve_engine_link_t ();

    //  out side.  0, or -1 with errno (EMSGSIZE: larger than a batcher slot;
    //  EPIPE: the connection has failed)
    int submit_send (const uint8_t *data_, size_t size_, uint8_t msg_flags_);
    //  the next encoded MESSAGE command, in submission order
    bool next_encoded (std::vector<uint8_t> &wire_);

    //  in side: the body of one ZMTP MESSAGE frame.  0, or -1 with errno
    //  (EPIPE: the connection has already failed)
    int submit_received (const uint8_t *wire_, size_t size_);
    //  the next decoded message (payload, MORE/COMMAND flags), in receive
    //  order; after a failure only those decoded before it
    bool next_decoded (msg_buf_t &msg_);
    //  0, or the first failure's ZMQ_PROTOCOL_ERROR_ZMTP_* code
    int failed () const { return _failed; }

    size_t sends_in_flight () const { return _send_pending; }
    size_t receives_in_flight () const { return _recv_pending; }

  private:
    friend class curve_io_hook_t;
    curve_io_hook_t *const _hook;
    curve_encoding_gpu_t *const _codec;
    std::deque<std::vector<uint8_t> > _encoded;
    std::deque<msg_buf_t> _decoded;
    size_t _send_pending, _recv_pending;
    int _failed;

    curve_engine_link_t (const curve_engine_link_t &);
    curve_engine_link_t &operator= (const curve_engine_link_t &);
};
}

#endif
