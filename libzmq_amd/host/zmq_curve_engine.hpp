// zmq_curve_engine.hpp -- the batched CURVE MESSAGE codec inside libzmq's
// stream engine: the engine half of SURVEY.md section 8f row 1 (INTEGRATION.md
// section 3), compiled into the reference library with
// ZMQ_USE_ZMQG_CURVE_BATCHED (tests/host/libzmq_zmqg_batched.patch, on top of
// the ZMQ_USE_ZMQG_CURVE swap of zmq_curve_encoding.hpp).
//
// The reference engine runs its mechanism synchronously, one message per
// call, inside its event handlers (src/stream_engine_base.cpp):
//   out_event (:314-381) fills its write buffer from _next_msg =
//     pull_and_encode (:607-616) -- one session message, one encode --
//     until out_batch_size bytes are queued; with nothing to write it resets
//     POLLOUT (:350-353) and sleeps until restart_output (:383-398);
//   in_event_internal (:220-312) hands every frame the ZMTP decoder
//     completes to _process_msg = decode_and_push (:618-647) -- one decode,
//     one session push; a push the pipe refuses stops input until the
//     session calls restart_input (:400-451);
//   heartbeats encode their PING / PONG commands with the same mechanism
//     (src/zmtp_engine.cpp:447-482).
// Here those calls feed the I/O thread's curve_io_hook_t (one device batch
// per poller turn for every connection of the thread) and the results come
// back through the hook's eventfd, which sits in the thread's poller beside
// its mailbox (src/io_thread.cpp:19-22):
//
//   pull_and_encode    moves what the session holds into the batch (up to a
//                      per-connection cap) and returns the next ENCODED
//                      message in submission order, or EAGAIN -- out_event
//                      then stops POLLOUT exactly as with an empty session;
//                      encoded_ready () (the batch came back) is
//                      restart_output ().
//   encode_command     PING / PONG: submitted behind the messages already
//                      queued, so the nonces reach the wire in order.
//   decode_and_push    copies the frame into the batch and returns 0 at
//                      once; decoded_ready () pushes the results to the
//                      session in receive order with the reference's
//                      per-message work (heartbeat timers, command flags,
//                      metadata), holds a message the pipe refuses until the
//                      session's restart_input, and turns the first failed
//                      frame into the reference's failure: the
//                      handshake-failed-protocol event with its
//                      ZMQ_PROTOCOL_ERROR_ZMTP_* code
//                      (src/curve_mechanism_base.cpp:38-52) and
//                      error (protocol_error).
//   terminate          (flush_on_terminate) what the engine pulled from the
//                      session is written before it goes, as the reference
//                      has it on the wire when it pulls it.
//
// A frame larger than a batch slot takes the per-message path of
// zmq_curve_encoding.hpp once the connection has nothing in flight, so
// nonces and results stay in order.  The device launch is held back while
// ZMQG_ENGINE_FLIGHT (default 2) batches are still running: messages then
// gather in the open slot and go with the completion's wake-up, so a busy
// thread launches large batches and an idle one launches at once.
#ifndef ZMQG_ZMQ_CURVE_ENGINE_HPP_INCLUDED
#define ZMQG_ZMQ_CURVE_ENGINE_HPP_INCLUDED

#include <stddef.h>
#include <stdint.h>

#include <deque>
#include <vector>

#include "curve_engine_hook.hpp"
#include "msg.hpp"

namespace zmq
{
class stream_engine_base_t;
class io_thread_t;
class curve_io_poll_t;

class curve_engine_codec_t : public zmqg::curve_link_events_t
{
  public:
    //  The batched codec for an engine whose mechanism has just become ready,
    //  or NULL: not CURVE, no device session, ZMQG_CURVE_BATCHED=0 in the
    //  environment, or the thread's hook could not be set up -- the engine
    //  then keeps the per-message codec.
    static curve_engine_codec_t *attach (stream_engine_base_t *engine_,
                                         io_thread_t *io_thread_);
    ~curve_engine_codec_t ();

    //  _next_msg after the handshake: 0 and the next MESSAGE command in
    //  msg_, or -1 with errno EAGAIN (none ready yet) or another errno.
    int pull_and_encode (msg_t *msg_);
    //  a PING / PONG command in msg_ (consumed): as pull_and_encode after it
    int encode_command (msg_t *msg_);
    //  _process_msg after the handshake: 0 (the frame was taken), or -1 with
    //  errno EAGAIN (not taken: too much in flight; input stops and resumes
    //  through restart_input) or the failure of a per-message decode.
    int decode_and_push (msg_t *msg_);
    //  restart_input's first step: push what the pipe refused before.
    //  1: nothing held back; 0: the pipe is full again; -1: the engine has
    //  failed and is gone.
    int resume_input ();
    //  the engine's terminate (): write everything pulled so far
    void flush_on_terminate ();
    //  Input failed (the peer closed, a read error, or a framing error the
    //  ZMTP decoder found) while frames before it may still be on the
    //  device: in the reference they were decoded and pushed before the
    //  failure was seen, so they reach the session first.  1: the engine
    //  fails now with reason_; 0: the session's pipe is full, the engine
    //  stays with its input stopped and fails with reason_ once the held
    //  messages are pushed (resume_input); -1: a frame failed to decode and
    //  the engine has already failed and is gone.
    int input_failed (int reason_);
    //  after resume_input returned 1: the deferred failure, or -1
    int deferred_failure () const { return _failure; }

    //  curve_link_events_t
    void encoded_ready ();
    void decoded_ready ();

  private:
    curve_engine_codec_t (stream_engine_base_t *engine_,
                          curve_io_poll_t *io_,
                          zmqg::curve_encoding_gpu_t *codec_);

    //  session messages into the batch while under the caps
    void pull_into_batch ();
    //  the next encoded message into msg_ (0), or -1 with EAGAIN
    int take_encoded (msg_t *msg_);
    //  results into the session: 1 all delivered, 0 the pipe refused one,
    //  -1 the connection failed (the engine is gone)
    int deliver ();
    //  the reference's decode_and_push tail for a decoded msg_ (:625-646)
    int push_decoded (msg_t *msg_);
    bool receive_idle () const;
    bool receive_room () const;

    stream_engine_base_t *const _engine;
    curve_io_poll_t *const _io;
    zmqg::curve_engine_link_t _link;
    const size_t _slot_bytes;

    msg_t _pulled;   //  a session message too large for a slot, held
    bool _big_held;  //  until the connection has nothing in flight
    std::deque<size_t> _tx_sizes; //  payload bytes of the sends pending
    size_t _tx_bytes;
    bool _tx_error; //  the device refused a submission: sending stops

    msg_t _rx_msg;  //  a decoded message the session's pipe refused
    bool _rx_held;
    size_t _rx_bytes; //  wire bytes submitted and not yet delivered
    std::deque<size_t> _rx_sizes;
    bool _rx_blocked; //  decode_and_push refused a frame (input stopped)
    bool _delivering;
    bool _quiet;       //  delivery may not fail the engine (terminate, drain)
    int _failure;      //  a deferred input failure's reason, or -1

    curve_engine_codec_t (const curve_engine_codec_t &);
    curve_engine_codec_t &operator= (const curve_engine_codec_t &);
};
}

#endif
