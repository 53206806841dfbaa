// zmq_curve_encoding.hpp -- zmq::curve_encoding_t on the MI355X codec: the
// reference-side half of the drop-in.
//
// libzmq builds its CURVE message codec into curve_mechanism_base_t
// (src/curve_mechanism_base.hpp:24-58, src/curve_mechanism_base.cpp:54-284);
// with ZMQ_USE_ZMQG_CURVE defined, src/curve_mechanism_base.hpp includes this
// file instead of declaring its own class, so curve_mechanism_base_t,
// curve_client_t / curve_server_t and the handshake code (which calls
// get_writable_precom_buffer, get_and_inc_nonce and set_peer_nonce) compile
// unchanged.  It is written against the reference's own msg_t
// (src/msg.hpp: init_size, move, shrink, set_flags, data, size, flags),
// errno_assert (src/err.hpp) and ZMQ_NON_COPYABLE_NOR_MOVABLE
// (src/macros.hpp); tests/test_reference_binding.py compiles it against
// those headers.
//
// Each connection takes one session slot of its I/O thread's device context
// (zmqg::thread_ctx, curve_encoding_gpu.hpp) and gives it back when the
// mechanism is destroyed.  One message per call, as the reference engine
// calls its codec (src/stream_engine_base.cpp:281-291, :331-348); the
// batched path for many connections is curve_batcher_t (INTEGRATION.md
// section 3).
#ifndef ZMQG_ZMQ_CURVE_ENCODING_HPP_INCLUDED
#define ZMQG_ZMQ_CURVE_ENCODING_HPP_INCLUDED

#include <string.h>

#include "curve_encoding_gpu.hpp"
#include "err.hpp"
#include "macros.hpp"
#include "msg.hpp"

namespace zmq
{
class curve_encoding_t
{
  public:
    //  The reference's constructor cannot fail.  Here a connection needs a
    //  session slot of its I/O thread's device context; when none can be had
    //  (all zmqg::thread_sessions slots in use: ENOMEM; no device context:
    //  EIO) the object is still constructed, without a slot, and its encode
    //  and decode fail (below), so the engine drops that one connection --
    //  the process is never aborted for it.
    curve_encoding_t (const char *encode_nonce_prefix_,
                      const char *decode_nonce_prefix_,
                      const bool downgrade_sub_) :
        _sid_errno (acquire_sid (&_sid)),
        _gpu (_sid_errno ? NULL : zmqg::thread_ctx (),
              _sid,
              encode_nonce_prefix_,
              decode_nonce_prefix_,
              downgrade_sub_)
    {
    }

    ~curve_encoding_t ()
    {
        if (!_sid_errno)
            zmqg::release_session (_sid);
    }

    //  src/curve_mechanism_base.cpp:111-205: msg_ becomes the MESSAGE
    //  command (a fresh msg_t without flags, as msg_->move (msg_box) leaves
    //  it).  -1 with errno set where the reference's rc would be non-zero;
    //  a connection without a session slot fails with EPROTO (the engine's
    //  out_event stops pulling, src/stream_engine_base.cpp:331-339).
    int encode (msg_t *msg_)
    {
        if (_sid_errno) {
            errno = EPROTO;
            return -1;
        }
        //  more / command / subscribe / cancel
        const uint8_t fl = static_cast<uint8_t> (msg_->flags ());
        msg_t box;
        int rc = box.init_size (_gpu.wire_size (fl, msg_->size ()));
        errno_assert (rc == 0);
        //  the device writes the box straight from the message's bytes
        if (_gpu.encode_msg (static_cast<const uint8_t *> (msg_->data ()),
                             msg_->size (), fl,
                             static_cast<uint8_t *> (box.data ()))
            == -1)
            return -1;
        rc = msg_->move (box);
        errno_assert (rc == 0);
        return 0;
    }

    //  src/curve_mechanism_base.cpp:207-284: on success msg_ holds the
    //  payload (shrunk, :253-260) with the plaintext MORE/COMMAND bits ORed
    //  into its flags (msg_t::set_flags ORs, src/msg.cpp:433-436).  On
    //  failure -1, errno EPROTO and *error_event_code_ =
    //  ZMQ_PROTOCOL_ERROR_ZMTP_*, as check_validity and the MAC check set
    //  them, with the peer nonce advanced as the reference advances it.
    int decode (msg_t *msg_, int *error_event_code_)
    {
        if (_sid_errno) {
            //  rejected like a frame that fails its MAC: the mechanism emits
            //  the handshake-failed event and the engine closes this
            //  connection (src/curve_mechanism_base.cpp:38-52)
            if (error_event_code_)
                *error_event_code_ = ZMQG_ERR_CRYPTOGRAPHIC; //  = ZMQ_PROTOCOL_ERROR_ZMTP_CRYPTOGRAPHIC
            errno = EPROTO;
            return -1;
        }
        //  decoded in place: the payload lands at the front of the
        //  message, which is then shrunk to it (:253-260)
        uint8_t *p = static_cast<uint8_t *> (msg_->data ());
        uint8_t fl = 0;
        if (_gpu.decode_msg (p, msg_->size (), p, &fl, error_event_code_)
            == -1)
            return -1;
        msg_->shrink (msg_->size () - 33);
        msg_->set_flags (fl);
        return 0;
    }

    uint8_t *get_writable_precom_buffer ()
    {
        return _gpu.get_writable_precom_buffer ();
    }
    const uint8_t *get_precom_buffer () const
    {
        return _gpu.get_precom_buffer ();
    }

    //  the connection's device session for the batched engine path
    //  (zmq_curve_engine.hpp), NULL when it has no session slot.  Encodes and
    //  decodes through it share this object's nonces and the device's peer
    //  nonce, so the two paths can follow one another on a connection.
    zmqg::curve_encoding_gpu_t *batched_codec ()
    {
        return _sid_errno ? NULL : &_gpu;
    }

    typedef uint64_t nonce_t;

    nonce_t get_and_inc_nonce () { return _gpu.get_and_inc_nonce (); }
    void set_peer_nonce (nonce_t peer_nonce_)
    {
        _gpu.set_peer_nonce (peer_nonce_);
    }

  private:
    //  0 and *sid_ set, or the errno of zmqg::acquire_session
    static int acquire_sid (uint32_t *sid_)
    {
        *sid_ = 0;
        return zmqg::acquire_session (sid_) == 0 ? 0 : errno;
    }

    uint32_t _sid;
    const int _sid_errno; //  0: this connection holds session slot _sid
    zmqg::curve_encoding_gpu_t _gpu;

    ZMQ_NON_COPYABLE_NOR_MOVABLE (curve_encoding_t)
};
}

#endif
