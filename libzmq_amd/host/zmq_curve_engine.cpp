// zmq_curve_engine.cpp -- see zmq_curve_engine.hpp.  Compiled into the
// reference library (tests/host/build_libzmq.sh, variant zmqgb) with its own
// headers on the include path; a friend of stream_engine_base_t
// (tests/host/libzmq_zmqg_batched.patch).
#include "precompiled.hpp"

#include <errno.h>
#include <poll.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <new>

#include "zmq_curve_engine.hpp"

#include "curve_mechanism_base.hpp"
#include "err.hpp"
#include "i_poll_events.hpp"
#include "io_thread.hpp"
#include "poller.hpp"
#include "session_base.hpp"
#include "socket_base.hpp"
#include "stream_engine_base.hpp"

namespace zmq
{
namespace
{
size_t env_size (const char *name_, size_t dflt_)
{
    const char *e = getenv (name_);
    const long long v = e ? atoll (e) : 0;
    return v > 0 ? static_cast<size_t> (v) : dflt_;
}

//  per connection and direction: messages and payload bytes the codec may
//  hold (in the batch, in flight or delivered and not yet taken)
size_t max_msgs ()
{
    static const size_t v = env_size ("ZMQG_ENGINE_MSGS", 8192);
    return v;
}
size_t max_bytes ()
{
    static const size_t v = env_size ("ZMQG_ENGINE_BYTES", 16u << 20);
    return v;
}
//  the send side pulls from the session only when fewer messages than this
//  are still to be written (in the batch, on the device or encoded): pulling
//  on every out_event would empty the pipe each time, and the sender's next
//  message would then wake this thread through the mailbox (the pipe's
//  activate_read) for a handful of messages
size_t low_water ()
{
    static const size_t v = env_size ("ZMQG_ENGINE_LOW_WATER", 512);
    return v;
}

uint64_t now_ms ()
{
    timespec t;
    clock_gettime (CLOCK_MONOTONIC, &t);
    return static_cast<uint64_t> (t.tv_sec) * 1000 + t.tv_nsec / 1000000;
}
}

//  One per I/O thread (thread-local; engines never leave the thread they
//  were plugged into): the hook and its eventfd in the thread's poller, next
//  to the mailbox, for as long as a batched engine lives on the thread.
class curve_io_poll_t : public i_poll_events
{
  public:
    //  the calling I/O thread's instance, its eventfd watched by poller_;
    //  NULL when no device context or batcher can be had
    static curve_io_poll_t *acquire (poller_t *poller_);
    void release ();

    zmqg::curve_io_hook_t *hook () { return _hook; }
    size_t slot_bytes () const { return _config.slot_bytes; }

    //  launch what the engines queued before the poller blocks again
    void flush_soon ()
    {
        if (!_timer) {
            _poller->add_timer (0, this, flush_timer_id);
            _timer = true;
        }
    }

    //  i_poll_events: the eventfd (batches came back) and the flush timer
    void in_event ()
    {
        const uint64_t t0 = stats_ns ();
        const int rc = _hook->in_event ();
        errno_assert (rc >= 0);
        ++_wakes;
        _delivered += rc;
        _deliver_ns += stats_ns () - t0;
        launch_if_idle ();
    }
    void out_event () { zmq_assert (false); }
    void timer_event (int)
    {
        _timer = false;
        launch_if_idle ();
    }

    ~curve_io_poll_t ()
    {
        //  the thread is exiting: its poller no longer runs this object
        if (getenv ("ZMQG_ENGINE_STATS"))
            fprintf (stderr,
                     "zmqg engine: %llu wake-ups, %llu launches, %llu "
                     "messages launched, %llu delivered by wake-ups, "
                     "%.3f ms in launches (%llu batch calls %.3f ms, "
                     "fences %.3f ms), %.3f ms in deliveries\n",
                     (unsigned long long) _wakes,
                     (unsigned long long) _launches,
                     (unsigned long long) _launched,
                     (unsigned long long) _delivered, _launch_ns * 1e-6,
                     (unsigned long long) _hook->launch_stats ().launches,
                     _hook->launch_stats ().batch_ns * 1e-6,
                     _hook->launch_stats ().fence_ns * 1e-6,
                     _deliver_ns * 1e-6);
        delete _hook;
    }

  private:
    enum
    {
        flush_timer_id = 0x5a
    };

    explicit curve_io_poll_t (poller_t *poller_) :
        _poller (poller_),
        _hook (NULL),
        _handle (static_cast<poller_t::handle_t> (NULL)),
        _users (0),
        _timer (false),
        _max_flight (env_size ("ZMQG_ENGINE_FLIGHT", 2)),
        _min_batch (env_size ("ZMQG_ENGINE_MIN_BATCH", 64)),
        _wakes (0),
        _launches (0),
        _launched (0),
        _delivered (0),
        _launch_ns (0),
        _deliver_ns (0),
        _stats (getenv ("ZMQG_ENGINE_STATS") != NULL)
    {
        _config.slots = static_cast<int> (env_size ("ZMQG_ENGINE_SLOTS", 6));
        _config.slot_msgs = env_size ("ZMQG_ENGINE_SLOT_MSGS", 8192);
        _config.slot_bytes = env_size ("ZMQG_ENGINE_SLOT_BYTES", 8u << 20);
    }

    int init ()
    {
        zmqg_ctx *ctx = zmqg::thread_ctx ();
        if (!ctx)
            return -1;
        _hook = new (std::nothrow) zmqg::curve_io_hook_t (ctx, _config);
        return _hook && _hook->init () == 0 ? 0 : -1;
    }

    //  The device runs at most _max_flight batches of this thread at once:
    //  beyond that, new messages wait in the open slot and go with the next
    //  completion (in_event), so a loaded thread launches big batches.
    void launch_if_idle ()
    {
        const size_t flying = _hook->batches_in_flight ();
        //  an idle device takes any batch (latency); a busy one only a
        //  batch worth a launch, else the completion's wake-up sends it
        if (!_hook->flush_pending () || flying >= _max_flight
            || (flying > 0
                && _hook->outstanding () - _hook->in_flight () < _min_batch))
            return;
        ++_launches;
        _launched += _hook->outstanding () - _hook->in_flight ();
        const uint64_t t0 = stats_ns ();
        const int rc = _hook->timer_event ();
        errno_assert (rc == 0);
        _launch_ns += stats_ns () - t0;
    }

    poller_t *const _poller;
    zmqg::curve_batcher_t::config_t _config;
    zmqg::curve_io_hook_t *_hook;
    poller_t::handle_t _handle;
    int _users;
    bool _timer;
    const size_t _max_flight;
    const size_t _min_batch;
    //  ZMQG_ENGINE_STATS: printed when the thread exits
    uint64_t _wakes, _launches, _launched, _delivered, _launch_ns, _deliver_ns;
    const bool _stats;
    uint64_t stats_ns () const
    {
        if (!_stats)
            return 0;
        timespec t;
        clock_gettime (CLOCK_MONOTONIC, &t);
        return static_cast<uint64_t> (t.tv_sec) * 1000000000u + t.tv_nsec;
    }

    struct holder_t
    {
        curve_io_poll_t *p;
        bool failed;
        ~holder_t () { delete p; }
    };
    static thread_local holder_t tls;
};

thread_local curve_io_poll_t::holder_t curve_io_poll_t::tls = {NULL, false};

curve_io_poll_t *curve_io_poll_t::acquire (poller_t *poller_)
{
    holder_t &h = tls;
    if (!h.p) {
        if (h.failed)
            return NULL;
        h.p = new (std::nothrow) curve_io_poll_t (poller_);
        if (!h.p || h.p->init () != 0) {
            delete h.p;
            h.p = NULL;
            h.failed = true;
            return NULL;
        }
    }
    curve_io_poll_t *p = h.p;
    zmq_assert (p->_poller == poller_);
    if (p->_users++ == 0) {
        //  as io_thread_t does with its mailbox (src/io_thread.cpp:19-22)
        p->_handle = poller_->add_fd (p->_hook->get_fd (), p);
        poller_->set_pollin (p->_handle);
    }
    return p;
}

void curve_io_poll_t::release ()
{
    zmq_assert (_users > 0);
    if (--_users == 0) {
        //  the poller stops when nothing is left in it (src/epoll.cpp:144-151)
        _poller->rm_fd (_handle);
        if (_timer) {
            _poller->cancel_timer (this, flush_timer_id);
            _timer = false;
        }
    }
}

curve_engine_codec_t *curve_engine_codec_t::attach (stream_engine_base_t *engine_,
                                                    io_thread_t *io_thread_)
{
    const char *e = getenv ("ZMQG_CURVE_BATCHED");
    if ((e && strcmp (e, "0") == 0) || !io_thread_ || !engine_->_mechanism
        || engine_->_options.mechanism != ZMQ_CURVE)
        return NULL;
    curve_mechanism_base_t *m =
      dynamic_cast<curve_mechanism_base_t *> (engine_->_mechanism);
    zmqg::curve_encoding_gpu_t *g = m ? m->batched_codec () : NULL;
    if (!g)
        return NULL;
    curve_io_poll_t *io = curve_io_poll_t::acquire (io_thread_->get_poller ());
    if (!io)
        return NULL;
    curve_engine_codec_t *c =
      new (std::nothrow) curve_engine_codec_t (engine_, io, g);
    if (!c)
        io->release ();
    return c;
}

curve_engine_codec_t::curve_engine_codec_t (stream_engine_base_t *engine_,
                                            curve_io_poll_t *io_,
                                            zmqg::curve_encoding_gpu_t *codec_) :
    _engine (engine_),
    _io (io_),
    _link (io_->hook (), codec_, this),
    _slot_bytes (io_->slot_bytes ()),
    _big_held (false),
    _tx_bytes (0),
    _tx_error (false),
    _rx_held (false),
    _rx_bytes (0),
    _rx_blocked (false),
    _delivering (false),
    _quiet (false),
    _failure (-1)
{
    int rc = _pulled.init ();
    errno_assert (rc == 0);
    rc = _rx_msg.init ();
    errno_assert (rc == 0);
}

curve_engine_codec_t::~curve_engine_codec_t ()
{
    //  results still in flight for this connection are dropped by the hook
    //  (routed by link id); the session slot stays valid until the mechanism
    //  is destroyed after this object
    _pulled.close ();
    _rx_msg.close ();
    _io->release ();
}

// ---------------------------------------------------------------- out side

void curve_engine_codec_t::pull_into_batch ()
{
    while (!_big_held && !_tx_error
           && _link.sends_in_flight () + _link.encoded_queued () < max_msgs ()
           && _tx_bytes < max_bytes ()) {
        //  EAGAIN: the pipe is empty; the session's read_activated calls
        //  restart_output when it is not (src/session_base.cpp)
        if (_engine->_session->pull_msg (&_pulled) == -1)
            return;
        const size_t n = _pulled.size ();
        if (n > _slot_bytes) {
            _big_held = true;
            return;
        }
        //  the flags byte as curve_encoding_t::encode reads it (more,
        //  command, subscribe / cancel: src/curve_mechanism_base.cpp:118-128)
        if (_link.submit_send (static_cast<const uint8_t *> (_pulled.data ()),
                               n, static_cast<uint8_t> (_pulled.flags ()))
            != 0)
            _tx_error = true;
        else {
            _tx_sizes.push_back (n);
            _tx_bytes += n;
            _io->flush_soon ();
        }
        int rc = _pulled.close ();
        errno_assert (rc == 0);
        rc = _pulled.init ();
        errno_assert (rc == 0);
    }
}

int curve_engine_codec_t::take_encoded (msg_t *msg_)
{
    const uint8_t *wire;
    size_t size;
    if (!_link.peek_encoded (&wire, &size)) {
        errno = EAGAIN;
        return -1;
    }
    _tx_bytes -= _tx_sizes.front ();
    _tx_sizes.pop_front ();
    //  the MESSAGE command is a fresh msg_t without flags, as msg_->move
    //  (msg_box) leaves it (src/curve_mechanism_base.cpp:203)
    const int rc = msg_->init_size (size);
    errno_assert (rc == 0);
    memcpy (msg_->data (), wire, size);
    _link.pop_encoded ();
    return 0;
}

int curve_engine_codec_t::pull_and_encode (msg_t *msg_)
{
    if (_link.sends_in_flight () + _link.encoded_queued () < low_water ())
        pull_into_batch ();
    if (take_encoded (msg_) == 0)
        return 0;
    if (_tx_error) {
        //  the device refused a batch: the connection stops sending, as the
        //  per-message codec's EPROTO stops out_event
        errno = EPROTO;
        return -1;
    }
    if (_big_held && _link.sends_in_flight () == 0) {
        //  larger than a slot: the per-message codec, after everything
        //  submitted before it, so its nonce follows theirs on the wire
        _big_held = false;
        const int rc = msg_->move (_pulled);
        errno_assert (rc == 0);
        return _engine->_mechanism->encode (msg_);
    }
    errno = EAGAIN;
    return -1;
}

int curve_engine_codec_t::encode_command (msg_t *msg_)
{
    const size_t n = msg_->size ();
    if (!_tx_error
        && _link.submit_send (static_cast<const uint8_t *> (msg_->data ()), n,
                              static_cast<uint8_t> (msg_->flags ()))
             == 0) {
        _tx_sizes.push_back (n);
        _tx_bytes += n;
        _io->flush_soon ();
    } else
        _tx_error = true;
    int rc = msg_->close ();
    errno_assert (rc == 0);
    rc = msg_->init ();
    errno_assert (rc == 0);
    return pull_and_encode (msg_);
}

void curve_engine_codec_t::encoded_ready ()
{
    _engine->restart_output ();
}

void curve_engine_codec_t::flush_on_terminate ()
{
    stream_engine_base_t *const e = _engine;
    if (e->_io_error || !e->_encoder)
        return;
    //  a failed frame found while waiting must not tear the engine down
    //  under this call: terminate () deletes it anyway
    _quiet = true;
    //  bounded like a linger: ZMQ_LINGER when set (capped at 5 s), else 5 s
    const int linger = e->_options.linger.load ();
    const uint64_t deadline =
      now_ms () + (linger >= 0 && linger < 5000 ? linger : 5000);
    for (;;) {
        if (!e->_outsize) {
            if (_link.encoded_queued () == 0 && _link.sends_in_flight () != 0) {
                //  wait for the thread's batches (every connection's results
                //  are delivered, this one's into _link)
                if (_io->hook ()->drain () < 0)
                    return;
                continue;
            }
            //  out_event's refill (src/stream_engine_base.cpp:328-348)
            e->_outpos = NULL;
            e->_outsize = e->_encoder->encode (&e->_outpos, 0);
            while (e->_outsize
                   < static_cast<size_t> (e->_options.out_batch_size)) {
                if ((e->*(e->_next_msg)) (&e->_tx_msg) == -1)
                    break;
                e->_encoder->load_msg (&e->_tx_msg);
                unsigned char *bufptr = e->_outpos + e->_outsize;
                const size_t n = e->_encoder->encode (
                  &bufptr, e->_options.out_batch_size - e->_outsize);
                if (e->_outpos == NULL)
                    e->_outpos = bufptr;
                e->_outsize += n;
            }
            if (!e->_outsize && _link.sends_in_flight () == 0)
                return;
            continue;
        }
        const int nbytes = e->write (e->_outpos, e->_outsize);
        if (nbytes < 0)
            return;
        e->_outpos += nbytes;
        e->_outsize -= nbytes;
        if (e->_outsize) {
            const uint64_t t = now_ms ();
            if (t >= deadline)
                return;
            pollfd p;
            p.fd = e->_s;
            p.events = POLLOUT;
            p.revents = 0;
            if (poll (&p, 1, static_cast<int> (deadline - t)) <= 0
                || (p.revents & (POLLERR | POLLHUP)))
                return;
        }
    }
}

// ----------------------------------------------------------------- in side

bool curve_engine_codec_t::receive_idle () const
{
    return _link.receives_in_flight () == 0 && _link.decoded_queued () == 0
           && !_rx_held;
}

bool curve_engine_codec_t::receive_room () const
{
    return _link.receives_in_flight () + _link.decoded_queued () < max_msgs ()
           && _rx_bytes < max_bytes ();
}

int curve_engine_codec_t::decode_and_push (msg_t *msg_)
{
    const size_t n = msg_->size ();
    if (n > _slot_bytes) {
        //  larger than a slot: the per-message codec once everything before
        //  it has reached the session (the replay rule sees nonces in order)
        if (!receive_idle () || _link.failed ()) {
            _rx_blocked = true;
            errno = EAGAIN;
            return -1;
        }
        if (_engine->_mechanism->decode (msg_) == -1)
            return -1;
        return push_decoded (msg_);
    }
    if (!receive_room () || _link.failed ()) {
        //  not taken: in_event_internal stops input with this frame kept in
        //  the decoder; decoded_ready restarts it
        _rx_blocked = true;
        errno = EAGAIN;
        return -1;
    }
    if (_link.submit_received (static_cast<const uint8_t *> (msg_->data ()), n)
        != 0) {
        errno = EPROTO;
        return -1;
    }
    _rx_sizes.push_back (n);
    _rx_bytes += n;
    _io->flush_soon ();
    //  msg_ stays with the decoder, which closes it for the next frame
    return 0;
}

int curve_engine_codec_t::push_decoded (msg_t *msg_)
{
    //  src/stream_engine_base.cpp:625-646
    stream_engine_base_t *const e = _engine;
    if (e->_has_timeout_timer) {
        e->_has_timeout_timer = false;
        e->cancel_timer (stream_engine_base_t::heartbeat_timeout_timer_id);
    }
    if (e->_has_ttl_timer) {
        e->_has_ttl_timer = false;
        e->cancel_timer (stream_engine_base_t::heartbeat_ttl_timer_id);
    }
    if (msg_->flags () & msg_t::command)
        e->process_command_message (msg_);
    if (e->_metadata)
        msg_->set_metadata (e->_metadata);
    if (e->_session->push_msg (msg_) == -1) {
        if (errno == EAGAIN)
            e->_process_msg = &stream_engine_base_t::push_one_then_decode_and_push;
        return -1;
    }
    return 0;
}

int curve_engine_codec_t::deliver ()
{
    if (_delivering)
        return 1;
    _delivering = true;
    stream_engine_base_t *const e = _engine;
    int rc = 1;
    for (;;) {
        if (!_rx_held) {
            const uint8_t *payload;
            size_t size;
            uint8_t flags;
            if (!_link.peek_decoded (&payload, &size, &flags))
                break;
            _rx_bytes -= _rx_sizes.front ();
            _rx_sizes.pop_front ();
            int r = _rx_msg.init_size (size);
            errno_assert (r == 0);
            if (size)
                memcpy (_rx_msg.data (), payload, size);
            _link.pop_decoded ();
            //  the plaintext MORE / COMMAND bits, ORed as set_flags does
            _rx_msg.set_flags (flags);
            //  the reference's per-message work before the push (:625-640)
            if (e->_has_timeout_timer) {
                e->_has_timeout_timer = false;
                e->cancel_timer (stream_engine_base_t::heartbeat_timeout_timer_id);
            }
            if (e->_has_ttl_timer) {
                e->_has_ttl_timer = false;
                e->cancel_timer (stream_engine_base_t::heartbeat_ttl_timer_id);
            }
            if (_rx_msg.flags () & msg_t::command)
                e->process_command_message (&_rx_msg); //  a PING sends its PONG
            if (e->_metadata)
                _rx_msg.set_metadata (e->_metadata);
            _rx_held = true;
        }
        if (e->_session->push_msg (&_rx_msg) == -1) {
            //  the pipe is full: held until the session's restart_input
            rc = 0;
            break;
        }
        //  (push_msg takes the message, or drops a command that is not
        //  SUBSCRIBE / CANCEL without taking it)
        int r = _rx_msg.close ();
        errno_assert (r == 0);
        r = _rx_msg.init ();
        errno_assert (r == 0);
        _rx_held = false;
    }
    e->_session->flush ();
    _delivering = false;
    if (rc == 1 && _link.failed () && !_quiet) {
        //  every frame before the failed one has reached the session; now
        //  curve_mechanism_base_t::decode's event (:46-49) and the engine's
        //  protocol-error teardown (:293-305): the engine and this codec go
        const int code = _link.failed ();
        e->_socket->event_handshake_failed_protocol (
          e->_session->get_endpoint (), code);
        e->error (i_engine::protocol_error);
        return -1;
    }
    return rc;
}

void curve_engine_codec_t::decoded_ready ()
{
    if (deliver () < 0)
        return;
    stream_engine_base_t *const e = _engine;
    if (_rx_blocked && !_quiet && _failure < 0 && e->_input_stopped
        && !_rx_held && receive_room ()) {
        //  decode_and_push refused a frame for room: take it now
        _rx_blocked = false;
        e->restart_input ();
    }
}

int curve_engine_codec_t::input_failed (int reason_)
{
    stream_engine_base_t *const e = _engine;
    if (_link.receives_in_flight () != 0) {
        //  wait for this thread's batches; what comes back for this
        //  connection is pushed, but a failed frame is acted on below
        _quiet = true;
        const int rc = _io->hook ()->drain ();
        _quiet = false;
        if (rc < 0)
            return 1;
    }
    const int rc = deliver ();
    if (rc != 0)
        return rc;
    //  the pipe is full: stop reading, as the reference has stopped by now
    //  (its push failed before it read on); the engine fails after the
    //  session has taken the rest (restart_input -> resume_input)
    _failure = reason_;
    if (!e->_input_stopped) {
        e->_input_stopped = true;
        e->reset_pollin (e->_handle);
    }
    return 0;
}

int curve_engine_codec_t::resume_input ()
{
    const int rc = deliver ();
    if (rc == 1)
        _rx_blocked = false;
    return rc;
}
}
