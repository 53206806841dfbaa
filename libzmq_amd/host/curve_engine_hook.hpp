// curve_engine_hook.hpp -- the stream-engine side of the batched CURVE
// codec: what src/stream_engine_base.cpp's two
// codec call sites and the I/O thread's poller loop become when the
// MESSAGE AEAD runs on the GPU in batches.
//
// The reference engine calls its mechanism synchronously, one message at a
// time, inside its event handlers:
//   out_event (src/stream_engine_base.cpp:331-348): _next_msg =
//     pull_and_encode (:607-616) pulls a message from the session and
//     encodes it, until out_batch_size bytes are queued for the socket; with
//     nothing to write it resets POLLOUT (:350-353) and sleeps until
//     restart_output (:383-390) sets it again;
//   in_event_internal (:281-291): for every frame the ZMTP decoder
//     completes, _process_msg = decode_and_push (:618-647) decodes it and
//     pushes it to the session; a stalled input resumes through
//     restart_input (:400-442).
// The I/O thread sleeps in epoll_wait (src/epoll.cpp:140-179) and wakes only
// for a file descriptor it watches (its mailbox, src/io_thread.cpp:54, or a
// socket) or a timer (execute_timers runs before each epoll_wait).
//
// With curve_batcher_t (one per I/O thread) the codec becomes asynchronous.
// The two objects here carry the rest of the change:
//
//   curve_io_hook_t       one per I/O thread: owns the batcher and an
//                         eventfd that the batcher's fences write when a
//                         launched batch completes (zmqg_fence_record_notify).
//                         The poller watches get_fd () for POLLIN like the
//                         mailbox (add_fd + set_pollin); in_event () clears
//                         it, delivers the finished batches and resumes the
//                         engines they belong to.  Messages the engines
//                         queued are launched by timer_event () -- a
//                         zero-delay timer the engine's first submit of a
//                         poller turn asks for (flush_pending ()), run by
//                         execute_timers before the poller blocks again.
//   curve_engine_link_t   one per engine (connection): replaces the two
//                         mechanism calls.
//     out side   submit_send()   where pull_and_encode called encode ();
//                next_encoded()  where the encoder's load_msg took the
//                                encoded msg_t, in submission order;
//     in side    submit_received()  where decode_and_push called decode ();
//                next_decoded()     the session push: decoded messages in
//                                   receive order, flags ORed as set_flags
//                                   does (src/msg.cpp:433-436);
//                failed ()          the first failure's error_event_code:
//                                   the engine's error (protocol_error) path,
//                                   as curve_mechanism_base_t::decode's -1.
//     events     curve_link_events_t: encoded_ready () is the engine's
//                restart_output, decoded_ready () its restart_input; the
//                hook calls them once results for the link have arrived.
// Results are routed by a link id (a per-hook counter), never by address: a
// link closed while its messages are in flight simply loses them, and a new
// link at the same address cannot receive them.
// A connection's messages keep the reference's per-connection order in both
// directions; its failure stops its own delivery (the reference tears the
// connection down on the first decode failure) and no one else's.
// Single-threaded, like the I/O thread it serves.
#ifndef ZMQG_CURVE_ENGINE_HOOK_HPP_INCLUDED
#define ZMQG_CURVE_ENGINE_HOOK_HPP_INCLUDED

#include <stddef.h>
#include <stdint.h>

#include <deque>
#include <map>
#include <vector>

#include "curve_batcher.hpp"

namespace zmqg
{
class curve_engine_link_t;

//  Results waiting for their engine: the bytes back to back in one growing
//  buffer, (size, flags) per record -- no allocation per message once the
//  buffer has grown to the connection's working depth.
class result_fifo_t
{
  public:
    result_fifo_t () : _head (0), _tail (0) {}
    void push (const uint8_t *data_, size_t size_, uint8_t flags_);
    bool empty () const { return _recs.empty (); }
    size_t size () const { return _recs.size (); }
    //  the oldest record; valid until the next push
    const uint8_t *front_data () const { return &_buf[0] + _head; }
    size_t front_size () const { return _recs.front ().first; }
    uint8_t front_flags () const { return _recs.front ().second; }
    void pop ();

  private:
    std::vector<uint8_t> _buf;
    size_t _head, _tail;
    std::deque<std::pair<size_t, uint8_t> > _recs;
};

//  The engine's resume points (implemented by the engine).  Called from the
//  hook's in_event () / timer_event () / iteration () / drain (), never from
//  inside a submit.
struct curve_link_events_t
{
    virtual ~curve_link_events_t () {}
    //  encoded MESSAGE commands are ready (next_encoded): restart_output
    virtual void encoded_ready () = 0;
    //  decoded messages or a failure are ready (next_decoded, failed):
    //  restart_input
    virtual void decoded_ready () = 0;
};

class curve_io_hook_t : private curve_sink_t
{
  public:
    curve_io_hook_t (zmqg_ctx *ctx_,
                     const curve_batcher_t::config_t &config_ =
                       curve_batcher_t::config_t (),
                     void *stream_ = NULL);
    //  waits for the batches in flight (nothing is delivered) and closes the
    //  eventfd once their notifications have run
    ~curve_io_hook_t ();

    //  0, or -1 (errno) when the eventfd or the batcher's slots cannot be
    //  allocated
    int init ();
    //  the eventfd to watch for POLLIN (io_thread_t: add_fd, set_pollin)
    int get_fd () const { return _fd; }
    //  POLLIN on get_fd (): clear it, deliver every finished batch, resume
    //  the engines that got results.  Messages delivered, or -1 (errno).
    int in_event ();
    //  true when engines have queued messages since the last launch: the
    //  poller should run timer_event () before it blocks again
    bool flush_pending () const { return _batcher.queued () != 0; }
    //  launch what the engines queued (and resume any engine a back-pressure
    //  wait delivered to).  0 or -1 (errno).
    int timer_event ();
    //  both, for loops that call the hook once per turn (never blocks)
    int iteration ();
    //  launch and wait for everything queued (shutdown, tests)
    int drain ();
    size_t outstanding () const;
    //  messages launched and not yet delivered
    size_t in_flight () const { return _batcher.in_flight (); }
    //  launched batches whose results have not been delivered yet (a poller
    //  that holds new messages back while the device is busy uses it)
    size_t batches_in_flight () const { return _batcher.batches_in_flight (); }
    const curve_batcher_t::launch_stats_t &launch_stats () const
    {
        return _batcher.launch_stats ();
    }

  private:
    friend class curve_engine_link_t;
    void on_encoded (uint64_t tag_, const uint8_t *wire_, size_t size_);
    void on_decoded (uint64_t tag_,
                     int status_,
                     const uint8_t *payload_,
                     size_t size_,
                     uint8_t flags_);
    curve_engine_link_t *find (uint64_t id_) const;
    //  call the events of every link marked since the last call, until no
    //  callback marks another
    void resume ();

    zmqg_ctx *const _ctx;
    int _fd;
    curve_batcher_t _batcher;
    std::map<uint64_t, curve_engine_link_t *> _links; //  live links by id
    uint64_t _next_id;
    std::vector<uint64_t> _out_ready, _in_ready; //  ids with new results
};

class curve_engine_link_t
{
  public:
    //  codec_: this connection's session (its ctx must be the hook's);
    //  events_: the engine's resume points (NULL: the engine polls
    //  next_encoded / next_decoded itself)
    curve_engine_link_t (curve_io_hook_t *hook_,
                         curve_encoding_gpu_t *codec_,
                         curve_link_events_t *events_ = NULL);
    ~curve_engine_link_t ();

    //  out side.  0, or -1 with errno (EMSGSIZE: larger than a batcher slot;
    //  EPIPE: the connection has failed)
    int submit_send (const uint8_t *data_, size_t size_, uint8_t msg_flags_);
    //  the next encoded MESSAGE command, in submission order
    bool next_encoded (std::vector<uint8_t> &wire_);
    //  the same without a copy: the command's bytes stay valid until the
    //  next pop_encoded or hook call
    bool peek_encoded (const uint8_t **wire_, size_t *size_) const;
    void pop_encoded () { _encoded.pop (); }

    //  in side: the body of one ZMTP MESSAGE frame.  0, or -1 with errno
    //  (EPIPE: the connection has already failed)
    int submit_received (const uint8_t *wire_, size_t size_);
    //  the next decoded message (payload, MORE/COMMAND flags), in receive
    //  order; after a failure only those decoded before it
    bool next_decoded (msg_buf_t &msg_);
    //  the same without a copy (valid until pop_decoded or a hook call)
    bool peek_decoded (const uint8_t **payload_,
                       size_t *size_,
                       uint8_t *flags_) const;
    void pop_decoded () { _decoded.pop (); }
    //  0, or the first failure's ZMQ_PROTOCOL_ERROR_ZMTP_* code
    int failed () const { return _failed; }

    size_t sends_in_flight () const { return _send_pending; }
    size_t receives_in_flight () const { return _recv_pending; }
    //  results delivered and not yet taken by next_encoded / next_decoded
    size_t encoded_queued () const { return _encoded.size (); }
    size_t decoded_queued () const { return _decoded.size (); }

  private:
    friend class curve_io_hook_t;
    curve_io_hook_t *const _hook;
    curve_encoding_gpu_t *const _codec;
    curve_link_events_t *const _events;
    const uint64_t _id;
    result_fifo_t _encoded, _decoded;
    size_t _send_pending, _recv_pending;
    int _failed;

    curve_engine_link_t (const curve_engine_link_t &);
    curve_engine_link_t &operator= (const curve_engine_link_t &);
};
}

#endif
