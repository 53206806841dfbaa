// curve_batcher.hpp -- asynchronous, batched CURVE MESSAGE codec for one
// I/O thread.
//
// The reference's stream engine runs the codec synchronously, one message
// per call, inside its event handlers: out_event pulls a message and encodes
// it (_next_msg = pull_and_encode, src/stream_engine_base.cpp:331-348, up to
// out_batch_size bytes per round, src/options.cpp:222), in_event decodes
// each MESSAGE frame the ZMTP decoder completes (:281-291, _process_msg =
// decode_and_push).  A per-message GPU call would be all launch latency, so
// this object sits between the engines of one I/O thread and the device:
//
//   engine (any connection)          curve_batcher_t                 device
//   -----------------------          ---------------                 ------
//   submit_encode(conn, msg)  ->  copy into the open pinned slot,
//                                  take the connection's next nonce
//   submit_decode(conn, wire) ->  copy into the open decode slot
//   flush()  (end of the poller   ->  launch each open slot as ONE   -> k_frames
//             iteration)               zmqg_*_batch on pinned memory    (zero-copy)
//   poll()   (every iteration)    ->  slots whose fence is reached,
//                                  in launch order: sink callbacks
//   on_encoded / on_decoded   <-   per message, per connection in
//                                  submission order
//
// Slots are page-locked, device-mapped host memory (zmqg_host_alloc): the
// kernels read the payload and write the result over PCIe in place, so the
// only host copies are the submit copy (the engine's own copy into its send
// or receive buffer in the reference) and whatever the sink does.  Decode
// runs in place inside the slot's input area: each payload is left at wire
// offset 33 of its frame, every byte over its own ciphertext byte (the
// reference's crypto_box_open_easy_afternm decrypts into message + 16,
// src/curve_mechanism_base.cpp:222-228, before its memmove).  Slots
// cycle free -> open -> in flight -> free; when none is free, a submit
// blocks on the oldest in-flight slot and delivers it (back-pressure).
//
// Semantics are the reference codec's, per connection: encode nonces are
// taken in submission order (get_and_inc_nonce,
// src/curve_mechanism_base.cpp:114-116), decode's replay rule sees a
// connection's frames in submission order across slots (one ctx, one
// stream), and per-message failures come back as the reference's
// ZMQ_PROTOCOL_ERROR_ZMTP_* codes (src/curve_mechanism_base.cpp:84-108,
// 277-281).  Single-threaded, like the I/O thread it serves.
#ifndef ZMQG_CURVE_BATCHER_HPP_INCLUDED
#define ZMQG_CURVE_BATCHER_HPP_INCLUDED

#include <stddef.h>
#include <stdint.h>

#include <deque>
#include <vector>

#include "curve_encoding_gpu.hpp"

namespace zmqg
{
//  Receives results.  Pointers are valid only during the callback (they
//  point into a slot that is recycled afterwards).
struct curve_sink_t
{
    virtual ~curve_sink_t () {}
    //  wire_: the MESSAGE command, wire_size_ bytes (a fresh msg_t with no
    //  flags, as msg_->move (msg_box) leaves it).
    virtual void on_encoded (uint64_t tag_,
                             const uint8_t *wire_,
                             size_t wire_size_) = 0;
    //  status_ 0: payload_/size_ hold the plaintext and flags_ the
    //  MORE/COMMAND bits to OR into the msg_t.  Otherwise status_ is the
    //  error_event_code and payload_ is NULL.
    virtual void on_decoded (uint64_t tag_,
                             int status_,
                             const uint8_t *payload_,
                             size_t size_,
                             uint8_t flags_) = 0;
};

class curve_batcher_t
{
  public:
    struct config_t
    {
        size_t slot_msgs;  //  messages per slot
        size_t slot_bytes; //  input bytes per slot (payloads or wire frames)
        int slots;         //  slots in rotation (>= 2)
        //  receive slots decoded with ZMQG_OPT_VERIFY_FIRST: the pinned slot
        //  never holds plaintext of a frame that fails (default on)
        bool verify_first;
        //  receive slots carry the host's header / replay verdict per frame
        //  (ZMQG_OPT_REPLAY_HOST, with verify_first): the batcher sees each
        //  connection's frames in order and applies check_validity's rules
        //  itself, so the device only authenticates and opens (two kernel
        //  launches a batch instead of seven).  Default on.
        bool replay_host;
        //  >= 0: every launched slot's fence also writes this eventfd when
        //  the stream reaches it (zmqg_fence_record_notify), so a poller
        //  sleeping on it wakes for the completion.  -1: fences only.
        int notify_fd;
        config_t () :
            slot_msgs (8192),
            slot_bytes (8u << 20),
            slots (4),
            verify_first (true),
            replay_host (true),
            notify_fd (-1)
        {
        }
    };

    //  All connections submitted must live on ctx_.  stream_: a hipStream_t
    //  for the batches (NULL: the ctx's own stream).
    curve_batcher_t (zmqg_ctx *ctx_,
                     curve_sink_t *sink_,
                     const config_t &config_ = config_t (),
                     void *stream_ = NULL);
    ~curve_batcher_t ();

    //  0 once the slots are allocated, -1 (errno) otherwise.
    int init ();

    //  Queue one message.  Return 0, or -1 with errno: EINVAL (bad
    //  argument, other ctx), EMSGSIZE (larger than a slot), EIO (device).
    int submit_encode (curve_encoding_gpu_t *conn_,
                       const uint8_t *data_,
                       size_t size_,
                       uint8_t msg_flags_,
                       uint64_t tag_);
    int submit_decode (curve_encoding_gpu_t *conn_,
                       const uint8_t *wire_,
                       size_t size_,
                       uint64_t tag_);

    //  Launch the open slots (those with messages).  0 or -1 (errno).
    int flush ();
    //  Deliver every finished slot, oldest first, without blocking.
    //  Returns the number of messages delivered, or -1 (errno).
    int poll ();
    //  flush () and wait for and deliver everything.  Messages or -1.
    int drain ();

    //  wait until no launched slot is still running (nothing delivered)
    int wait_idle ();

    size_t queued () const;    //  messages submitted and not yet launched
    size_t in_flight () const; //  messages launched and not yet delivered
    //  slots launched and not yet delivered
    size_t batches_in_flight () const { return _flight.size (); }

    //  host time spent in the device calls of launch (): the batch call and
    //  the fence (+ notification), nanoseconds since construction
    struct launch_stats_t
    {
        uint64_t batch_ns, fence_ns, launches;
    };
    const launch_stats_t &launch_stats () const { return _stats; }

  private:
    enum kind_t
    {
        encode_kind,
        decode_kind
    };
    struct slot_t
    {
        uint8_t *base;
        //  descriptor arrays and data, all inside the pinned block
        uint32_t *sid;
        uint64_t *nonce;
        uint8_t *flags;
        uint64_t *in_off;
        uint32_t *len; //  payload length (encode) / wire length (decode)
        uint64_t *out_off;
        uint8_t *flags_out;
        int32_t *status;
        int32_t *verdict; //  decode: the host's verdict (replay_host)
        uint8_t *in;
        uint8_t *out;
        std::vector<uint64_t> tags;
        kind_t kind;
        size_t n, in_used, out_used;
        uint64_t max_len; //  longest payload (encode) / wire frame (decode) so far
        uint64_t fence;
    };

    int open_slot (kind_t kind_, size_t in_need_, size_t out_need_);
    int launch (slot_t *slot_);
    int deliver (slot_t *slot_);
    int wait_oldest ();

    zmqg_ctx *const _ctx;
    curve_sink_t *const _sink;
    const config_t _config;
    void *_stream;
    size_t _out_cap;
    std::vector<slot_t> _slots;
    std::vector<slot_t *> _free;
    slot_t *_open[2];
    std::deque<slot_t *> _flight;
    launch_stats_t _stats;

    curve_batcher_t (const curve_batcher_t &);
    curve_batcher_t &operator= (const curve_batcher_t &);
};
}

#endif
