/*
 * zmqg_curve.h -- C ABI of the MI355X CurveZMQ MESSAGE AEAD path.
 *
 * This is the drop-in boundary for libzmq's CURVE message codec:
 *
 *   reference call                                   replaced by
 *   -----------------------------------------------  ---------------------------
 *   curve_encoding_t::encode
 *     src/curve_mechanism_base.cpp:111-205           zmqg_encode_batch
 *     (crypto_box_easy_afternm :172-174)
 *   curve_mechanism_base_t::decode
 *     src/curve_mechanism_base.cpp:38-52             zmqg_decode_batch
 *     check_basic_command_structure
 *       src/mechanism_base.cpp:14-25
 *     curve_encoding_t::decode / check_validity
 *       src/curve_mechanism_base.cpp:80-109, 207-284
 *     (crypto_box_open_easy_afternm :226-228)
 *   curve_encoding_t state (_cn_precom, prefixes,
 *     _downgrade_sub, _cn_peer_nonce)
 *     src/curve_mechanism_base.hpp:44-58             zmqg_session_set,
 *                                                    zmqg_session_*_peer_nonce
 *   curve_encoding_t::get_writable_precom_buffer
 *     src/curve_mechanism_base.hpp:36                zmqg_session_set (precom)
 *   curve_encoding_t::set_peer_nonce
 *     src/curve_mechanism_base.hpp:42                zmqg_session_set_peer_nonce
 *   curve_encoding_t::get_and_inc_nonce (_cn_nonce)
 *     src/curve_mechanism_base.hpp:41                ZMQG_OPT_NONCE_AUTO,
 *                                                    zmqg_session_*_nonce
 *
 * One call processes a batch of independent MESSAGE frames.  Each frame
 * belongs to a session (one CURVE connection = one curve_encoding_t).  The
 * caller assigns encode nonces, or lets the device take them from each
 * session's send counter (ZMQG_OPT_NONCE_AUTO; the reference's
 * get_and_inc_nonce, src/curve_mechanism_base.hpp:41).  Decode applies the reference's replay
 * rule exactly as if curve_encoding_t::decode had been called on the batch's
 * frames one by one in batch order, and updates each session's peer nonce.
 *
 * Conventions
 *   - Return 0 on success, a negative errno value on failure (-EINVAL bad
 *     argument, -ENOMEM, -EIO a HIP runtime error).  Per-frame protocol
 *     errors are not call failures: they are reported in status_out with the
 *     reference's codes (ZMQ_PROTOCOL_ERROR_ZMTP_*, include/zmq.h:424-437).
 *   - Batch pointers (descriptors, in, out, flags_out, status_out) must be
 *     device memory of the ctx's device, or host memory the device can
 *     access (hipHostMalloc).  Batch calls are asynchronous on `stream`
 *     (a hipStream_t; NULL = the null stream); results are valid once the
 *     stream has been synchronised.
 *   - A ctx is externally synchronised, like the reference's mechanism (one
 *     I/O thread per connection): issue one ctx's batches on one stream.
 *   - No exceptions cross this boundary.
 */
#ifndef ZMQG_CURVE_H_INCLUDED
#define ZMQG_CURVE_H_INCLUDED

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ZMQG_CURVE_ABI_VERSION 5

/* Per-frame status codes, identical to include/zmq.h:424-437. */
#define ZMQG_STATUS_OK 0
#define ZMQG_ERR_UNEXPECTED_COMMAND 0x10000001  /* ZMQ_PROTOCOL_ERROR_ZMTP_UNEXPECTED_COMMAND */
#define ZMQG_ERR_INVALID_SEQUENCE 0x10000002    /* ZMQ_PROTOCOL_ERROR_ZMTP_INVALID_SEQUENCE */
#define ZMQG_ERR_MALFORMED_UNSPECIFIED 0x10000011 /* ..._MALFORMED_COMMAND_UNSPECIFIED */
#define ZMQG_ERR_MALFORMED_MESSAGE 0x10000012   /* ..._MALFORMED_COMMAND_MESSAGE */
#define ZMQG_ERR_CRYPTOGRAPHIC 0x11000001       /* ZMQ_PROTOCOL_ERROR_ZMTP_CRYPTOGRAPHIC */
/* Library codes (not protocol errors; the reference has no equivalent):
 * ZMQG_ERR_SESSION  sid[i] >= the ctx's max_sessions (the frame is not
 *                   processed; decode: payload region zero-filled as for a
 *                   header failure)
 * ZMQG_ERR_BOUND    the frame is longer than zmqg_batch_opts.max_len (the
 *                   caller's promise was broken; the frame is not processed
 *                   and its output region is left as it was) */
#define ZMQG_ERR_SESSION 0x7a000001
#define ZMQG_ERR_BOUND 0x7a000002

/* msg_t flag bits used on this path (src/msg.hpp:55-62). */
#define ZMQG_MSG_MORE 1
#define ZMQG_MSG_COMMAND 2
#define ZMQG_MSG_SUBSCRIBE 12
#define ZMQG_MSG_CANCEL 16

typedef struct zmqg_ctx zmqg_ctx;

/* ABI version of the loaded library (== ZMQG_CURVE_ABI_VERSION). */
int zmqg_abi_version(void);

/* Create a context on HIP device `device` with a session table of
 * `max_sessions` entries (sids 0 .. max_sessions-1). */
int zmqg_ctx_create(int device, uint32_t max_sessions, zmqg_ctx **ctx_out);
int zmqg_ctx_destroy(zmqg_ctx *ctx);

/* Install session `sid`: the connection's precomputed key (_cn_precom, the
 * output of crypto_box_beforenm, src/curve_client_tools.hpp:105 /
 * src/curve_server.cpp:382-383), the 16-byte encode/decode nonce prefixes
 * ("CurveZMQMESSAGEC"/"CurveZMQMESSAGES" swapped per side,
 * src/curve_client.cpp:22-23, src/curve_server.cpp:24-25), the downgrade_sub
 * flag (src/zmtp_engine.cpp:339-351) and the initial peer nonce (the
 * reference starts at 1 and the handshake advances it).  The two XSalsa20
 * subkeys HSalsa20(precom, prefix) are derived on the device.  Synchronous. */
int zmqg_session_set(zmqg_ctx *ctx, uint32_t sid, const uint8_t precom[32], const uint8_t enc_prefix[16],
                     const uint8_t dec_prefix[16], int downgrade_sub, uint64_t peer_nonce);

/* Install n sessions in one launch, asynchronously on `stream`: the mass
 * handshake's counterpart of zmqg_session_set (each server connection's
 * precom comes from crypto_box_beforenm at src/curve_server.cpp:382-383, each
 * client's at src/curve_client_tools.hpp:105; zmqg_box_beforenm_batch
 * derives them on the device and its k_out is passed here as is).
 *   sid          host array: n distinct session ids below max_sessions
 *                (-EINVAL otherwise)
 *   precom       device-accessible, 4-byte aligned: session i's 32-byte
 *                precomputed key at precom[32*i]
 *   enc_prefix, dec_prefix   the 16-byte nonce prefixes, common to the batch
 *                (one side's connections all use the same pair)
 *   downgrade    host array of n downgrade_sub flags, or NULL (all 0)
 *   peer_nonce   host array of n initial peer nonces, or NULL (all 1)
 * The send nonce of each session starts at 1, as with zmqg_session_set.
 * The host arrays are copied before the call returns; the install runs on
 * `stream` (batch calls issued after it on that stream see the sessions),
 * and the ctx's accessors order after it.  A second install waits for the
 * first to have read its descriptors. */
int zmqg_session_set_batch(zmqg_ctx *ctx, uint64_t n, const uint32_t *sid, const uint8_t *precom,
                           const uint8_t enc_prefix[16], const uint8_t dec_prefix[16], const uint8_t *downgrade,
                           const uint64_t *peer_nonce, void *stream);
/* The same with each session's send nonce: send_nonce is a host array of n
 * initial send nonces, or NULL (all 1).  A connection installed after its
 * handshake continues from the handshake's nonces -- the client's MESSAGE
 * nonces start at 3 after HELLO (1) and INITIATE (2), src/curve_client.cpp
 * and curve_client_tools.hpp; the server's at 2 after READY (1) -- so a
 * mass install needs no zmqg_session_set_nonce call per session. */
int zmqg_session_set_batch_ex(zmqg_ctx *ctx, uint64_t n, const uint32_t *sid, const uint8_t *precom,
                              const uint8_t enc_prefix[16], const uint8_t dec_prefix[16], const uint8_t *downgrade,
                              const uint64_t *peer_nonce, const uint64_t *send_nonce, void *stream);

/* curve_encoding_t::set_peer_nonce / read back _cn_peer_nonce.  Synchronous:
 * they are ordered after the work previously issued on the stream of the
 * ctx's last batch call (no device-wide synchronisation). */
int zmqg_session_set_peer_nonce(zmqg_ctx *ctx, uint32_t sid, uint64_t peer_nonce);
int zmqg_session_get_peer_nonce(zmqg_ctx *ctx, uint32_t sid, uint64_t *peer_nonce_out);

/* The session's send nonce (_cn_nonce, src/curve_mechanism_base.hpp:41-50):
 * the next nonce zmqg_encode_batch_ex assigns under ZMQG_OPT_NONCE_AUTO.
 * zmqg_session_set starts it at 1, as the reference's constructor does
 * (src/curve_mechanism_base.cpp:59); set it after the handshake has used its
 * nonces.  Synchronous, ordered like the peer-nonce accessors. */
int zmqg_session_set_nonce(zmqg_ctx *ctx, uint32_t sid, uint64_t nonce);
int zmqg_session_get_nonce(zmqg_ctx *ctx, uint32_t sid, uint64_t *nonce_out);

/* Bytes of the encoded frame for a payload of `payload_len` bytes and msg_t
 * flags `msg_flags`: "\x07MESSAGE"(8) + nonce(8) + tag(16) + mlen, where
 * mlen = 1 + [1 | 7 | 10 for SUBSCRIBE/CANCEL] + payload_len
 * (src/curve_mechanism_base.cpp:113-128, 169). */
uint64_t zmqg_wire_size(uint8_t msg_flags, int downgrade_sub, uint64_t payload_len);

/* Encode n frames (curve_encoding_t::encode).  Frame i: session sid[i],
 * nonce nonce[i], msg_t flags flags[i], payload in[in_off[i] .. +len[i]).
 * Writes zmqg_wire_size(flags[i], session.downgrade_sub, len[i]) bytes at
 * out[out_off[i]]: "\x07MESSAGE" || BE64(nonce) || tag || ciphertext.
 * Output frames must not overlap each other or the input.  sid[i] must be
 * below max_sessions: a frame with another sid is not encoded (its output
 * region is left as it was; zmqg_encode_batch_ex reports it). */
int zmqg_encode_batch(zmqg_ctx *ctx, uint64_t n, const uint32_t *sid, const uint64_t *nonce, const uint8_t *flags,
                      const uint64_t *in_off, const uint32_t *len, const uint8_t *in, const uint64_t *out_off,
                      uint8_t *out, void *stream);

/* Decode n frames (curve_mechanism_base_t::decode).  Frame i: session sid[i],
 * wire bytes in[in_off[i] .. +wire_len[i]).  On success status_out[i] = 0,
 * flags_out[i] = plaintext flags & (MORE|COMMAND) (the caller ORs them into
 * the msg_t, as msg_t::set_flags does, src/msg.cpp:433-436) and the payload,
 * wire_len[i] - 33 bytes, is written at out[out_off[i]].  On failure
 * status_out[i] is the reference's error code, flags_out[i] = 0 and, when
 * wire_len[i] >= 33, the payload region is zero-filled: plaintext of a frame
 * that failed is never left in `out`.  Each session's peer nonce advances as
 * the reference's check_validity does (src/curve_mechanism_base.cpp:98-106,
 * including on a later MAC failure).
 *
 * In-place decode: `out` may be `in`, with every frame in one of two
 * layouts: out_off[i] = in_off[i] + 33, each payload byte over its own
 * ciphertext byte (the reference's crypto_box_open_easy_afternm decrypts
 * into message + 16, src/curve_mechanism_base.cpp:222-228, which puts the
 * flags byte at wire offset 16 and the payload at 17 -- a different layout,
 * not offered here), or out_off[i] = in_off[i], the payload at the frame's
 * start as after the reference's memmove (:253-260).  Otherwise `out` must not overlap `in`.  On
 * failure the payload region is zero-filled as above; in the second layout a
 * frame of more than 4.5 KiB that fails has its whole wire region zeroed.
 *
 * Unauthenticated plaintext: the kernels decrypt and authenticate in one
 * pass, so until the call has completed on its stream, `out` may hold
 * plaintext of frames that then fail (it is zeroed before completion).  The
 * reference's libsodium verifies first and writes nothing for a forged frame
 * (SURVEY.md a12).  Results at completion are identical; a caller whose
 * `out` is visible to another party while the call runs (e.g. mapped host
 * memory read by a second thread) sets ZMQG_OPT_VERIFY_FIRST
 * (zmqg_decode_batch_ex), under which `out` only ever receives verified
 * payloads and zeros. */
int zmqg_decode_batch(zmqg_ctx *ctx, uint64_t n, const uint32_t *sid, const uint64_t *in_off,
                      const uint32_t *wire_len, const uint8_t *in, const uint64_t *out_off, uint8_t *out,
                      uint8_t *flags_out, int32_t *status_out, void *stream);

/* Options of the _ex batch calls (every field optional: a zeroed struct, or
 * opts = NULL, gives the plain calls' behaviour).
 *   size             sizeof(zmqg_batch_opts) (ABI check)
 *   flags            ZMQG_OPT_NONCE_AUTO (encode): ignore `nonce` (it may be
 *                    NULL) and take each frame's nonce from its session's
 *                    send counter on the device, in batch order, as
 *                    curve_encoding_t::get_and_inc_nonce does per message
 *                    (src/curve_mechanism_base.hpp:41, called at
 *                    src/curve_mechanism_base.cpp:116); the counters advance
 *                    by each session's frame count.  Several sessions: at
 *                    most 8192 (-EINVAL above).
 *   max_len          0, or a bound on every len[i] (encode) / wire_len[i]
 *                    (decode).  A bound under which every frame fits the frame
 *                    kernel (stream <= 4.5 KiB: decode wire_len <= 4608, encode
 *                    len <= 4565) lets the call skip the large-frame kernels
 *                    (two fewer launches).  A frame above the bound fails with
 *                    ZMQG_ERR_BOUND.
 *   status_out       encode only: n entries (device-accessible), 0 or
 *                    ZMQG_ERR_SESSION / ZMQG_ERR_BOUND per frame.
 *   session_max_out  decode only: max_sessions entries (device-accessible):
 *                    per session, the largest header-valid nonce among this
 *                    batch's frames (0 where it has none) -- the value a rank
 *                    contributes to shard.peer_prefix when a session's frames
 *                    span GPUs.
 *   flags            ZMQG_OPT_VERIFY_FIRST (decode): no byte of `out` is
 *                    written before the frame's tag and replay verdict, as
 *                    libsodium's open verifies before it decrypts
 *                    (src/curve_mechanism_base.cpp:226-228).  The frames are
 *                    decoded into a device staging area of the ctx laid out
 *                    like `out`, then one kernel copies each verified payload
 *                    to out[out_off[i]] and zero-fills the payload region of
 *                    each failed one (a frame above max_len, or shorter than
 *                    33 bytes, is left as it was).  Needs out_bytes.  For
 *                    `out` another party can read while the call runs (mapped
 *                    host memory: curve_batcher_t's receive slots).  Costs one
 *                    extra read and write of the payload bytes.
 *   out_bytes        extent of `out`: every out_off[i] + wire_len[i] - 33 is
 *                    at most this (required by ZMQG_OPT_VERIFY_FIRST, which
 *                    checks it on the device: a frame whose payload region
 *                    would end past out_bytes fails with ZMQG_ERR_BOUND and
 *                    nothing of it is written; 0 is valid for a batch whose
 *                    frames carry no payload bytes).
 *   flags            ZMQG_OPT_REPLAY_HOST (decode, with VERIFY_FIRST and
 *                    verdict_in): the caller has already applied the header
 *                    rules and the replay rule to the frames in batch order,
 *                    as check_basic_command_structure and check_validity do
 *                    (src/mechanism_base.cpp:14-25,
 *                    src/curve_mechanism_base.cpp:80-106: the nonce must
 *                    exceed the connection's peer nonce, which advances
 *                    before the MAC), keeping the connections' peer nonces
 *                    itself -- a host that sees every frame in order does
 *                    this with one compare per frame.  The device then only
 *                    authenticates and opens: it neither reads nor writes its
 *                    sessions' peer nonces (zmqg_session_set_peer_nonce
 *                    before a later call that does), and the call is two
 *                    kernel launches instead of seven for several sessions.
 *   verdict_in       with ZMQG_OPT_REPLAY_HOST: n entries (device-accessible),
 *                    per frame 0 (open it) or the ZMQG_ERR_* code the host's
 *                    rules gave it, which is then the frame's status (its
 *                    payload region zero-filled, flags 0).
 *   flags            ZMQG_OPT_STREAM_OUT (decode, and encode in
 *                    zmqg_encode_batch_ex): a cache hint, results unchanged.
 *                    The outputs go to memory the device's caches do not
 *                    hold (batches rotating over more buffers than the 256
 *                    MiB Infinity Cache keeps, as a receive ring does): each
 *                    64-byte output piece is staged through LDS and leaves a
 *                    step later with 15 other frames' in one store
 *                    instruction, instead of each lane's own 16-byte pieces.
 *                    Config 2 from HBM: decode 60 against 75 us, encode 66
 *                    against 71 us; with the output lines already cached it
 *                    costs the decode ~5 us.
 *                    Applies to the one-lane-per-frame kernel; on decode
 *                    when every payload starts 64-byte aligned.
 * A caller built against the struct without out_bytes (or verdict_in)
 * passes the smaller size and gets the old behaviour. */
#define ZMQG_OPT_NONCE_AUTO 1u
#define ZMQG_OPT_VERIFY_FIRST 2u
#define ZMQG_OPT_REPLAY_HOST 4u
#define ZMQG_OPT_STREAM_OUT 8u
typedef struct zmqg_batch_opts {
    uint32_t size;
    uint32_t flags;
    uint64_t max_len;
    int32_t *status_out;
    uint64_t *session_max_out;
    uint64_t out_bytes;
    const int32_t *verdict_in;
} zmqg_batch_opts;
int zmqg_encode_batch_ex(zmqg_ctx *ctx, uint64_t n, const uint32_t *sid, const uint64_t *nonce, const uint8_t *flags,
                         const uint64_t *in_off, const uint32_t *len, const uint8_t *in, const uint64_t *out_off,
                         uint8_t *out, const zmqg_batch_opts *opts, void *stream);
int zmqg_decode_batch_ex(zmqg_ctx *ctx, uint64_t n, const uint32_t *sid, const uint64_t *in_off,
                         const uint32_t *wire_len, const uint8_t *in, const uint64_t *out_off, uint8_t *out,
                         uint8_t *flags_out, int32_t *status_out, const zmqg_batch_opts *opts, void *stream);

/* Header pass of a sharded decode: writes
 * session_max_out[s] (max_sessions entries, device-accessible) = the largest
 * header-valid nonce among the n wire frames of session s (0 where none).
 * When one session's frames are split over ranks (GPUs), rank r decodes its
 * slice after setting each session's peer nonce to max(peer before the batch,
 * the session maxima of ranks < r) -- the exclusive max-scan over ranks of
 * these vectors (libzmq_amd/shard.py peer_prefix) -- and the slices' results
 * equal one decode of the whole batch.  Reads 16 bytes per frame.
 * Asynchronous on `stream`. */
int zmqg_session_max_batch(zmqg_ctx *ctx, uint64_t n, const uint32_t *sid, const uint64_t *in_off,
                           const uint32_t *wire_len, const uint8_t *in, uint64_t *session_max_out, void *stream);

/* Host-memory convenience forms of the two batch calls: every pointer is
 * ordinary (pageable) host memory.  They stage through the ctx's pinned
 * buffers with hipMemcpyAsync H2D, run the batch and copy back D2H, and
 * return after the stream has synchronised.  This is the path an I/O thread
 * calling with socket buffers takes. */
int zmqg_encode_host(zmqg_ctx *ctx, uint64_t n, const uint32_t *sid, const uint64_t *nonce, const uint8_t *flags,
                     const uint64_t *in_off, const uint32_t *len, const uint8_t *in, uint64_t in_bytes,
                     const uint64_t *out_off, uint8_t *out, uint64_t out_bytes);
int zmqg_decode_host(zmqg_ctx *ctx, uint64_t n, const uint32_t *sid, const uint64_t *in_off,
                     const uint32_t *wire_len, const uint8_t *in, uint64_t in_bytes, const uint64_t *out_off,
                     uint8_t *out, uint64_t out_bytes, uint8_t *flags_out, int32_t *status_out);

/* One message on one session, host memory in and out: the call the
 * reference engine makes per message (curve_encoding_t::encode / decode,
 * src/curve_mechanism_base.cpp:111-205, :207-284, from
 * src/stream_engine_base.cpp:331-348 / :281-291) without descriptor arrays.
 * The bytes are copied once into the ctx's page-locked, device-mapped
 * message buffer, the frame kernel works on it in place over PCIe (no
 * hipMemcpy), and the result is copied once out of it after the stream
 * has synchronised.
 *
 * zmqg_encode_msg: `out` receives zmqg_wire_size(flags, downgrade of sid,
 * len) bytes, the MESSAGE command for `nonce`.
 * zmqg_decode_msg: `out` receives wire_len - 33 payload bytes (`out` may be
 * `in`: the payload then starts at in[0]; a frame shorter than 33 bytes
 * fails its header checks and needs no room), *flags_out the
 * plaintext MORE / COMMAND bits and *status_out 0 or the
 * ZMQ_PROTOCOL_ERROR_ZMTP_* code; on a failure `out` is left untouched and
 * the session's peer nonce advances as the reference's does.
 * Both return 0 or -errno (-EINVAL for bad arguments). */
int zmqg_encode_msg(zmqg_ctx *ctx, uint32_t sid, uint64_t nonce, uint8_t flags, const uint8_t *in, uint32_t len,
                    uint8_t *out);
int zmqg_decode_msg(zmqg_ctx *ctx, uint32_t sid, const uint8_t *in, uint32_t wire_len, uint8_t *out,
                    uint8_t *flags_out, int32_t *status_out);

/* Asynchronous host path.  The reference's
 * engine encodes and decodes one message at a time on the I/O thread
 * (src/stream_engine_base.cpp:281-291 in_event, :331-348 out_event); an
 * engine that batches across its connections instead needs host memory the
 * kernels can work on in place and a way to learn, without blocking, that a
 * submitted batch is finished.
 *
 * zmqg_host_alloc returns page-locked host memory mapped into the device's
 * address space: batch calls take pointers into it directly (descriptors,
 * `in`, `out`, flags_out, status_out) and the kernels read and write it over
 * PCIe with no staging copy.  Free it with zmqg_host_free (after the batches
 * using it have finished).
 *
 * zmqg_ctx_stream gives the ctx's own non-blocking stream for callers without
 * one.  zmqg_fence_record marks the point after everything issued so far on
 * `stream` and returns a fence id (ids increase per ctx); zmqg_fence_query
 * returns 1 once the stream has passed it, 0 while it has not (never
 * blocks), and zmqg_fence_wait blocks until it has.  A fence is released by
 * the first query or wait that finds it reached; later queries of a released
 * or unknown id below the last issued one return 1. */
int zmqg_host_alloc(zmqg_ctx *ctx, uint64_t bytes, void **ptr_out);
int zmqg_host_free(zmqg_ctx *ctx, void *ptr);
int zmqg_ctx_stream(zmqg_ctx *ctx, void **stream_out);
int zmqg_fence_record(zmqg_ctx *ctx, void *stream, uint64_t *fence_out);
int zmqg_fence_query(zmqg_ctx *ctx, uint64_t fence);
int zmqg_fence_wait(zmqg_ctx *ctx, uint64_t fence);

/* Completion wake-up for a sleeping I/O thread.  The reference's I/O thread
 * sleeps in epoll_wait (src/epoll.cpp:157-158) and is woken only by a file
 * descriptor it watches -- its mailbox's eventfd (src/io_thread.cpp:54,
 * src/signaler.cpp) or a socket; an engine with nothing to write has reset
 * POLLOUT (src/stream_engine_base.cpp:350-353) and resumes only through
 * restart_output / restart_input (:383-390, :400-442).
 *
 * zmqg_fence_record_notify is zmqg_fence_record plus a wake-up: once the
 * stream has passed the fence, an 8-byte 1 is written to `fd` (eventfd
 * counter semantics; a pipe's write end works too) from a HIP runtime thread,
 * and from then on zmqg_fence_query of that fence returns 1.  The poller
 * watches `fd` for POLLIN, reads it, and polls its fences.  `fd` must stay
 * open until zmqg_notify_quiesce has returned 0: that call waits until every
 * notification enqueued on the ctx so far has been delivered (the streams
 * must be able to reach them), at most ~10 s: -ETIMEDOUT then (a stuck
 * stream), and `fd` must stay open.  zmqg_ctx_destroy waits for them too and,
 * on such a timeout, returns -ETIMEDOUT with the ctx's host state left
 * allocated for the late host functions.  If the fence is recorded but its
 * notification cannot be queued, the call fails with *fence_out set (the
 * fence can still be waited for); a failure before the fence leaves it 0.
 * (Replaces no reference symbol: the reference codec is synchronous.) */
int zmqg_fence_record_notify(zmqg_ctx *ctx, void *stream, int fd, uint64_t *fence_out);
int zmqg_notify_quiesce(zmqg_ctx *ctx);

/* ZMTP framing on the device.
 *
 * zmqg_encode_zmtp: zmqg_encode_batch plus the engine's ZMTP encoder
 * (src/v3_1_encoder.cpp:23-60) in one call: the n encoded MESSAGE commands
 * are laid out back to back in `out` as ZMTP frames -- flags (0, or LARGE
 * when the body exceeds 255 bytes; the boxed msg_t carries no MORE/COMMAND,
 * src/curve_mechanism_base.cpp:166-177), size (1 byte, or 8 bytes big
 * endian), body -- ready to be written to the socket.  frame_off[0..n]
 * (device-accessible, n + 1 entries) receives each frame's offset and the
 * total in frame_off[n]; offsets are computed on the device.  Asynchronous.
 *
 * zmqg_decode_zmtp: the engine's ZMTP decoder (src/v2_decoder.cpp:35-140)
 * and curve_mechanism_base_t::decode over a received byte stream of one
 * connection (session sid), on the device.  Frames are found from offset 0;
 * up to max_frames of them are decoded: frame i's body is
 * in[frame_in_off[i] .. +frame_len[i]), its payload (frame_len[i] - 33
 * bytes) is written at out[out_off[i]] with out_off[i] = frame_in_off[i] --
 * the body's own offset, so `out` may be `in` (decoded in place, each
 * payload left at its body's start as after the reference's memmove,
 * src/curve_mechanism_base.cpp:253-260: a received buffer becomes the
 * messages' data without a copy, as v2_decoder's zero-copy msg_t slices do,
 * src/v2_decoder.cpp:88-113) -- and flags_out / status_out are as for zmqg_decode_batch,
 * with the ZMTP frame's MORE / COMMAND bits ORed into flags_out of a
 * decoded frame (msg_t::set_flags ORs, src/msg.cpp:433-436).  result:
 * frames returned, bytes of `in` they cover (an incomplete last frame is
 * left for the next call), payload bytes written (their sum), and error = EMSGSIZE when
 * a frame's size exceeds max_msg_size (>= 0; -1 = no limit), where the
 * reference decoder fails (src/v2_decoder.cpp:74-84): the frames before it
 * are returned.  A size above 2^32 - 1 also ends the parse with EMSGSIZE:
 * that is a restriction of this library (frame lengths are 32-bit), not
 * reference behaviour -- on LP64 the reference's size_t check
 * (src/v2_decoder.cpp:78) never fires and it would accept such a frame.  A complete frame that is not a MESSAGE command
 * is returned as the last frame, with the status the mechanism gives it;
 * the reference's engine stops at the first failing frame, and so should
 * the caller.  Arrays hold max_frames entries (entries from result.frames
 * on hold empty frames: length 0, a malformed status); `out` at least
 * in_bytes.  Returns after the stream has synchronised: the result is the
 * call's only read back (the frame count stays on the device; the decode
 * runs over max_frames).  in_bytes < 2^31.
 *
 * zmqg_decode_zmtp_async: the same, without synchronising: `result` must be
 * device-accessible (device memory, or pinned host memory from
 * zmqg_host_alloc) and holds the result once the stream reaches this point
 * (zmqg_fence_record / _query). */
typedef struct zmqg_zmtp_result {
    uint64_t frames;
    uint64_t consumed;
    uint64_t out_bytes;
    int32_t error;
    int32_t pad;
} zmqg_zmtp_result;
int zmqg_encode_zmtp(zmqg_ctx *ctx, uint64_t n, const uint32_t *sid, const uint64_t *nonce, const uint8_t *flags,
                     const uint64_t *in_off, const uint32_t *len, const uint8_t *in, uint8_t *out,
                     uint64_t *frame_off, void *stream);
int zmqg_decode_zmtp(zmqg_ctx *ctx, uint32_t sid, const uint8_t *in, uint64_t in_bytes, int64_t max_msg_size,
                     uint64_t max_frames, uint64_t *frame_in_off, uint32_t *frame_len, uint64_t *out_off,
                     uint8_t *out, uint8_t *flags_out, int32_t *status_out, zmqg_zmtp_result *result,
                     void *stream);
int zmqg_decode_zmtp_async(zmqg_ctx *ctx, uint32_t sid, const uint8_t *in, uint64_t in_bytes, int64_t max_msg_size,
                           uint64_t max_frames, uint64_t *frame_in_off, uint32_t *frame_len, uint64_t *out_off,
                           uint8_t *out, uint8_t *flags_out, int32_t *status_out, zmqg_zmtp_result *result,
                           void *stream);

/* Handshake key derivation in batches, one
 * 32-byte item per thread, items packed back to back:
 *   zmqg_scalarmult_batch: crypto_scalarmult_curve25519(out, scalar, point)
 *     (libsodium 1.0.18; RFC 7748 X25519): status -1 where the result is all
 *     zero (a small-order point), else 0.  point == NULL: the base point, as
 *     crypto_scalarmult_base for zmq_curve_public (src/zmq_utils.cpp:222-245);
 *     status always 0.
 *   zmqg_box_beforenm_batch: crypto_box_beforenm(k, pk, sk) =
 *     HSalsa20(X25519(sk, pk), 0^16), the connection's precomputed key
 *     (src/curve_client_tools.hpp:105, src/curve_server.cpp:382-383; the
 *     reference asserts success): status -1 and k not written where the
 *     scalar multiplication fails.
 * Asynchronous on `stream`; pointers as for the batch calls. */
int zmqg_scalarmult_batch(zmqg_ctx *ctx, uint64_t n, const uint8_t *scalar, const uint8_t *point, uint8_t *out,
                          int32_t *status_out, void *stream);
int zmqg_box_beforenm_batch(zmqg_ctx *ctx, uint64_t n, const uint8_t *pk, const uint8_t *sk, uint8_t *k_out,
                            int32_t *status_out, void *stream);

/* Handshake boxes in batches: every CURVE
 * command body is one crypto_box / crypto_secretbox with its own key and
 * 24-byte nonce -- HELLO (src/curve_client_tools.hpp:45), WELCOME
 * (src/curve_server.cpp:232, opened at src/curve_client_tools.hpp:92), the
 * cookie (src/curve_server.cpp:208, :334), INITIATE's vouch and box
 * (src/curve_client_tools.hpp:140, :177; src/curve_server.cpp:291, :359) and
 * READY (src/curve_server.cpp:441, src/curve_client.cpp:206).  With
 * crypto_box(pk, sk) = crypto_box_afternm(crypto_box_beforenm(pk, sk)) and
 * crypto_secretbox(k) = crypto_box_afternm(k) (libsodium 1.0.18), these two
 * calls plus zmqg_box_beforenm_batch seal and open all of them.  Item i:
 * key[32i .. +32], nonce[24i .. +24], input in[in_off[i] .. +len[i]], output
 * at out[out_off[i]] (the "easy" layouts: no NaCl zero padding).
 *   zmqg_box_afternm_batch: crypto_box_easy_afternm -- writes
 *     tag(16) || ciphertext(len[i]).
 *   zmqg_box_open_afternm_batch: crypto_box_open_easy_afternm -- reads
 *     tag || ciphertext (len[i] bytes), writes len[i] - 16 plaintext bytes,
 *     status_out[i] = 0; -1 where len[i] < 16 or the tag does not verify
 *     (checked before any plaintext is written; the region is then
 *     zero-filled).
 * One thread per box; inputs and outputs must not overlap.  Asynchronous on
 * `stream`; pointers as for the batch calls. */
int zmqg_box_afternm_batch(zmqg_ctx *ctx, uint64_t n, const uint8_t *key, const uint8_t *nonce,
                           const uint64_t *in_off, const uint32_t *len, const uint8_t *in, const uint64_t *out_off,
                           uint8_t *out, void *stream);
int zmqg_box_open_afternm_batch(zmqg_ctx *ctx, uint64_t n, const uint8_t *key, const uint8_t *nonce,
                                const uint64_t *in_off, const uint32_t *len, const uint8_t *in,
                                const uint64_t *out_off, uint8_t *out, int32_t *status_out, void *stream);

/* Batched Z85 key codec: zmq_z85_encode /
 * zmq_z85_decode (src/zmq_utils.cpp:100-180, include/zmq.h:537-540) over n
 * independent items, one per thread.  Item i: input bytes
 * in[in_off[i] .. +len[i]), output at out[out_off[i]]; status_out[i] = 0 or
 * EINVAL where the reference returns NULL with errno EINVAL.
 *   encode: len % 4 == 0, writes len * 5 / 4 characters and a NUL.
 *   decode: len = strlen of the string (>= 5, multiple of 5), writes
 *     len * 4 / 5 bytes; an invalid character or a group above 0xffffffff
 *     fails the item after the groups before it were written, as the
 *     reference's loop does.
 * Pointers as for the batch calls (device or device-accessible host memory);
 * asynchronous on `stream`. */
int zmqg_z85_encode_batch(zmqg_ctx *ctx, uint64_t n, const uint64_t *in_off, const uint32_t *len, const uint8_t *in,
                          const uint64_t *out_off, char *out, int32_t *status_out, void *stream);
int zmqg_z85_decode_batch(zmqg_ctx *ctx, uint64_t n, const uint64_t *in_off, const uint32_t *len, const char *in,
                          const uint64_t *out_off, uint8_t *out, int32_t *status_out, void *stream);

/* Profiling hooks (off by default).  When enabled, the ctx records a HIP
 * event pair on the batch's stream around each of its kernels of one kind:
 *   ZMQG_PROF_ENCODE_MAIN / ZMQG_PROF_DECODE_MAIN  the frame kernel alone
 *     (every frame up to 4.5 KiB of stream: the dominant kernel),
 *   ZMQG_PROF_ENCODE_CALL / ZMQG_PROF_DECODE_CALL  the whole batch call,
 *   ZMQG_PROF_ENCODE_BODY / ZMQG_PROF_DECODE_BODY  the chunked body kernel
 *     (larger frames) alone.
 * zmqg_ctx_get_profile synchronises the device, returns the summed elapsed
 * milliseconds and launch count for `kind` since the last reset, and resets. */
#define ZMQG_PROF_ENCODE_MAIN 0
#define ZMQG_PROF_DECODE_MAIN 1
#define ZMQG_PROF_ENCODE_CALL 2
#define ZMQG_PROF_DECODE_CALL 3
#define ZMQG_PROF_ENCODE_BODY 4
#define ZMQG_PROF_DECODE_BODY 5
int zmqg_ctx_set_profiling(zmqg_ctx *ctx, int enable);
int zmqg_ctx_get_profile(zmqg_ctx *ctx, int kind, double *ms_total, uint64_t *launches);

/* Text for the last HIP error seen by this ctx (static storage). */
const char *zmqg_last_error(zmqg_ctx *ctx);

/* Build identity, "<source id> <commit>": the first 16 hex digits of the
 * SHA-256 of the library's sources (the .hip and .hpp files of libzmq_amd/csrc and this
 * header, in name order) and the git commit the tree was at when it was
 * built.  Measurement files under profiles/ carry the source id of the
 * library they measured; bench.py folds them into its line only when it
 * equals the loaded library's. */
const char *zmqg_build_id(void);

#ifdef __cplusplus
}
#endif

#endif
