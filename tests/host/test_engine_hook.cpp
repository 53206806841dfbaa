// The engine side of the batched codec (libzmq_amd/host/curve_engine_hook)
// driven by loops shaped like the reference's stream engine and I/O thread
// (SURVEY.md section 8f row 1):
//   * client engines (I/O thread A) run out_event as
//     src/stream_engine_base.cpp:331-348 does: pull messages from the
//     session up to out_batch_size bytes per event (pull_and_encode's place:
//     submit_send), and frame every encoded MESSAGE command that is ready,
//     in order, into the socket's send buffer with the ZMTP 3.1 encoder's
//     framing (src/v3_1_encoder.cpp:23-60: flags 0 or LARGE, 1- or 8-byte
//     size);
//   * the bytes cross an in-memory "socket" in random-sized pieces;
//   * server engines (I/O thread B) run in_event_internal as :281-291 does:
//     a ZMTP frame parser (src/v2_decoder.cpp:35-140) completes frames from
//     whatever bytes arrived, each MESSAGE body goes to submit_received
//     (decode_and_push's place), decoded messages are pushed to the session;
//   * each I/O thread's poller iteration calls its hook's iteration().
// 16 connections x 300 messages of mixed sizes and msg_t flags (plain, MORE,
// SUBSCRIBE, CANCEL), small batcher slots (roll-over and back-pressure).
// Checked: every server session receives exactly its client's messages, in
// order, as the reference codec would deliver them (subscriptions as
// "\x09SUBSCRIBE"/"\x06CANCEL" command bodies with the COMMAND flag,
// src/curve_mechanism_base.cpp:118-164); connection 3 gets one ciphertext
// byte flipped in its 51st message: its engine fails with
// ZMQ_PROTOCOL_ERROR_ZMTP_CRYPTOGRAPHIC after delivering the 50 before it,
// and every other connection completes.  Needs a GPU; prints "OK <n>".
#include "../../libzmq_amd/host/curve_engine_hook.hpp"

#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#define CHECK(c)                                                              \
    do {                                                                      \
        if (!(c)) {                                                           \
            fprintf (stderr, "%s:%d: check failed: %s\n", __FILE__, __LINE__, \
                     #c);                                                     \
            exit (1);                                                         \
        }                                                                     \
    } while (0)

static const char client_prefix[] = "CurveZMQMESSAGEC";
static const char server_prefix[] = "CurveZMQMESSAGES";
static const int n_conn = 16;
static const int n_msgs = 300;
static const int bad_conn = 3, bad_msg = 50;

static uint64_t rng_state = 0x2545f4914f6cdd1dull;
static uint64_t rnd ()
{
    rng_state ^= rng_state << 13;
    rng_state ^= rng_state >> 7;
    rng_state ^= rng_state << 17;
    return rng_state;
}

struct client_t
{
    zmqg::curve_encoding_gpu_t *codec;
    zmqg::curve_engine_link_t *link;
    std::vector<zmqg::msg_buf_t> session; //  what the session will hand over
    size_t pulled;                        //  session messages pulled so far
    size_t framed;                        //  encoded messages framed so far
    std::vector<uint8_t> out;             //  the socket's send buffer
};

struct server_t
{
    zmqg::curve_encoding_gpu_t *codec;
    zmqg::curve_engine_link_t *link;
    std::vector<uint8_t> in; //  received, not yet parsed
    std::vector<zmqg::msg_buf_t> session;
};

//  the v3.1 encoder's framing of one body (a CURVE MESSAGE has no MORE or
//  COMMAND bit on the ZMTP frame, src/curve_mechanism_base.cpp:166-177)
static void zmtp_frame (std::vector<uint8_t> &out_, const std::vector<uint8_t> &body_)
{
    const uint64_t n = body_.size ();
    if (n > 255) {
        out_.push_back (2); //  LARGE
        for (int i = 7; i >= 0; --i)
            out_.push_back ((uint8_t) (n >> (8 * i)));
    } else {
        out_.push_back (0);
        out_.push_back ((uint8_t) n);
    }
    out_.insert (out_.end (), body_.begin (), body_.end ());
}

//  out_event: pull up to out_batch_size bytes, frame what is encoded
static void out_event (client_t &c_, int conn_)
{
    const size_t out_batch_size = 8192; //  src/options.cpp:222
    size_t bytes = 0;
    while (c_.pulled < c_.session.size () && bytes < out_batch_size) {
        const zmqg::msg_buf_t &m = c_.session[c_.pulled];
        CHECK (c_.link->submit_send (m.bytes.empty () ? NULL : &m.bytes[0],
                                     m.bytes.size (), m.flags)
               == 0);
        bytes += m.bytes.size () + 1;
        ++c_.pulled;
    }
    std::vector<uint8_t> w;
    while (c_.link->next_encoded (w)) {
        if (conn_ == bad_conn && c_.framed == (size_t) bad_msg)
            w[w.size () - 1] ^= 0x10; //  the last ciphertext byte, in transit
        zmtp_frame (c_.out, w);
        ++c_.framed;
    }
}

//  in_event: parse complete frames, hand MESSAGE bodies to the codec, push
//  decoded messages to the session
static void in_event (server_t &s_)
{
    size_t pos = 0;
    while (!s_.link->failed ()) {
        if (s_.in.size () - pos < 2)
            break;
        const uint8_t fl = s_.in[pos];
        size_t hdr = 2;
        uint64_t n = s_.in[pos + 1];
        if (fl & 2) {
            hdr = 9;
            if (s_.in.size () - pos < 9)
                break;
            n = 0;
            for (int i = 0; i < 8; ++i)
                n = (n << 8) | s_.in[pos + 1 + i];
        }
        if (s_.in.size () - pos - hdr < n)
            break; //  incomplete: wait for more bytes
        CHECK (s_.link->submit_received (n ? &s_.in[pos + hdr] : NULL, (size_t) n) == 0);
        pos += hdr + (size_t) n;
    }
    s_.in.erase (s_.in.begin (), s_.in.begin () + (long) pos);
    zmqg::msg_buf_t m;
    while (s_.link->next_decoded (m))
        s_.session.push_back (m);
}

int main ()
{
    zmqg_ctx *ctx_a = NULL, *ctx_b = NULL;
    CHECK (zmqg_ctx_create (0, n_conn, &ctx_a) == 0);
    CHECK (zmqg_ctx_create (0, n_conn, &ctx_b) == 0);
    zmqg::curve_batcher_t::config_t cfg;
    cfg.slot_msgs = 64;
    cfg.slot_bytes = 64 << 10;
    cfg.slots = 3;
    zmqg::curve_io_hook_t hook_a (ctx_a, cfg), hook_b (ctx_b, cfg);
    CHECK (hook_a.init () == 0 && hook_b.init () == 0);

    static const size_t sizes[] = {0, 1, 31, 32, 33, 100, 255, 256, 1000, 4000, 5000, 20000};
    static const uint8_t flag_set[] = {0, 0, 0, zmqg::msg_more, zmqg::msg_subscribe, zmqg::msg_cancel};
    std::vector<client_t> cl (n_conn);
    std::vector<server_t> sv (n_conn);
    for (int c = 0; c < n_conn; ++c) {
        cl[c].codec = new zmqg::curve_encoding_gpu_t (ctx_a, c, client_prefix, server_prefix, false);
        sv[c].codec = new zmqg::curve_encoding_gpu_t (ctx_b, c, server_prefix, client_prefix, false);
        for (int i = 0; i < 32; ++i)
            cl[c].codec->get_writable_precom_buffer ()[i] =
              sv[c].codec->get_writable_precom_buffer ()[i] = (uint8_t) rnd ();
        //  the handshake's nonces (HELLO 1, INITIATE 2; the server saw INITIATE's)
        cl[c].codec->get_and_inc_nonce ();
        cl[c].codec->get_and_inc_nonce ();
        sv[c].codec->set_peer_nonce (2);
        cl[c].link = new zmqg::curve_engine_link_t (&hook_a, cl[c].codec);
        sv[c].link = new zmqg::curve_engine_link_t (&hook_b, sv[c].codec);
        cl[c].pulled = cl[c].framed = 0;
        for (int m = 0; m < n_msgs; ++m) {
            zmqg::msg_buf_t msg;
            msg.bytes.resize (sizes[rnd () % (sizeof sizes / sizeof sizes[0])]);
            for (size_t k = 0; k < msg.bytes.size (); ++k)
                msg.bytes[k] = (uint8_t) rnd ();
            msg.flags = flag_set[rnd () % (sizeof flag_set / sizeof flag_set[0])];
            cl[c].session.push_back (msg);
        }
    }

    //  the two I/O threads' poller loops, interleaved
    int iterations = 0;
    for (;; ++iterations) {
        CHECK (iterations < 200000);
        bool done = true;
        for (int c = 0; c < n_conn; ++c) {
            out_event (cl[c], c);
            //  the socket: a random-sized piece of what is queued
            const size_t piece = 1 + rnd () % 6000;
            const size_t k = cl[c].out.size () < piece ? cl[c].out.size () : piece;
            if (!sv[c].link->failed ())
                sv[c].in.insert (sv[c].in.end (), cl[c].out.begin (), cl[c].out.begin () + (long) k);
            cl[c].out.erase (cl[c].out.begin (), cl[c].out.begin () + (long) k);
            in_event (sv[c]);
            const bool finished = sv[c].link->failed ()
                                    ? sv[c].link->receives_in_flight () == 0
                                    : sv[c].session.size () == (size_t) n_msgs;
            done = done && finished;
        }
        CHECK (hook_a.iteration () >= 0);
        CHECK (hook_b.iteration () >= 0);
        if (done)
            break;
    }

    for (int c = 0; c < n_conn; ++c) {
        const size_t expect = c == bad_conn ? (size_t) bad_msg : (size_t) n_msgs;
        CHECK (sv[c].session.size () == expect);
        CHECK (sv[c].link->failed () == (c == bad_conn ? ZMQG_ERR_CRYPTOGRAPHIC : 0));
        for (size_t m = 0; m < expect; ++m) {
            const zmqg::msg_buf_t &sent = cl[c].session[m], &got = sv[c].session[m];
            const int ct = sent.flags & 0x1c;
            std::vector<uint8_t> body;
            uint8_t flags = sent.flags & (zmqg::msg_more | zmqg::msg_command);
            if (ct == zmqg::msg_subscribe || ct == zmqg::msg_cancel) {
                //  ZMTP 3.1 command bodies (src/curve_mechanism_base.cpp:143-159)
                const char *name = ct == zmqg::msg_subscribe ? "\x09" "SUBSCRIBE" : "\x06" "CANCEL";
                body.assign (name, name + strlen (name));
                flags |= zmqg::msg_command;
            }
            body.insert (body.end (), sent.bytes.begin (), sent.bytes.end ());
            CHECK (got.bytes == body);
            CHECK (got.flags == flags);
        }
    }
    CHECK (hook_a.drain () >= 0 && hook_b.drain () >= 0);
    for (int c = 0; c < n_conn; ++c) {
        delete cl[c].link;
        delete sv[c].link;
        delete cl[c].codec;
        delete sv[c].codec;
    }
    CHECK (zmqg_ctx_destroy (ctx_a) == 0 && zmqg_ctx_destroy (ctx_b) == 0);
    printf ("OK %d\n", n_conn * n_msgs);
    return 0;
}
