// The drop-in zmq::curve_encoding_t (libzmq_amd/host/zmq_curve_encoding.hpp)
// run on zmq::msg_t objects, with the four round trips of the reference's
// unittests/unittest_curve_encoding.cpp:26-130 (empty, 32 B, 2048 B,
// empty + MORE) -- each side's precom from its own key pair by
// crypto_box_beforenm, here zmqg_box_beforenm_batch -- plus the msg_t
// buffer-management cases the binding must get right:
//   * the VSM / LMSG split of init_size (src/msg.cpp:62-94, max_vsm_size 33,
//     src/msg.hpp:154-156): payloads of 0, 1, 32, 33, 34, 35 and 2048 bytes,
//     i.e. boxes and decoded payloads on both sides of the split;
//   * move (src/msg.cpp:305-324): encode replaces the message with a fresh
//     one without flags;
//   * shrink (src/msg.cpp:404-425): decode leaves the payload in the same
//     msg_t, shrunk;
//   * set_flags ORs (src/msg.cpp:433-436): flags already on the received
//     msg_t survive, the plaintext MORE / COMMAND bits are added;
//   * a connection that gets no session slot (ZMQG_THREAD_SESSIONS = 4, the
//     fifth codec) fails its calls without aborting the process.
//   * (ZMQG_REAL_MSG_T builds only) zero-copy receive: decode in place on a
//     zclmsg over a shared receive buffer, as src/v2_decoder.cpp:88-113
//     builds it (msg_t::init with an external content_t,
//     src/msg.cpp:30-47, 108-129).
// Two builds: tests/host/build_ref_binding.sh links the REFERENCE's own
// msg_t (src/msg.cpp, metadata.cpp, err.cpp under /root/reference, with
// -DZMQG_REAL_MSG_T; prints "OK 15"); tests/test_host_adapter.py also builds
// it on the test double in tests/host/msg_model/ (prints "OK 14"), which
// needs no reference sources.  Needs a GPU.
#if defined ZMQG_REAL_MSG_T
//  as every reference translation unit starts (platform.hpp, zmq.h,
//  zmq_draft.h), before src/curve_mechanism_base.hpp would include the codec
#include "precompiled.hpp"
#endif
#include "zmq_curve_encoding.hpp"

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

static int tests_run = 0;

#if defined ZMQG_REAL_MSG_T
//  the receive buffer's free function (shared_message_memory_allocator::
//  call_dec_ref in the reference): counts its calls
static void zc_free (void *, void *hint_)
{
    ++*static_cast<int *> (hint_);
}
#endif
static uint32_t key_seed = 1;

static void fill (uint8_t *p, size_t n)
{
    uint32_t x = key_seed++ * 2654435761u + 7;
    for (size_t i = 0; i < n; ++i) {
        x ^= x << 13;
        x ^= x >> 17;
        x ^= x << 5;
        p[i] = (uint8_t) x;
    }
}

//  crypto_box_keypair for both sides, then crypto_box_beforenm on each side
//  (unittest_curve_encoding.cpp:40-55), on the device
static void make_precoms (uint8_t *client_precom_, uint8_t *server_precom_)
{
    zmqg_ctx *ctx = zmqg::thread_ctx ();
    CHECK (ctx != NULL);
    uint8_t *h = NULL;
    CHECK (zmqg_host_alloc (ctx, 512, (void **) &h) == 0);
    uint8_t *sec = h, *pub = h + 64, *pk = h + 128, *sk = h + 192, *k = h + 256;
    int32_t *st = (int32_t *) (h + 384);
    fill (sec, 64); //  client secret, server secret
    void *stream = NULL;
    CHECK (zmqg_ctx_stream (ctx, &stream) == 0);
    CHECK (zmqg_scalarmult_batch (ctx, 2, sec, NULL, pub, st, stream) == 0);
    uint64_t f = 0;
    CHECK (zmqg_fence_record (ctx, stream, &f) == 0);
    CHECK (zmqg_fence_wait (ctx, f) == 0);
    //  client: (server public, client secret); server: (client public, server secret)
    memcpy (pk, pub + 32, 32);
    memcpy (sk, sec, 32);
    memcpy (pk + 32, pub, 32);
    memcpy (sk + 32, sec + 32, 32);
    CHECK (zmqg_box_beforenm_batch (ctx, 2, pk, sk, k, st, stream) == 0);
    CHECK (zmqg_fence_record (ctx, stream, &f) == 0);
    CHECK (zmqg_fence_wait (ctx, f) == 0);
    CHECK (st[0] == 0 && st[1] == 0);
    CHECK (memcmp (k, k + 32, 32) == 0); //  both sides derive the same key
    memcpy (client_precom_, k, 32);
    memcpy (server_precom_, k + 32, 32);
    CHECK (zmqg_host_free (ctx, h) == 0);
}

//  unittest_curve_encoding.cpp:26-71, plus msg_t state checks
static void test_roundtrip (zmq::msg_t *msg_, unsigned char received_flags_)
{
    const std::vector<uint8_t> original (
      static_cast<uint8_t *> (msg_->data ()),
      static_cast<uint8_t *> (msg_->data ()) + msg_->size ());
    const unsigned char sent_flags = msg_->flags ();

    zmq::curve_encoding_t encoding_client ("CurveZMQMESSAGEC",
                                           "CurveZMQMESSAGES", false);
    zmq::curve_encoding_t encoding_server ("CurveZMQMESSAGES",
                                           "CurveZMQMESSAGEC", false);
    make_precoms (encoding_client.get_writable_precom_buffer (),
                  encoding_server.get_writable_precom_buffer ());

    CHECK (encoding_client.encode (msg_) == 0);
    //  msg_->move (msg_box): a fresh message of the box's size, no flags
    CHECK (msg_->size () == original.size () + 33);
    CHECK (msg_->is_vsm () == (msg_->size () <= zmq::msg_t::max_vsm_size));
    CHECK (msg_->flags () == 0);
    CHECK (memcmp (msg_->data (), "\x07MESSAGE", 8) == 0);

    //  the engine's receive side may carry flags of its own on the msg_t
    msg_->set_flags (received_flags_);
    const bool was_vsm = msg_->is_vsm ();
    const void *was_data = msg_->data ();

    encoding_server.set_peer_nonce (0);
    int error_event_code = 0;
    CHECK (encoding_server.decode (msg_, &error_event_code) == 0);

    //  decoded in the same msg_t (memmove + shrink, no new buffer)
    CHECK (msg_->is_vsm () == was_vsm && msg_->data () == was_data);
    CHECK (msg_->size () == original.size ());
    if (!original.empty ())
        CHECK (memcmp (&original[0], msg_->data (), original.size ()) == 0);
    //  set_flags ORs: what was there, plus the plaintext MORE / COMMAND bits
    CHECK (msg_->flags ()
           == (received_flags_
               | (sent_flags & (zmq::msg_t::more | zmq::msg_t::command))));
    ++tests_run;
}

int main ()
{
    {   //  test_roundtrip_empty
        zmq::msg_t msg;
        msg.init ();
        test_roundtrip (&msg, 0);
        msg.close ();
    }
    {   //  test_roundtrip_small
        zmq::msg_t msg;
        msg.init_size (32);
        memcpy (msg.data (), "0123456789ABCDEF0123456789ABCDEF", 32);
        test_roundtrip (&msg, 0);
        msg.close ();
    }
    {   //  test_roundtrip_large
        zmq::msg_t msg;
        msg.init_size (2048);
        for (size_t pos = 0; pos < 2048; pos += 32)
            memcpy (static_cast<char *> (msg.data ()) + pos,
                    "0123456789ABCDEF0123456789ABCDEF", 32);
        test_roundtrip (&msg, 0);
        msg.close ();
    }
    {   //  test_roundtrip_empty_more
        zmq::msg_t msg;
        msg.init ();
        msg.set_flags (zmq::msg_t::more);
        test_roundtrip (&msg, 0);
        CHECK (msg.flags () & zmq::msg_t::more);
        msg.close ();
    }
    //  the VSM / LMSG boundary on both sides (payload P: box P + 33)
    const size_t sizes[] = {0, 1, 32, 33, 34, 35, 2048};
    for (size_t k = 0; k < sizeof sizes / sizeof sizes[0]; ++k) {
        zmq::msg_t msg;
        msg.init_size (sizes[k]);
        CHECK (msg.is_vsm () == (sizes[k] <= 33));
        fill (static_cast<uint8_t *> (msg.data ()), sizes[k]);
        msg.set_flags (k % 2 ? zmq::msg_t::more : 0);
        //  a received frame flagged as a command keeps that bit
        test_roundtrip (&msg, k == 3 ? zmq::msg_t::command : 0);
        msg.close ();
    }
    {   //  subscribe: the ZMTP 3.1 command body travels in the box
        //  (src/curve_mechanism_base.cpp:118-164) and comes back as a
        //  COMMAND-flagged payload "\x09SUBSCRIBE" + topic
        zmq::curve_encoding_t cli ("CurveZMQMESSAGEC", "CurveZMQMESSAGES",
                                   false);
        zmq::curve_encoding_t srv ("CurveZMQMESSAGES", "CurveZMQMESSAGEC",
                                   false);
        make_precoms (cli.get_writable_precom_buffer (),
                      srv.get_writable_precom_buffer ());
        zmq::msg_t msg;
        msg.init_size (5);
        memcpy (msg.data (), "topic", 5);
        msg.set_flags (zmq::msg_t::subscribe);
        CHECK (cli.encode (&msg) == 0);
        CHECK (msg.size () == 5 + 10 + 33 && msg.flags () == 0);
        srv.set_peer_nonce (0);
        int ev = 0;
        CHECK (srv.decode (&msg, &ev) == 0);
        CHECK (msg.size () == 15
               && memcmp (msg.data (), "\x09SUBSCRIBEtopic", 15) == 0);
        CHECK (msg.flags () == zmq::msg_t::command);
        ++tests_run;
    }
    {   //  a tampered box: -1, EPROTO, CRYPTOGRAPHIC, the msg_t untouched
        zmq::curve_encoding_t cli ("CurveZMQMESSAGEC", "CurveZMQMESSAGES",
                                   false);
        zmq::curve_encoding_t srv ("CurveZMQMESSAGES", "CurveZMQMESSAGEC",
                                   false);
        make_precoms (cli.get_writable_precom_buffer (),
                      srv.get_writable_precom_buffer ());
        zmq::msg_t msg;
        msg.init_size (100);
        memset (msg.data (), 0x42, 100);
        CHECK (cli.encode (&msg) == 0);
        static_cast<uint8_t *> (msg.data ())[60] ^= 1;
        std::vector<uint8_t> wire (static_cast<uint8_t *> (msg.data ()),
                                   static_cast<uint8_t *> (msg.data ())
                                     + msg.size ());
        srv.set_peer_nonce (0);
        int ev = 0;
        errno = 0;
        CHECK (srv.decode (&msg, &ev) == -1);
        CHECK (errno == EPROTO && ev == ZMQG_ERR_CRYPTOGRAPHIC);
        CHECK (msg.size () == wire.size ()
               && memcmp (msg.data (), &wire[0], wire.size ()) == 0);
        ++tests_run;
    }
    {   //  session slots: this thread's ctx was made with
        //  ZMQG_THREAD_SESSIONS = 4 slots (set by the runner); the codecs
        //  above gave theirs back, so four fit and the fifth has none
        zmq::curve_encoding_t *c[5];
        for (int i = 0; i < 5; ++i)
            c[i] = new zmq::curve_encoding_t ("CurveZMQMESSAGEC",
                                              "CurveZMQMESSAGES", false);
        zmq::msg_t msg;
        msg.init_size (10);
        memset (msg.data (), 1, 10);
        errno = 0;
        CHECK (c[4]->encode (&msg) == -1 && errno == EPROTO);
        CHECK (msg.size () == 10); //  left as it was
        int ev = 0;
        CHECK (c[4]->decode (&msg, &ev) == -1 && errno == EPROTO
               && ev == ZMQG_ERR_CRYPTOGRAPHIC);
        CHECK (c[3]->encode (&msg) == 0 && msg.size () == 43);
        delete c[4];
        delete c[0];
        //  a slot given back is taken by the next connection
        zmq::curve_encoding_t again ("CurveZMQMESSAGEC", "CurveZMQMESSAGES",
                                     false);
        zmq::msg_t m2;
        m2.init_size (3);
        CHECK (again.encode (&m2) == 0);
        for (int i = 1; i < 4; ++i)
            delete c[i];
        ++tests_run;
    }
#if defined ZMQG_REAL_MSG_T
    {   //  zero-copy receive (src/v2_decoder.cpp:88-113): each received
        //  frame is a zclmsg whose data is the frame's place in the shared
        //  receive buffer; decode leaves the payload there (no copy, no new
        //  allocation, src/curve_mechanism_base.cpp:253-260) and the
        //  buffer's free function runs once when the message closes
        zmq::curve_encoding_t cli ("CurveZMQMESSAGEC", "CurveZMQMESSAGES",
                                   false);
        zmq::curve_encoding_t srv ("CurveZMQMESSAGES", "CurveZMQMESSAGEC",
                                   false);
        make_precoms (cli.get_writable_precom_buffer (),
                      srv.get_writable_precom_buffer ());
        const size_t P[3] = {200, 1, 3000}; //  boxes of 233, 34, 3033 bytes
        std::vector<uint8_t> rx, expect[3];
        size_t off[3], wlen[3];
        for (int k = 0; k < 3; ++k) {
            zmq::msg_t m;
            CHECK (m.init_size (P[k]) == 0);
            fill (static_cast<uint8_t *> (m.data ()), P[k]);
            expect[k].assign (static_cast<uint8_t *> (m.data ()),
                              static_cast<uint8_t *> (m.data ()) + P[k]);
            m.set_flags (k == 1 ? zmq::msg_t::more : 0);
            CHECK (cli.encode (&m) == 0);
            off[k] = rx.size ();
            wlen[k] = m.size ();
            rx.insert (rx.end (), static_cast<uint8_t *> (m.data ()),
                       static_cast<uint8_t *> (m.data ()) + m.size ());
            CHECK (m.close () == 0);
        }
        srv.set_peer_nonce (0);
        for (int k = 0; k < 3; ++k) {
            zmq::msg_t::content_t content;
            int frees = 0;
            zmq::msg_t m;
            CHECK (m.init (&rx[off[k]], wlen[k], zc_free, &frees, &content)
                   == 0);
            CHECK (m.is_zcmsg () && m.data () == &rx[off[k]]);
            int ev = 0;
            CHECK (srv.decode (&m, &ev) == 0);
            CHECK (m.is_zcmsg () && m.data () == &rx[off[k]]);
            CHECK (m.size () == P[k]);
            CHECK (memcmp (&rx[off[k]], &expect[k][0], P[k]) == 0);
            CHECK (m.flags () == (k == 1 ? zmq::msg_t::more : 0));
            CHECK (m.close () == 0 && frees == 1);
        }
        ++tests_run;
    }
#endif
    printf ("OK %d\n", tests_run);
    return 0;
}
