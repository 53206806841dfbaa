// Round trips through the C++ curve_encoding_t mirror (libzmq_amd/host),
// modelled on the reference's unittests/unittest_curve_encoding.cpp
// (test_roundtrip_empty / _small / _large / _empty_more), plus the error
// paths of src/curve_mechanism_base.cpp:80-109, 277-281 and the batched
// forms.  Needs a GPU; prints "OK <n>" on success.
#include "../../libzmq_amd/host/curve_encoding_gpu.hpp"

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
static int tests_run = 0;

static void fill_precom (uint8_t *p, uint32_t seed)
{
    uint32_t x = seed * 2654435761u + 1;
    for (int i = 0; i < 32; ++i) {
        x ^= x << 13;
        x ^= x >> 17;
        x ^= x << 5;
        p[i] = (uint8_t) x;
    }
}

// unittest_curve_encoding.cpp test_roundtrip: client encodes, server
// (peer nonce reset to 0) decodes, size and bytes must survive
static void test_roundtrip (zmqg_ctx *ctx, zmqg::msg_buf_t *msg)
{
    const std::vector<uint8_t> original = msg->bytes;
    zmqg::curve_encoding_gpu_t client (ctx, 0, client_prefix, server_prefix, false);
    zmqg::curve_encoding_gpu_t server (ctx, 1, server_prefix, client_prefix, false);
    fill_precom (client.get_writable_precom_buffer (), 11);
    memcpy (server.get_writable_precom_buffer (), client.get_precom_buffer (), 32);
    CHECK (client.encode (msg) == 0);
    CHECK (msg->size () == original.size () + 33);
    server.set_peer_nonce (0);
    int code = 0;
    CHECK (server.decode (msg, &code) == 0);
    CHECK (msg->size () == original.size ());
    CHECK (msg->bytes == original);
    ++tests_run;
}

int main ()
{
    zmqg_ctx *ctx = nullptr;
    CHECK (zmqg_ctx_create (0, 8, &ctx) == 0);

    {   // test_roundtrip_empty
        zmqg::msg_buf_t m;
        test_roundtrip (ctx, &m);
    }
    {   // test_roundtrip_small
        zmqg::msg_buf_t m;
        const char *s = "0123456789ABCDEF0123456789ABCDEF";
        m.bytes.assign (s, s + 32);
        test_roundtrip (ctx, &m);
    }
    {   // test_roundtrip_large
        zmqg::msg_buf_t m;
        const char *s = "0123456789ABCDEF0123456789ABCDEF";
        for (int pos = 0; pos < 2048; pos += 32)
            m.bytes.insert (m.bytes.end (), s, s + 32);
        test_roundtrip (ctx, &m);
    }
    {   // test_roundtrip_empty_more
        zmqg::msg_buf_t m;
        m.flags = zmqg::msg_more;
        test_roundtrip (ctx, &m);
        CHECK (m.flags & zmqg::msg_more);
    }
    {   // known answer (SURVEY.md 8c probe): precom 00..1f, client prefix,
        // first nonce 1, 1 KiB payload i*7+3
        zmqg::curve_encoding_gpu_t client (ctx, 2, client_prefix, server_prefix, false);
        for (int i = 0; i < 32; ++i)
            client.get_writable_precom_buffer ()[i] = (uint8_t) i;
        zmqg::msg_buf_t m;
        for (int i = 0; i < 1024; ++i)
            m.bytes.push_back ((uint8_t) (i * 7 + 3));
        CHECK (client.encode (&m) == 0);
        static const uint8_t want[36] = {
          0x07, 0x4d, 0x45, 0x53, 0x53, 0x41, 0x47, 0x45, 0, 0, 0, 0,
          0,    0,    0,    1,    0x21, 0x1a, 0xc2, 0x5d, 0x7f, 0xfe, 0x52, 0x01,
          0xb4, 0x38, 0x80, 0xd3, 0xfb, 0x29, 0xfb, 0x06, 0x94, 0xb7, 0x29, 0x81};
        CHECK (m.size () == 1024 + 33);
        CHECK (memcmp (m.data (), want, 36) == 0);
        ++tests_run;
    }
    {   // errors: tampered MAC, replay, bad command name, short frame
        zmqg::curve_encoding_gpu_t client (ctx, 3, client_prefix, server_prefix, false);
        zmqg::curve_encoding_gpu_t server (ctx, 4, server_prefix, client_prefix, false);
        fill_precom (client.get_writable_precom_buffer (), 5);
        memcpy (server.get_writable_precom_buffer (), client.get_precom_buffer (), 32);
        zmqg::msg_buf_t a, b;
        a.bytes.assign (100, 0x5a);
        b.bytes.assign (100, 0x33);
        CHECK (client.encode (&a) == 0); // nonce 1
        CHECK (client.encode (&b) == 0); // nonce 2
        zmqg::msg_buf_t bad = b;
        bad.bytes[40] ^= 1;
        int code = 0;
        errno = 0;
        CHECK (server.decode (&bad, &code) == -1);
        CHECK (errno == EPROTO && code == ZMQG_ERR_CRYPTOGRAPHIC);
        // check_validity set the peer nonce to 2 before the MAC failed
        CHECK (server.get_peer_nonce () == 2);
        zmqg::msg_buf_t a2 = a;
        CHECK (server.decode (&a2, &code) == -1 && code == ZMQG_ERR_INVALID_SEQUENCE);
        server.set_peer_nonce (0);
        CHECK (server.decode (&a, &code) == 0);
        CHECK (a.bytes == std::vector<uint8_t> (100, 0x5a));
        zmqg::msg_buf_t wrong = b;
        wrong.bytes[1] = 'm';
        CHECK (server.decode (&wrong, &code) == -1 && code == ZMQG_ERR_UNEXPECTED_COMMAND);
        zmqg::msg_buf_t shrt;
        shrt.bytes.assign (b.bytes.begin (), b.bytes.begin () + 20);
        CHECK (server.decode (&shrt, &code) == -1 && code == ZMQG_ERR_MALFORMED_MESSAGE);
        CHECK (server.decode (&b, &code) == 0);
        CHECK (b.bytes == std::vector<uint8_t> (100, 0x33));
        ++tests_run;
    }
    {   // batched: three connections, interleaved, one submission each way
        std::vector<zmqg::curve_encoding_gpu_t *> cl, sv;
        for (uint32_t c = 0; c < 3; ++c) {
            cl.push_back (new zmqg::curve_encoding_gpu_t (ctx, c, client_prefix, server_prefix, c == 2));
            sv.push_back (new zmqg::curve_encoding_gpu_t (ctx, 4 + c, server_prefix, client_prefix, c == 2));
            fill_precom (cl[c]->get_writable_precom_buffer (), 100 + c);
            memcpy (sv[c]->get_writable_precom_buffer (), cl[c]->get_precom_buffer (), 32);
            // the first MESSAGE nonce here is 1: reset the peer nonce as the
            // reference's unittest does (no handshake advanced it)
            sv[c]->set_peer_nonce (0);
        }
        const int n = 30;
        std::vector<zmqg::msg_buf_t> msgs (n);
        std::vector<std::vector<uint8_t> > orig (n);
        std::vector<zmqg::curve_encoding_gpu_t *> e (n), d (n);
        std::vector<zmqg::msg_buf_t *> mp (n);
        for (int i = 0; i < n; ++i) {
            msgs[i].bytes.assign ((size_t) (i * 97) % 3000, (uint8_t) i);
            msgs[i].flags = (i % 4 == 1) ? zmqg::msg_more : 0;
            orig[i] = msgs[i].bytes;
            e[i] = cl[i % 3];
            d[i] = sv[i % 3];
            mp[i] = &msgs[i];
        }
        CHECK (zmqg::curve_encoding_gpu_t::encode_many (&e[0], &mp[0], n) == 0);
        std::vector<int32_t> status (n, -1);
        CHECK (zmqg::curve_encoding_gpu_t::decode_many (&d[0], &mp[0], n, &status[0]) == 0);
        for (int i = 0; i < n; ++i) {
            CHECK (status[i] == 0);
            CHECK (msgs[i].bytes == orig[i]);
            CHECK ((msgs[i].flags & zmqg::msg_more) == ((i % 4 == 1) ? zmqg::msg_more : 0));
        }
        for (uint32_t c = 0; c < 3; ++c) {
            CHECK (sv[c]->get_peer_nonce () == 10); // nonces 1..10 per connection
            delete cl[c];
            delete sv[c];
        }
        ++tests_run;
    }
    CHECK (zmqg_ctx_destroy (ctx) == 0);
    {
        //  per-I/O-thread ctx and session slots of the drop-in
        //  zmq::curve_encoding_t (zmq_curve_encoding.hpp): a round trip
        //  between two codecs on slots of the thread's ctx, and slot reuse
        zmqg_ctx *tc = zmqg::thread_ctx ();
        CHECK (tc != NULL && zmqg::thread_ctx () == tc);
        uint32_t a = 99, b = 99, c = 99;
        CHECK (zmqg::acquire_session (&a) == 0 && zmqg::acquire_session (&b) == 0 && a != b);
        zmqg::curve_encoding_gpu_t cli (tc, a, client_prefix, server_prefix, false);
        zmqg::curve_encoding_gpu_t srv (tc, b, server_prefix, client_prefix, false);
        fill_precom (cli.get_writable_precom_buffer (), 5);
        fill_precom (srv.get_writable_precom_buffer (), 5);
        zmqg::msg_buf_t m;
        m.bytes.assign (300, 0x5a);
        CHECK (cli.encode (&m) == 0);
        srv.set_peer_nonce (0); // (the handshake leaves it below the first MESSAGE nonce)
        int ev = 0;
        CHECK (srv.decode (&m, &ev) == 0 && m.bytes == std::vector<uint8_t> (300, 0x5a));
        zmqg::release_session (a);
        CHECK (zmqg::acquire_session (&c) == 0 && c == a);
        zmqg::release_session (b);
        zmqg::release_session (c);
        ++tests_run;
    }
    printf ("OK %d\n", tests_run);
    return 0;
}
