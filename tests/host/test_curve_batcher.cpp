// The asynchronous batched codec (libzmq_amd/host/curve_batcher) against the
// per-message path: many connections on one ctx, interleaved messages of
// mixed sizes and msg_t flags, small slots so batches roll over and submits
// hit back-pressure.  Every encoded frame must equal, byte for byte, what
// curve_encoding_gpu_t::encode (n = 1, the reference's call pattern) gives
// for the same connection and nonce on a second ctx; the inbound stream --
// the frames plus replays, tampered and truncated frames -- must give the
// same status, payload and flags through the batcher as through
// curve_encoding_gpu_t::decode one message at a time.  Also the fence API.
// With a path argument, writes the encode records for the oracle check in
// tests/test_host_adapter.py.  Needs a GPU; prints "OK <n>".
#include "../../libzmq_amd/host/curve_batcher.hpp"

#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <map>
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

static uint64_t rng_state = 0x9e3779b97f4a7c15ull;
static uint64_t rnd ()
{
    rng_state ^= rng_state << 13;
    rng_state ^= rng_state >> 7;
    rng_state ^= rng_state << 17;
    return rng_state;
}

struct result_t
{
    std::vector<uint8_t> bytes;
    int status;
    uint8_t flags;
    bool seen;
    result_t () : status (-1), flags (0), seen (false) {}
};

struct sink_t : zmqg::curve_sink_t
{
    std::map<uint64_t, result_t> got;
    std::vector<uint64_t> order; // delivery order of tags

    void on_encoded (uint64_t tag_, const uint8_t *wire_, size_t size_)
    {
        result_t &r = got[tag_];
        CHECK (!r.seen);
        r.seen = true;
        r.status = 0;
        r.bytes.assign (wire_, wire_ + size_);
        order.push_back (tag_);
    }
    void on_decoded (uint64_t tag_, int status_, const uint8_t *payload_, size_t size_, uint8_t flags_)
    {
        result_t &r = got[tag_];
        CHECK (!r.seen);
        r.seen = true;
        r.status = status_;
        r.flags = flags_;
        if (status_ == 0)
            r.bytes.assign (payload_, payload_ + size_);
        else
            CHECK (payload_ == NULL && size_ == 0);
        order.push_back (tag_);
    }
};

static const int n_conn = 24;
static const uint32_t server_sid0 = 32;

struct side_t
{
    zmqg_ctx *ctx;
    std::vector<zmqg::curve_encoding_gpu_t *> client, server;
};

static void make_side (side_t &s, const uint8_t (*precom)[32], const bool *downgrade)
{
    CHECK (zmqg_ctx_create (0, 64, &s.ctx) == 0);
    for (int c = 0; c < n_conn; ++c) {
        s.client.push_back (new zmqg::curve_encoding_gpu_t (s.ctx, c, client_prefix, server_prefix, downgrade[c]));
        s.server.push_back (
          new zmqg::curve_encoding_gpu_t (s.ctx, server_sid0 + c, server_prefix, client_prefix, false));
        memcpy (s.client[c]->get_writable_precom_buffer (), precom[c], 32);
        memcpy (s.server[c]->get_writable_precom_buffer (), precom[c], 32);
    }
}

static void free_side (side_t &s)
{
    for (int c = 0; c < n_conn; ++c) {
        delete s.client[c];
        delete s.server[c];
    }
    CHECK (zmqg_ctx_destroy (s.ctx) == 0);
}

static void test_fences (zmqg_ctx *ctx)
{
    void *stream = NULL;
    CHECK (zmqg_ctx_stream (ctx, &stream) == 0 && stream != NULL);
    uint64_t f1 = 0, f2 = 0;
    CHECK (zmqg_fence_record (ctx, stream, &f1) == 0);
    CHECK (zmqg_fence_record (ctx, stream, &f2) == 0);
    CHECK (f2 == f1 + 1);
    CHECK (zmqg_fence_wait (ctx, f2) == 0);
    CHECK (zmqg_fence_query (ctx, f2) == 1); // released
    CHECK (zmqg_fence_query (ctx, f1) == 1); // same stream, earlier
    CHECK (zmqg_fence_query (ctx, 0) == -EINVAL);
    CHECK (zmqg_fence_query (ctx, f2 + 1) == -EINVAL);
    void *p = NULL;
    CHECK (zmqg_host_alloc (ctx, 4096, &p) == 0 && p != NULL);
    memset (p, 0xab, 4096);
    CHECK (zmqg_host_free (ctx, p) == 0);
    CHECK (zmqg_host_alloc (ctx, 0, &p) == -EINVAL);
}

int main (int argc, char **argv)
{
    const int n_msgs = 3000;
    uint8_t precom[n_conn][32];
    bool downgrade[n_conn];
    for (int c = 0; c < n_conn; ++c) {
        for (int i = 0; i < 32; ++i)
            precom[c][i] = (uint8_t) rnd ();
        downgrade[c] = c % 5 == 0;
    }
    static const size_t sizes[] = {0, 1, 15, 16, 17, 31, 32, 33, 63, 64, 65, 100, 255, 1024, 1500, 4000, 4500, 9000};
    static const uint8_t flag_set[] = {0, 0, 0, ZMQG_MSG_MORE, ZMQG_MSG_COMMAND, ZMQG_MSG_SUBSCRIBE,
                                       ZMQG_MSG_CANCEL, ZMQG_MSG_MORE | ZMQG_MSG_COMMAND};
    std::vector<int> conn (n_msgs);
    std::vector<uint8_t> mflags (n_msgs);
    std::vector<std::vector<uint8_t> > payload (n_msgs);
    for (int m = 0; m < n_msgs; ++m) {
        conn[m] = (int) (rnd () % n_conn);
        size_t sz = sizes[rnd () % (sizeof sizes / sizeof sizes[0])];
        if (rnd () % 200 == 0)
            sz = 70000 + rnd () % 3000; // larger than the frame kernel's limit
        payload[m].resize (sz);
        for (size_t i = 0; i < sz; ++i)
            payload[m][i] = (uint8_t) rnd ();
        mflags[m] = flag_set[rnd () % (sizeof flag_set / sizeof flag_set[0])];
    }

    side_t a, b; // a: through the batcher; b: one message per call
    make_side (a, precom, downgrade);
    make_side (b, precom, downgrade);
    test_fences (a.ctx);

    // ---- encode ----
    sink_t sink;
    zmqg::curve_batcher_t::config_t cfg;
    cfg.slot_msgs = 256;
    cfg.slot_bytes = 256 << 10;
    cfg.slots = 3;
    zmqg::curve_batcher_t *bp = new zmqg::curve_batcher_t (a.ctx, &sink, cfg);
    zmqg::curve_batcher_t &batcher = *bp;
    CHECK (batcher.init () == 0);
    {   // a message larger than a slot is refused and takes no nonce
        std::vector<uint8_t> big (cfg.slot_bytes + 1);
        const zmqg::curve_encoding_gpu_t::nonce_t before = a.client[0]->get_and_inc_nonce ();
        CHECK (batcher.submit_encode (a.client[0], &big[0], big.size (), 0, 999999) == -1 && errno == EMSGSIZE);
        CHECK (a.client[0]->get_and_inc_nonce () == before + 1);
        zmqg::curve_encoding_gpu_t::nonce_t n = b.client[0]->get_and_inc_nonce ();
        b.client[0]->get_and_inc_nonce (); // keep both sides' nonces in step
        (void) n;
    }
    for (int m = 0; m < n_msgs; ++m) {
        const uint8_t *p = payload[m].empty () ? NULL : &payload[m][0];
        CHECK (batcher.submit_encode (a.client[conn[m]], p, payload[m].size (), mflags[m], (uint64_t) m) == 0);
        if (m % 97 == 96)
            CHECK (batcher.flush () == 0);
        CHECK (batcher.poll () >= 0);
    }
    CHECK (batcher.drain () >= 0);
    CHECK (batcher.queued () == 0 && batcher.in_flight () == 0);
    CHECK ((int) sink.order.size () == n_msgs);
    delete bp;
    for (int m = 1; m < n_msgs; ++m)
        CHECK (sink.order[m] == sink.order[m - 1] + 1); // launch order = submit order

    std::vector<std::vector<uint8_t> > wire (n_msgs);
    for (int m = 0; m < n_msgs; ++m) {
        zmqg::msg_buf_t msg;
        msg.bytes = payload[m];
        msg.flags = mflags[m];
        CHECK (b.client[conn[m]]->encode (&msg) == 0);
        CHECK (sink.got[m].bytes == msg.bytes);
        wire[m] = msg.bytes;
    }

    if (argc > 1) {
        // records for the oracle: precoms, downgrade flags, then per message
        // conn, flags, payload, wire
        FILE *f = fopen (argv[1], "wb");
        CHECK (f != NULL);
        const uint32_t hdr[2] = {(uint32_t) n_conn, (uint32_t) n_msgs};
        CHECK (fwrite (hdr, sizeof hdr, 1, f) == 1);
        CHECK (fwrite (precom, sizeof precom, 1, f) == 1);
        for (int c = 0; c < n_conn; ++c) {
            const uint8_t d = downgrade[c] ? 1 : 0;
            CHECK (fwrite (&d, 1, 1, f) == 1);
        }
        for (int m = 0; m < n_msgs; ++m) {
            const uint32_t rec[4] = {(uint32_t) conn[m], mflags[m], (uint32_t) payload[m].size (),
                                     (uint32_t) wire[m].size ()};
            CHECK (fwrite (rec, sizeof rec, 1, f) == 1);
            if (!payload[m].empty ())
                CHECK (fwrite (&payload[m][0], payload[m].size (), 1, f) == 1);
            CHECK (fwrite (&wire[m][0], wire[m].size (), 1, f) == 1);
        }
        CHECK (fclose (f) == 0);
    }

    // ---- decode: the frames in order plus replays, tampering, truncation ----
    std::vector<int> in_conn;
    std::vector<std::vector<uint8_t> > in_wire;
    std::vector<int> in_src; // message index for untouched first deliveries, else -1
    for (int m = 0; m < n_msgs; ++m) {
        in_conn.push_back (conn[m]);
        in_wire.push_back (wire[m]);
        in_src.push_back (m);
        const uint64_t r = rnd () % 100;
        if (r < 6) { // replay an earlier frame of any connection
            const int j = (int) (rnd () % (uint64_t) (m + 1));
            in_conn.push_back (conn[j]);
            in_wire.push_back (wire[j]);
            in_src.push_back (-1);
        } else if (r < 10) { // a tampered copy of the next frame's bytes
            std::vector<uint8_t> t = wire[m];
            // tag or ciphertext: a raised nonce would (as in the reference,
            // check_validity before the MAC) move the peer nonce past the
            // connection's later genuine frames
            t[16 + rnd () % (t.size () - 16)] ^= (uint8_t) (1u << (rnd () % 8));
            in_conn.push_back (conn[m]);
            in_wire.push_back (t);
            in_src.push_back (-1);
        } else if (r < 12) { // truncated below the MESSAGE minimum
            std::vector<uint8_t> t (wire[m].begin (), wire[m].begin () + (long) (rnd () % 33));
            in_conn.push_back (conn[m]);
            in_wire.push_back (t);
            in_src.push_back (-1);
        }
    }
    const int n_in = (int) in_wire.size ();
    //  twice: with the host applying the header / replay rules
    //  (ZMQG_OPT_REPLAY_HOST, the default) and with the device applying them
    for (int pass = 0; pass < 2; ++pass) {
        zmqg::curve_batcher_t::config_t dcfg = cfg;
        dcfg.replay_host = pass == 0;
        for (int c = 0; c < n_conn; ++c) {
            a.server[c]->set_peer_nonce (0);
            b.server[c]->set_peer_nonce (0);
        }
        sink_t dsink;
        zmqg::curve_batcher_t *dbp = new zmqg::curve_batcher_t (a.ctx, &dsink, dcfg);
        zmqg::curve_batcher_t &dbatcher = *dbp;
        CHECK (dbatcher.init () == 0);
        for (int k = 0; k < n_in; ++k) {
            const uint8_t *p = in_wire[k].empty () ? NULL : &in_wire[k][0];
            CHECK (dbatcher.submit_decode (a.server[in_conn[k]], p, in_wire[k].size (), (uint64_t) k) == 0);
            if (k % 131 == 130)
                CHECK (dbatcher.flush () == 0);
            CHECK (dbatcher.poll () >= 0);
        }
        CHECK (dbatcher.drain () >= 0);
        CHECK ((int) dsink.order.size () == n_in);
        delete dbp;
        int failures = 0;
        for (int k = 0; k < n_in; ++k) {
            zmqg::msg_buf_t msg;
            msg.bytes = in_wire[k];
            int code = 0;
            const int rc = b.server[in_conn[k]]->decode (&msg, &code);
            const result_t &r = dsink.got[k];
            if (rc == 0) {
                CHECK (r.status == 0);
                CHECK (r.bytes == msg.bytes);
                CHECK (r.flags == msg.flags);
            } else {
                CHECK (r.status == code && code != 0);
                ++failures;
            }
            const int cmd_type = in_src[k] >= 0 ? mflags[in_src[k]] & 28 : 0; // msg_t CMD_TYPE_MASK
            if (in_src[k] >= 0 && cmd_type != ZMQG_MSG_SUBSCRIBE && cmd_type != ZMQG_MSG_CANCEL) {
                // plain messages come back as they went in (sub/cancel carry
                // their command name, src/curve_mechanism_base.cpp:143-159)
                const int m = in_src[k];
                CHECK (r.status == 0 && r.bytes == payload[m]);
                CHECK (r.flags == (mflags[m] & (ZMQG_MSG_MORE | ZMQG_MSG_COMMAND)));
            }
        }
        CHECK (failures > 0);
        for (int c = 0; c < n_conn; ++c)
            CHECK (a.server[c]->get_peer_nonce () == b.server[c]->get_peer_nonce ());
        if (pass == 0) {
            //  the host's peer nonces reach the device before a per-message
            //  decode: a replay of each connection's last frame fails there
            //  as it failed in the batch
            for (int k = n_in - 1, done = 0; k >= 0 && done < 4; --k) {
                if (in_src[k] < 0)
                    continue;
                zmqg::msg_buf_t msg;
                msg.bytes = in_wire[k];
                int code = 0;
                CHECK (a.server[in_conn[k]]->decode (&msg, &code) == -1 && code == ZMQG_ERR_INVALID_SEQUENCE);
                ++done;
            }
        }
    }

    {   //  receive slots holding no payload bytes at all (in_used == 0:
        //  empty frames) and frames under the 33-byte MESSAGE minimum: each
        //  frame gets its own status through the verify-first decode
        sink_t esink;
        zmqg::curve_batcher_t eb (a.ctx, &esink, cfg);
        CHECK (eb.init () == 0);
        CHECK (eb.submit_decode (a.server[0], NULL, 0, 1) == 0);
        CHECK (eb.flush () == 0);
        CHECK (eb.drain () >= 0);
        const uint8_t short_frame[20] = {7, 'M', 'E', 'S', 'S', 'A', 'G', 'E'};
        CHECK (eb.submit_decode (a.server[0], NULL, 0, 2) == 0);
        CHECK (eb.submit_decode (a.server[1], short_frame, sizeof short_frame, 3) == 0);
        CHECK (eb.flush () == 0);
        CHECK (eb.drain () >= 0);
        CHECK (esink.order.size () == 3);
        CHECK (esink.got[1].status == ZMQG_ERR_MALFORMED_UNSPECIFIED);
        CHECK (esink.got[2].status == ZMQG_ERR_MALFORMED_UNSPECIFIED);
        CHECK (esink.got[3].status == ZMQG_ERR_MALFORMED_MESSAGE);
    }

    free_side (a);
    free_side (b);
    printf ("OK %d\n", n_msgs + n_in);
    return 0;
}
