// The engine side of the batched codec (libzmq_amd/host/curve_engine_hook)
// driven the way libzmq drives its engines:
// two I/O threads, each sleeping in epoll_wait with no timeout
// (src/epoll.cpp:140-179), connected by real non-blocking stream sockets
// (socketpair), each with its own device ctx and curve_io_hook_t whose
// eventfd the poller watches like the mailbox (src/io_thread.cpp:54).
//   * client engines (thread A) run out_event as
//     src/stream_engine_base.cpp:314-354 does: when the output buffer is
//     empty they take every encoded MESSAGE command that is ready (the
//     encoder's load_msg), frame it with the ZMTP 3.1 encoder's framing
//     (src/v3_1_encoder.cpp:23-60: flags 0 or LARGE, 1- or 8-byte size) and
//     pull new messages from the session up to out_batch_size bytes
//     (pull_and_encode's place: submit_send); with nothing to write they
//     reset POLLOUT (:350-353) and sleep until the hook calls encoded_ready
//     = restart_output (:383-390: set_pollout, out_event);
//   * server engines (thread B) run in_event as :255-291 does: read what the
//     socket holds, complete ZMTP frames (src/v2_decoder.cpp:35-140) and hand
//     every MESSAGE body to submit_received (decode_and_push's place);
//     decoded messages reach the session when the hook calls decoded_ready
//     = restart_input (:400-442); a failure is the engine's
//     error (protocol_error): the connection is closed;
//   * the only wake-ups are the sockets and the hooks' eventfds (written by
//     the batches' completion fences); queued messages are launched by the
//     hook's zero-delay timer before the poller blocks (execute_timers).
// 16 connections x 300 messages of mixed sizes and msg_t flags (plain, MORE,
// SUBSCRIBE, CANCEL), small batcher slots (roll-over and back-pressure).
// Checked: every server session receives exactly its client's messages, in
// order, as the reference codec would deliver them (subscriptions as
// "\x09SUBSCRIBE"/"\x06CANCEL" command bodies with the COMMAND flag,
// src/curve_mechanism_base.cpp:118-164); connection 3 gets one ciphertext
// byte flipped in its 51st message: its engine fails with
// ZMQ_PROTOCOL_ERROR_ZMTP_CRYPTOGRAPHIC after delivering the 50 before it,
// and every other connection completes.  The whole exchange must finish
// within a wall-clock bound (a watchdog ends the process otherwise).
// Also: a link closed while its messages are in flight, with a new link
// opened at once (results are routed by link id).  Needs a GPU; prints
// "OK <n> ...".
#include "../../libzmq_amd/host/curve_engine_hook.hpp"

#include <errno.h>
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <thread>
#include <vector>

#define CHECK(c)                                                              \
    do {                                                                      \
        if (!(c)) {                                                           \
            fprintf (stderr, "%s:%d: check failed: %s\n", __FILE__, __LINE__, \
                     #c);                                                     \
            _exit (1);                                                        \
        }                                                                     \
    } while (0)

static const char client_prefix[] = "CurveZMQMESSAGEC";
static const char server_prefix[] = "CurveZMQMESSAGES";
static int n_conn = 16;
static int n_msgs = 300;
static int bad_conn = 3, bad_msg = 50;
//  "bench <connections> <messages> <size>": the same engines and threads as a
//  throughput run -- fixed-size plain messages, no tampering, the batcher's
//  default slots -- printing "RATE ..." 
static bool bench_mode = false;
static size_t bench_size = 1024;
static const int watchdog_s = 60;

static uint64_t rng_state = 0x2545f4914f6cdd1dull;
static uint64_t rnd ()
{
    rng_state ^= rng_state << 13;
    rng_state ^= rng_state >> 7;
    rng_state ^= rng_state << 17;
    return rng_state;
}

static double now_s ()
{
    timespec t;
    clock_gettime (CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}

//  An I/O thread: epoll set, device ctx, hook.  Handlers by fd.
struct io_thread_t;
struct handler_t
{
    virtual ~handler_t () {}
    virtual void in_event () = 0;
    virtual void out_event () = 0;
};

struct io_thread_t
{
    int ep;
    zmqg_ctx *ctx;
    zmqg::curve_io_hook_t *hook;
    std::vector<handler_t *> by_fd;
    long waits, hook_wakes;

    explicit io_thread_t (const zmqg::curve_batcher_t::config_t &cfg_) :
        ep (epoll_create1 (EPOLL_CLOEXEC)), ctx (NULL), hook (NULL), waits (0), hook_wakes (0)
    {
        CHECK (ep >= 0);
        CHECK (zmqg_ctx_create (0, n_conn * 2, &ctx) == 0);
        hook = new zmqg::curve_io_hook_t (ctx, cfg_);
        CHECK (hook->init () == 0);
        //  the hook's eventfd, like the mailbox: add_fd + set_pollin
        epoll_event e;
        memset (&e, 0, sizeof e);
        e.events = EPOLLIN;
        e.data.fd = hook->get_fd ();
        CHECK (epoll_ctl (ep, EPOLL_CTL_ADD, e.data.fd, &e) == 0);
    }
    void add_fd (int fd_, handler_t *h_, uint32_t events_)
    {
        if ((size_t) fd_ >= by_fd.size ())
            by_fd.resize (fd_ + 1, NULL);
        by_fd[fd_] = h_;
        epoll_event e;
        memset (&e, 0, sizeof e);
        e.events = events_;
        e.data.fd = fd_;
        CHECK (epoll_ctl (ep, EPOLL_CTL_ADD, fd_, &e) == 0);
    }
    void set_events (int fd_, uint32_t events_)
    {
        epoll_event e;
        memset (&e, 0, sizeof e);
        e.events = events_;
        e.data.fd = fd_;
        CHECK (epoll_ctl (ep, EPOLL_CTL_MOD, fd_, &e) == 0);
    }
    void rm_fd (int fd_)
    {
        CHECK (epoll_ctl (ep, EPOLL_CTL_DEL, fd_, NULL) == 0);
        by_fd[fd_] = NULL;
    }
    //  src/epoll.cpp:140-179: timers, then block with no timeout
    template <class Done> void loop (Done done_)
    {
        epoll_event ev[64];
        while (!done_ ()) {
            //  execute_timers: the hook's zero-delay flush
            while (hook->flush_pending ())
                CHECK (hook->timer_event () == 0);
            if (done_ ())
                break;
            const int n = epoll_wait (ep, ev, 64, -1);
            ++waits;
            if (n < 0 && errno == EINTR)
                continue;
            CHECK (n > 0); //  no timeout was given: never 0
            for (int i = 0; i < n; ++i) {
                const int fd = ev[i].data.fd;
                if (fd == hook->get_fd ()) {
                    ++hook_wakes;
                    CHECK (hook->in_event () >= 0);
                    continue;
                }
                handler_t *h = (size_t) fd < by_fd.size () ? by_fd[fd] : NULL;
                if (h && (ev[i].events & (EPOLLIN | EPOLLERR | EPOLLHUP)))
                    h->in_event ();
                h = (size_t) fd < by_fd.size () ? by_fd[fd] : NULL; //  (may have closed)
                if (h && (ev[i].events & (EPOLLOUT | EPOLLERR | EPOLLHUP)))
                    h->out_event ();
            }
        }
    }
};

struct client_t : handler_t, zmqg::curve_link_events_t
{
    io_thread_t *io;
    int fd, conn;
    zmqg::curve_encoding_gpu_t *codec;
    zmqg::curve_engine_link_t *link;
    std::vector<zmqg::msg_buf_t> session; //  what the session will hand over
    size_t pulled, framed;
    std::vector<uint8_t> out; //  the encoder's output buffer
    size_t out_pos;
    bool pollout, dead;

    void set_pollout (bool on_)
    {
        if (pollout != on_)
            io->set_events (fd, on_ ? EPOLLOUT : 0);
        pollout = on_;
    }
    void error ()
    {
        io->rm_fd (fd);
        close (fd);
        dead = true;
    }
    bool finished () const
    {
        return dead
               || (pulled == session.size () && framed == session.size ()
                   && out_pos == out.size ());
    }
    //  src/stream_engine_base.cpp:314-354
    void out_event ()
    {
        if (dead)
            return;
        if (out_pos == out.size ()) {
            out.clear ();
            out_pos = 0;
            std::vector<uint8_t> w;
            while (link->next_encoded (w)) {
                if (conn == bad_conn && framed == (size_t) bad_msg)
                    w[w.size () - 1] ^= 0x10; //  the last ciphertext byte, in transit
                const uint64_t n = w.size ();
                if (n > 255) {
                    out.push_back (2); //  LARGE
                    for (int i = 7; i >= 0; --i)
                        out.push_back ((uint8_t) (n >> (8 * i)));
                } else {
                    out.push_back (0);
                    out.push_back ((uint8_t) n);
                }
                out.insert (out.end (), w.begin (), w.end ());
                ++framed;
            }
            const size_t out_batch_size = 8192; //  src/options.cpp:222
            size_t bytes = 0;
            while (pulled < session.size () && bytes < out_batch_size) {
                const zmqg::msg_buf_t &m = session[pulled];
                CHECK (link->submit_send (m.bytes.empty () ? NULL : &m.bytes[0],
                                          m.bytes.size (), m.flags)
                       == 0);
                bytes += m.bytes.size () + 1;
                ++pulled;
            }
            if (out.empty ()) {
                set_pollout (false); //  nothing to write: sleep until restart_output
                return;
            }
        }
        const ssize_t n = send (fd, &out[out_pos], out.size () - out_pos,
                                MSG_NOSIGNAL | MSG_DONTWAIT);
        if (n < 0) {
            if (errno == EAGAIN || errno == EWOULDBLOCK)
                return;
            CHECK (conn == bad_conn); //  only the failed connection's peer closes
            error ();
            return;
        }
        out_pos += (size_t) n;
    }
    void in_event () {}
    //  restart_output: src/stream_engine_base.cpp:383-390
    void encoded_ready ()
    {
        if (dead)
            return;
        set_pollout (true);
        out_event ();
    }
    void decoded_ready () {}
};

struct server_t : handler_t, zmqg::curve_link_events_t
{
    io_thread_t *io;
    int fd;
    zmqg::curve_encoding_gpu_t *codec;
    zmqg::curve_engine_link_t *link;
    std::vector<uint8_t> in; //  received, not yet parsed
    std::vector<zmqg::msg_buf_t> session;
    bool dead;
    size_t expect;

    bool finished () const { return dead || session.size () == expect; }
    void error ()
    {
        io->rm_fd (fd);
        close (fd);
        dead = true;
    }
    //  src/stream_engine_base.cpp:255-291 with the v2 decoder's framing
    void in_event ()
    {
        if (dead)
            return;
        uint8_t buf[65536];
        for (;;) {
            const ssize_t n = recv (fd, buf, sizeof buf, MSG_DONTWAIT);
            if (n > 0) {
                in.insert (in.end (), buf, buf + n);
                continue;
            }
            CHECK (n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)); //  the client never closes first
            break;
        }
        size_t pos = 0;
        while (!link->failed ()) {
            if (in.size () - pos < 2)
                break;
            const uint8_t fl = in[pos];
            size_t hdr = 2;
            uint64_t n = in[pos + 1];
            if (fl & 2) {
                hdr = 9;
                if (in.size () - pos < 9)
                    break;
                n = 0;
                for (int i = 0; i < 8; ++i)
                    n = (n << 8) | in[pos + 1 + i];
            }
            if (in.size () - pos - hdr < n)
                break; //  incomplete: wait for more bytes
            CHECK (link->submit_received (n ? &in[pos + hdr] : NULL, (size_t) n) == 0);
            pos += hdr + (size_t) n;
        }
        in.erase (in.begin (), in.begin () + (long) pos);
    }
    void out_event () {}
    void encoded_ready () {}
    //  restart_input: decoded messages go to the session; a failure is the
    //  engine's error (protocol_error), which closes the connection
    void decoded_ready ()
    {
        if (dead)
            return;
        zmqg::msg_buf_t m;
        while (link->next_decoded (m))
            session.push_back (m);
        if (link->failed ())
            error ();
    }
};

//  A link closed with messages in flight and a new link opened at once: the
//  old results must not reach the new link (routed by id, not address).
static void close_in_flight (const zmqg::curve_batcher_t::config_t &cfg_)
{
    zmqg_ctx *ctx = NULL;
    CHECK (zmqg_ctx_create (0, 2, &ctx) == 0);
    {
        zmqg::curve_io_hook_t hook (ctx, cfg_);
        CHECK (hook.init () == 0);
        zmqg::curve_encoding_gpu_t a (ctx, 0, client_prefix, server_prefix, false),
          b (ctx, 1, client_prefix, server_prefix, false);
        for (int i = 0; i < 32; ++i)
            a.get_writable_precom_buffer ()[i] = b.get_writable_precom_buffer ()[i] = (uint8_t) i;
        std::vector<uint8_t> msg (700, 7);
        zmqg::curve_engine_link_t *l1 = new zmqg::curve_engine_link_t (&hook, &a);
        for (int i = 0; i < 20; ++i)
            CHECK (l1->submit_send (&msg[0], msg.size (), 0) == 0);
        CHECK (hook.timer_event () == 0); //  launched: in flight now
        delete l1;
        zmqg::curve_engine_link_t *l2 = new zmqg::curve_engine_link_t (&hook, &b);
        CHECK (l2->submit_send (&msg[0], 5, 0) == 0);
        CHECK (hook.drain () >= 0);
        std::vector<uint8_t> w;
        int got = 0;
        while (l2->next_encoded (w)) {
            CHECK (w.size () == 5 + 33);
            ++got;
        }
        CHECK (got == 1 && l2->sends_in_flight () == 0);
        delete l2;
    }
    CHECK (zmqg_ctx_destroy (ctx) == 0);
}

static std::atomic<int> threads_done (0);

int main (int argc, char **argv)
{
    if (argc == 5 && strcmp (argv[1], "bench") == 0) {
        bench_mode = true;
        n_conn = atoi (argv[2]);
        n_msgs = atoi (argv[3]);
        bench_size = (size_t) atol (argv[4]);
        bad_conn = bad_msg = -1;
        CHECK (n_conn > 0 && n_msgs > 0);
    }
    //  a hung exchange ends the process (the exit code names it)
    std::thread watchdog ([] {
        for (int i = 0; i < watchdog_s * 10; ++i) {
            if (threads_done.load () == 2)
                return;
            usleep (100000);
        }
        fprintf (stderr, "watchdog: no completion within %d s\n", watchdog_s);
        _exit (3);
    });

    zmqg::curve_batcher_t::config_t cfg;
    if (!bench_mode) {
        cfg.slot_msgs = 64;
        cfg.slot_bytes = 64 << 10;
        cfg.slots = 3;
        close_in_flight (cfg);
    }

    io_thread_t ta (cfg), tb (cfg);
    static const size_t sizes[] = {0, 1, 31, 32, 33, 100, 255, 256, 1000, 4000, 5000, 20000};
    static const uint8_t flag_set[] = {0, 0, 0, zmqg::msg_more, zmqg::msg_subscribe, zmqg::msg_cancel};
    std::vector<client_t> cl (n_conn);
    std::vector<server_t> sv (n_conn);
    for (int c = 0; c < n_conn; ++c) {
        int sp[2];
        CHECK (socketpair (AF_UNIX, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0, sp) == 0);
        client_t &k = cl[c];
        server_t &s = sv[c];
        k.io = &ta;
        k.fd = sp[0];
        k.conn = c;
        s.io = &tb;
        s.fd = sp[1];
        k.codec = new zmqg::curve_encoding_gpu_t (ta.ctx, c, client_prefix, server_prefix, false);
        s.codec = new zmqg::curve_encoding_gpu_t (tb.ctx, c, server_prefix, client_prefix, false);
        for (int i = 0; i < 32; ++i)
            k.codec->get_writable_precom_buffer ()[i] =
              s.codec->get_writable_precom_buffer ()[i] = (uint8_t) rnd ();
        //  the handshake's nonces (HELLO 1, INITIATE 2; the server saw INITIATE's)
        k.codec->get_and_inc_nonce ();
        k.codec->get_and_inc_nonce ();
        s.codec->set_peer_nonce (2);
        k.link = new zmqg::curve_engine_link_t (ta.hook, k.codec, &k);
        s.link = new zmqg::curve_engine_link_t (tb.hook, s.codec, &s);
        k.pulled = k.framed = k.out_pos = 0;
        k.pollout = true; //  the engine starts with POLLOUT set (plug)
        k.dead = s.dead = false;
        s.expect = c == bad_conn ? (size_t) bad_msg : (size_t) n_msgs;
        for (int m = 0; m < n_msgs; ++m) {
            zmqg::msg_buf_t msg;
            msg.bytes.resize (bench_mode ? bench_size : sizes[rnd () % (sizeof sizes / sizeof sizes[0])]);
            for (size_t j = 0; j < msg.bytes.size (); ++j)
                msg.bytes[j] = (uint8_t) rnd ();
            msg.flags = bench_mode ? 0 : flag_set[rnd () % (sizeof flag_set / sizeof flag_set[0])];
            k.session.push_back (msg);
        }
        ta.add_fd (k.fd, &k, EPOLLOUT);
        tb.add_fd (s.fd, &s, EPOLLIN);
    }

    const double t0 = now_s ();
    std::thread a ([&] {
        ta.loop ([&] {
            for (int c = 0; c < n_conn; ++c)
                if (!cl[c].finished ())
                    return false;
            return true;
        });
        ++threads_done;
    });
    std::thread b ([&] {
        tb.loop ([&] {
            for (int c = 0; c < n_conn; ++c)
                if (!sv[c].finished ())
                    return false;
            return true;
        });
        ++threads_done;
    });
    a.join ();
    b.join ();
    const double dt = now_s () - t0;
    watchdog.join ();

    for (int c = 0; c < n_conn; ++c) {
        const size_t expect = c == bad_conn ? (size_t) bad_msg : (size_t) n_msgs;
        CHECK (sv[c].session.size () == expect);
        CHECK (sv[c].link->failed () == (c == bad_conn ? ZMQG_ERR_CRYPTOGRAPHIC : 0));
        CHECK (sv[c].dead == (c == bad_conn));
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
    for (int c = 0; c < n_conn; ++c) {
        delete cl[c].link;
        delete sv[c].link;
        delete cl[c].codec;
        delete sv[c].codec;
        if (!cl[c].dead)
            close (cl[c].fd);
        if (!sv[c].dead)
            close (sv[c].fd);
    }
    delete ta.hook;
    delete tb.hook;
    CHECK (zmqg_ctx_destroy (ta.ctx) == 0 && zmqg_ctx_destroy (tb.ctx) == 0);
    if (bench_mode) {
        const double msgs = (double) n_conn * n_msgs;
        printf ("RATE conns %d msgs %d size %zu ms %.1f msgs_per_s %.0f payload_MB_per_s %.1f waits %ld/%ld "
                "hook_wakes %ld/%ld\n",
                n_conn, n_msgs, bench_size, dt * 1e3, msgs / dt, msgs * bench_size / dt / 1e6, ta.waits, tb.waits,
                ta.hook_wakes, tb.hook_wakes);
        return 0;
    }
    printf ("OK %d waits %ld/%ld hook_wakes %ld/%ld ms %.1f\n", n_conn * n_msgs, ta.waits, tb.waits,
            ta.hook_wakes, tb.hook_wakes, dt * 1e3);
    return 0;
}
