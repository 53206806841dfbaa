// CURVE PUSH/PULL over TCP between two libzmq builds (config 1's plumbing,
// BASELINE.json configs[0]): the stock reference library, whose MESSAGE
// codec is libsodium's, and the same library with the GPU codec swapped in
// (tests/host/build_libzmq.sh).  Written against the public zmq.h API only,
// in the shape of the reference's perf/local_thr.cpp (PULL, binds,
// receives) and perf/remote_thr.cpp (PUSH, connects, sends) with CURVE set
// up as tests/test_security_curve.cpp does (server: ZMQ_CURVE_SERVER and its
// secret key; client: the server's public key and its own key pair), using
// the test key pairs of doc/zmq_curve.adoc.
//
//   interop pull <endpoint> <ack_endpoint> <messages> <seed> <heartbeat_ivl_ms>
//   interop push <endpoint> <ack_endpoint> <messages> <seed> <heartbeat_ivl_ms>
//
// Once everything has arrived the PULL side answers on a second CURVE
// connection the other way (the PUSH process binds a CURVE-server PULL on
// ack_endpoint, the PULL process connects a client PUSH), so the sender
// closes only after delivery -- and each process runs both a CURVE client
// and a CURVE server.  (Closing right after the last send lost the tail of
// the stream with heartbeats on, with the stock library on both sides.)
//
// Message i of the plan (both sides derive it from the seed): one part of
// 1,024 bytes, except every 1,000th message from offset 1 .. 4 (0 B, 33 B,
// 64 KiB, 64 B) and every 50th (offset 7) is three parts (MORE) of 1 KiB,
// 100 B and 0 B; each byte comes from a splitmix64 stream keyed by (seed,
// message, part).  The receiver checks every part byte for byte, its size
// and its MORE flag, and prints "OK <messages> <parts> <msgs/s> <MB/s>".
// ZMTP heartbeats (ZMQ_HEARTBEAT_IVL) run on both sides, so PING/PONG
// commands go through the codec too (src/zmtp_engine.cpp:463, 479).
//
//   interop pub <endpoint> <ack_endpoint> - <seed> <heartbeat_ivl_ms>
//   interop sub <endpoint> <ack_endpoint> - <seed> <heartbeat_ivl_ms>
//
// PUB/SUB over CURVE: the SUB side's subscriptions travel as ZMTP 3.1
// SUBSCRIBE / CANCEL commands through the MESSAGE codec (msg_t::subscribe /
// cancel, src/curve_mechanism_base.cpp:118-164 on the encoding side, the
// other side's decode and src/xpub.cpp applying them), so a layout either
// codec got wrong shows up as a filter that does not match.  The PUB binds
// (CURVE server) and publishes rounds of "alpha", "beta" and "gamma" messages
// until told to stop; the SUB connects (CURVE client), subscribes to
// "alpha" and "beta", cancels "beta" once both arrive, then subscribes to
// "gamma": it checks every payload, that nothing outside its subscriptions
// ever arrives, that "beta" stops after the cancel and "gamma" starts after
// its subscription, then tells the PUB to stop (the acknowledgement
// connection) and prints "OK <received> <alpha> <beta> <gamma>".
#include <zmq.h>

#include <errno.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include <cxxabi.h>
#include <dirent.h>
#include <dlfcn.h>
#include <execinfo.h>
#include <pthread.h>
#include <signal.h>
#include <sys/syscall.h>

#include <algorithm>
#include <map>
#include <string>
#include <vector>

static const char server_public[] = "rq:rM>}U?@Lns47E1%kR.o@n%FcmmsL/@{H8]yf7";
static const char server_secret[] = "JTKVSB%%)wK0E.X)V>+}o?pNmC{O&4W4b!Ni{Lh6";
static const char client_public[] = "Yne@$w-vo<fVvi]a<NY6T1ed:M$fCG*[IaLV{hID";
static const char client_secret[] = "D:)Q[IlAW!ahhC2ac:9*A}h:p?([4%wOTJ%JR%cs";

#define CHECK(c)                                                               \
    do {                                                                       \
        if (!(c)) {                                                            \
            fprintf (stderr, "%s:%d: check failed: %s (errno %d: %s)\n",       \
                     __FILE__, __LINE__, #c, zmq_errno (),                      \
                     zmq_strerror (zmq_errno ()));                              \
            exit (1);                                                          \
        }                                                                      \
    } while (0)

static uint64_t splitmix (uint64_t &s_)
{
    uint64_t z = (s_ += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

//  the parts of message i
static void plan (uint64_t seed_, uint64_t i_, std::vector<std::vector<uint8_t> > &parts_)
{
    static const size_t special[] = {0, 33, 65536, 64};
    std::vector<size_t> sizes;
    if (i_ % 1000 >= 1 && i_ % 1000 <= 4)
        sizes.push_back (special[i_ % 1000 - 1]);
    else if (i_ % 50 == 7) {
        sizes.push_back (1024);
        sizes.push_back (100);
        sizes.push_back (0);
    } else
        sizes.push_back (1024);
    parts_.resize (sizes.size ());
    for (size_t p = 0; p < sizes.size (); ++p) {
        uint64_t s = seed_ * 0x100000001b3ull + i_ * 8 + p;
        parts_[p].resize (sizes[p]);
        for (size_t k = 0; k < sizes[p]; k += 8) {
            const uint64_t v = splitmix (s);
            for (size_t b = 0; b < 8 && k + b < sizes[p]; ++b)
                parts_[p][k + b] = (uint8_t) (v >> (8 * b));
        }
    }
}

static double now_s ()
{
    timespec t;
    clock_gettime (CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}

//  CPU seconds used so far by each thread of this process, by thread name
//  (/proc/self/task/*/stat: comm, utime, stime); INTEROP_THREAD_CPU set in
//  the environment makes both sides print the split of the timed window
//  to stderr ("cpu <thread> <seconds>"), to tell which thread bounds a rate.
typedef std::map<std::string, double> cpu_map_t;
static cpu_map_t thread_cpu ()
{
    cpu_map_t m;
    DIR *d = opendir ("/proc/self/task");
    if (!d)
        return m;
    const double tick = (double) sysconf (_SC_CLK_TCK);
    while (dirent *e = readdir (d)) {
        if (e->d_name[0] == '.')
            continue;
        char path[300], buf[1024];
        snprintf (path, sizeof path, "/proc/self/task/%s/stat", e->d_name);
        FILE *f = fopen (path, "r");
        if (!f)
            continue;
        const size_t n = fread (buf, 1, sizeof buf - 1, f);
        fclose (f);
        buf[n] = 0;
        char *l = strchr (buf, '('), *r = strrchr (buf, ')');
        if (!l || !r)
            continue;
        //  by name and thread id: threads a library starts from an I/O
        //  thread inherit its name (the HIP runtime's do)
        const std::string name = std::string (l + 1, r) + "#" + e->d_name;
        //  after ") ": state, then fields 4.. ; utime and stime are 14, 15
        unsigned long long ut = 0, st = 0;
        const char *q = r + 2;
        for (int field = 3; field < 14 && q; ++field) {
            q = strchr (q, ' ');
            if (q)
                ++q;
        }
        if (q && sscanf (q, "%llu %llu", &ut, &st) == 2)
            m[name] += (ut + st) / tick;
    }
    closedir (d);
    return m;
}

static void print_cpu (const cpu_map_t &a_, const cpu_map_t &b_, double wall_)
{
    if (!getenv ("INTEROP_THREAD_CPU"))
        return;
    for (cpu_map_t::const_iterator it = b_.begin (); it != b_.end (); ++it) {
        cpu_map_t::const_iterator p = a_.find (it->first);
        const double d = it->second - (p == a_.end () ? 0.0 : p->second);
        if (d > 0)
            fprintf (stderr, "cpu %s %.3f of %.3f s\n", it->first.c_str (), d, wall_);
    }
}

//  INTEROP_PROFILE set: a sampling profile of the threads named ZMQbg/IO/0
//  (the I/O thread, and threads it started) over the timed window -- a
//  sampler thread sends SIGPROF every 200 us, the handler records the stack
//  (backtrace), and stop () prints the functions seen most often on top of
//  the stack ("self") and anywhere in it ("incl"), per thread, to stderr.
//  A diagnostic of where the I/O thread's time goes; no effect otherwise.
namespace sampler
{
const int depth = 32;
const size_t cap = 60000;
static void *frames[cap][depth];
static int nframes[cap], owner[cap];
static volatile size_t count;
static volatile int active, stopping;
static std::vector<pid_t> targets;
static pthread_t thread;

static void on_signal (int)
{
    if (!active)
        return;
    const size_t i = __sync_fetch_and_add (&count, 1);
    if (i >= cap)
        return;
    const pid_t me = (pid_t) syscall (SYS_gettid);
    int k = 0;
    while (k < (int) targets.size () && targets[k] != me)
        ++k;
    owner[i] = k;
    nframes[i] = backtrace (frames[i], depth);
}

static void *loop (void *)
{
    while (!stopping) {
        for (size_t k = 0; k < targets.size (); ++k)
            syscall (SYS_tgkill, getpid (), targets[k], SIGPROF);
        usleep (200);
    }
    return NULL;
}

static void start ()
{
    if (!getenv ("INTEROP_PROFILE"))
        return;
    void *warm[4];
    backtrace (warm, 4); //  (loads libgcc before any signal arrives)
    DIR *d = opendir ("/proc/self/task");
    while (dirent *e = d ? readdir (d) : NULL) {
        char path[300], name[64] = "";
        snprintf (path, sizeof path, "/proc/self/task/%s/comm", e->d_name);
        FILE *f = fopen (path, "r");
        if (!f)
            continue;
        if (fgets (name, sizeof name, f) && strncmp (name, "ZMQbg/IO", 8) == 0)
            targets.push_back ((pid_t) atoi (e->d_name));
        fclose (f);
    }
    if (d)
        closedir (d);
    struct sigaction sa;
    memset (&sa, 0, sizeof sa);
    sa.sa_handler = on_signal;
    sa.sa_flags = SA_RESTART;
    sigaction (SIGPROF, &sa, NULL);
    active = 1;
    pthread_create (&thread, NULL, loop, NULL);
}

static std::string symbol (void *a_)
{
    Dl_info di;
    if (!dladdr (a_, &di) || !di.dli_sname) {
        char b[64];
        snprintf (b, sizeof b, "%s+?", di.dli_fname ? strrchr (di.dli_fname, '/') + 1 : "?");
        return b;
    }
    int st = 0;
    char *dm = abi::__cxa_demangle (di.dli_sname, NULL, NULL, &st);
    std::string r = st == 0 && dm ? dm : di.dli_sname;
    free (dm);
    const size_t paren = r.find ('(');
    return paren == std::string::npos ? r : r.substr (0, paren);
}

static void stop ()
{
    if (!active)
        return;
    active = 0;
    stopping = 1;
    pthread_join (thread, NULL);
    const size_t n = count < cap ? count : cap;
    fprintf (stderr, "prof threads %zu samples %zu\n", targets.size (), (size_t) count);
    for (size_t k = 0; k < targets.size (); ++k) {
        std::map<std::string, int> self, incl;
        int total = 0;
        for (size_t i = 0; i < n; ++i) {
            if (owner[i] != (int) k || nframes[i] <= 2)
                continue;
            ++total;
            //  frames 0, 1: the handler and the signal trampoline
            self[symbol (frames[i][2])]++;
            std::map<std::string, int> seen;
            for (int j = 2; j < nframes[i]; ++j)
                seen[symbol (frames[i][j])] = 1;
            for (std::map<std::string, int>::iterator it = seen.begin (); it != seen.end (); ++it)
                incl[it->first]++;
        }
        if (!total)
            continue;
        for (int pass = 0; pass < 2; ++pass) {
            std::map<std::string, int> &m = pass ? incl : self;
            std::vector<std::pair<int, std::string> > v;
            for (std::map<std::string, int>::iterator it = m.begin (); it != m.end (); ++it)
                v.push_back (std::make_pair (-it->second, it->first));
            std::sort (v.begin (), v.end ());
            for (size_t i = 0; i < v.size () && i < (pass ? 45u : 30u); ++i)
                fprintf (stderr, "prof %d %s %5.1f%% %s\n", (int) targets[k], pass ? "incl" : "self",
                         -100.0 * v[i].first / total, v[i].second.c_str ());
        }
        fprintf (stderr, "prof %d samples %d\n", (int) targets[k], total);
    }
}
}

static void setup_heartbeats (void *s_, int ivl_)
{
    if (ivl_ <= 0)
        return;
    const int timeout = 10000, ttl = 10000;
    CHECK (zmq_setsockopt (s_, ZMQ_HEARTBEAT_IVL, &ivl_, sizeof ivl_) == 0);
    CHECK (zmq_setsockopt (s_, ZMQ_HEARTBEAT_TIMEOUT, &timeout, sizeof timeout) == 0);
    CHECK (zmq_setsockopt (s_, ZMQ_HEARTBEAT_TTL, &ttl, sizeof ttl) == 0);
}

//  payload of round r of a topic: the topic, ':', 8 bytes of r, 100 bytes
static void pub_message (uint64_t seed_, const char *topic_, uint64_t r_, std::vector<uint8_t> &m_)
{
    const size_t tl = strlen (topic_);
    m_.assign (topic_, topic_ + tl);
    m_.push_back (':');
    for (int b = 0; b < 8; ++b)
        m_.push_back ((uint8_t) (r_ >> (8 * b)));
    uint64_t s = seed_ * 0x100000001b3ull + r_ * 4 + (uint64_t) tl;
    for (size_t k = 0; k < 100; k += 8) {
        const uint64_t v = splitmix (s);
        for (size_t b = 0; b < 8 && k + b < 100; ++b)
            m_.push_back ((uint8_t) (v >> (8 * b)));
    }
}

static void *curve_client (void *ctx_, int type_)
{
    void *s = zmq_socket (ctx_, type_);
    CHECK (s);
    CHECK (zmq_setsockopt (s, ZMQ_CURVE_SERVERKEY, server_public, 40) == 0);
    CHECK (zmq_setsockopt (s, ZMQ_CURVE_PUBLICKEY, client_public, 40) == 0);
    CHECK (zmq_setsockopt (s, ZMQ_CURVE_SECRETKEY, client_secret, 40) == 0);
    return s;
}

static void *curve_server (void *ctx_, int type_)
{
    void *s = zmq_socket (ctx_, type_);
    CHECK (s);
    const int one = 1;
    CHECK (zmq_setsockopt (s, ZMQ_CURVE_SERVER, &one, sizeof one) == 0);
    CHECK (zmq_setsockopt (s, ZMQ_CURVE_SECRETKEY, server_secret, 40) == 0);
    return s;
}

static const char *const topics[3] = {"alpha", "beta", "gamma"};

static int run_pub (void *ctx_, const char *ep_, const char *ack_ep_, uint64_t seed_, int ivl_)
{
    void *p = curve_server (ctx_, ZMQ_PUB);
    setup_heartbeats (p, ivl_);
    CHECK (zmq_bind (p, ep_) == 0);
    void *a = curve_server (ctx_, ZMQ_PULL);
    CHECK (zmq_bind (a, ack_ep_) == 0);
    printf ("READY\n");
    fflush (stdout);
    std::vector<uint8_t> m;
    const double t0 = now_s ();
    uint64_t r = 0;
    for (;; ++r) {
        for (int t = 0; t < 3; ++t) {
            pub_message (seed_, topics[t], r, m);
            CHECK (zmq_send (p, &m[0], m.size (), 0) == (int) m.size ());
        }
        char ack[8];
        const int rc = zmq_recv (a, ack, sizeof ack, ZMQ_DONTWAIT);
        if (rc == 4 && memcmp (ack, "STOP", 4) == 0)
            break;
        if (now_s () - t0 > 60) {
            fprintf (stderr, "FAIL: no STOP within 60 s\n");
            return 1;
        }
        usleep (50);
    }
    CHECK (zmq_close (a) == 0);
    CHECK (zmq_close (p) == 0);
    CHECK (zmq_ctx_term (ctx_) == 0);
    printf ("PUBLISHED %llu rounds\n", (unsigned long long) r + 1);
    return 0;
}

static int run_sub (void *ctx_, const char *ep_, const char *ack_ep_, uint64_t seed_, int ivl_)
{
    void *s = curve_client (ctx_, ZMQ_SUB);
    const int rcvtimeo = 30000;
    CHECK (zmq_setsockopt (s, ZMQ_RCVTIMEO, &rcvtimeo, sizeof rcvtimeo) == 0);
    setup_heartbeats (s, ivl_);
    CHECK (zmq_connect (s, ep_) == 0);
    CHECK (zmq_setsockopt (s, ZMQ_SUBSCRIBE, "alpha", 5) == 0);
    CHECK (zmq_setsockopt (s, ZMQ_SUBSCRIBE, "beta", 4) == 0);
    //  phases: 0 alpha + beta subscribed; 1 beta cancelled, waiting for it to
    //  stop; 2 gamma subscribed, waiting for it to start; 3 done
    int phase = 0;
    uint64_t got[3] = {0, 0, 0}, since_cancel = 0, last_beta = 0, received = 0;
    std::vector<uint8_t> want;
    char buf[256];
    while (phase < 3) {
        const int rc = zmq_recv (s, buf, sizeof buf, 0);
        if (rc < 0) {
            fprintf (stderr, "FAIL: receive in phase %d: %s\n", phase, zmq_strerror (zmq_errno ()));
            return 1;
        }
        int t = -1;
        for (int k = 0; k < 3; ++k)
            if ((size_t) rc > strlen (topics[k]) && memcmp (buf, topics[k], strlen (topics[k])) == 0
                && buf[strlen (topics[k])] == ':')
                t = k;
        if (t < 0 || (t == 2 && phase < 2)) {
            fprintf (stderr, "FAIL: message outside the subscriptions in phase %d\n", phase);
            return 1;
        }
        uint64_t r = 0;
        memcpy (&r, buf + strlen (topics[t]) + 1, 8);
        pub_message (seed_, topics[t], r, want);
        if ((size_t) rc != want.size () || memcmp (buf, &want[0], rc) != 0) {
            fprintf (stderr, "FAIL: payload of %s round %llu\n", topics[t], (unsigned long long) r);
            return 1;
        }
        ++got[t];
        ++received;
        if (t == 1)
            last_beta = received;
        if (phase == 0 && got[0] && got[1]) {
            CHECK (zmq_setsockopt (s, ZMQ_UNSUBSCRIBE, "beta", 4) == 0); //  a CANCEL command
            phase = 1;
            since_cancel = received;
        } else if (phase == 1 && received - last_beta >= 500 && received - since_cancel >= 500) {
            //  (beta published in the same rounds stopped coming: the cancel
            //  has been applied by the PUB side)
            CHECK (zmq_setsockopt (s, ZMQ_SUBSCRIBE, "gamma", 5) == 0);
            phase = 2;
        } else if (phase == 2 && t == 2) {
            phase = 3;
        }
        if (phase >= 2 && t == 1) {
            //  (every round publishes alpha and beta together: 500 alphas in
            //  a row mean the PUB has stopped queueing beta for this peer)
            fprintf (stderr, "FAIL: beta after its cancel had taken effect\n");
            return 1;
        }
    }
    void *a = curve_client (ctx_, ZMQ_PUSH);
    CHECK (zmq_connect (a, ack_ep_) == 0);
    CHECK (zmq_send (a, "STOP", 4, 0) == 4);
    CHECK (zmq_close (a) == 0);
    CHECK (zmq_close (s) == 0);
    CHECK (zmq_ctx_term (ctx_) == 0);
    printf ("OK %llu %llu %llu %llu\n", (unsigned long long) received, (unsigned long long) got[0],
            (unsigned long long) got[1], (unsigned long long) got[2]);
    return 0;
}

int main (int argc, char **argv)
{
    if (argc != 7) {
        fprintf (stderr, "usage: %s pull|push <endpoint> <ack_endpoint> <messages> <seed> <heartbeat_ivl_ms>\n",
                 argv[0]);
        return 2;
    }
    const bool pull = strcmp (argv[1], "pull") == 0;
    const char *endpoint = argv[2];
    const char *ack_endpoint = argv[3];
    const uint64_t n = strtoull (argv[4], NULL, 10);
    const uint64_t seed = strtoull (argv[5], NULL, 10);
    const int ivl = atoi (argv[6]);
    CHECK (zmq_has ("curve"));

    void *ctx = zmq_ctx_new ();
    CHECK (ctx);
    if (strcmp (argv[1], "pub") == 0)
        return run_pub (ctx, endpoint, ack_endpoint, seed, ivl);
    if (strcmp (argv[1], "sub") == 0)
        return run_sub (ctx, endpoint, ack_endpoint, seed, ivl);
    std::vector<std::vector<uint8_t> > parts;
    if (pull) {
        //  perf/local_thr.cpp, as the CURVE server (tests/test_security_curve.cpp)
        void *s = zmq_socket (ctx, ZMQ_PULL);
        CHECK (s);
        const int one = 1, rcvtimeo = 30000;
        CHECK (zmq_setsockopt (s, ZMQ_CURVE_SERVER, &one, sizeof one) == 0);
        CHECK (zmq_setsockopt (s, ZMQ_CURVE_SECRETKEY, server_secret, 40) == 0);
        CHECK (zmq_setsockopt (s, ZMQ_RCVTIMEO, &rcvtimeo, sizeof rcvtimeo) == 0);
        setup_heartbeats (s, ivl);
        CHECK (zmq_bind (s, endpoint) == 0);
        printf ("READY\n");
        fflush (stdout);
        zmq_msg_t m;
        CHECK (zmq_msg_init (&m) == 0);
        uint64_t frames = 0, bytes = 0;
        double t0 = 0;
        cpu_map_t c0;
        for (uint64_t i = 0; i < n; ++i) {
            plan (seed, i, parts);
            for (size_t p = 0; p < parts.size (); ++p) {
                const int rc = zmq_msg_recv (&m, s, 0);
                if (rc < 0) {
                    fprintf (stderr, "FAIL: receive of message %llu part %zu: %s\n", (unsigned long long) i, p,
                             zmq_strerror (zmq_errno ()));
                    return 1;
                }
                if (i == 0 && p == 0) {
                    t0 = now_s ();
                    c0 = thread_cpu ();
                }
                if (i == n / 5 && p == 0)
                    sampler::start (); //  (long after the device was set up: a
                                       //  signal storm during HIP's start-up
                                       //  fails it)
                const bool more = zmq_msg_more (&m) != 0;
                if ((size_t) rc != parts[p].size () || more != (p + 1 < parts.size ())
                    || (rc && memcmp (zmq_msg_data (&m), &parts[p][0], rc) != 0)) {
                    fprintf (stderr, "FAIL: message %llu part %zu: size %d (want %zu), more %d\n",
                             (unsigned long long) i, p, rc, parts[p].size (), (int) more);
                    return 1;
                }
                ++frames;
                bytes += rc;
            }
        }
        const double dt = now_s () - t0;
        sampler::stop ();
        print_cpu (c0, thread_cpu (), dt);
        CHECK (zmq_msg_close (&m) == 0);
        //  the acknowledgement, as a CURVE client of the sender's process
        void *a = zmq_socket (ctx, ZMQ_PUSH);
        CHECK (a);
        CHECK (zmq_setsockopt (a, ZMQ_CURVE_SERVERKEY, server_public, 40) == 0);
        CHECK (zmq_setsockopt (a, ZMQ_CURVE_PUBLICKEY, client_public, 40) == 0);
        CHECK (zmq_setsockopt (a, ZMQ_CURVE_SECRETKEY, client_secret, 40) == 0);
        CHECK (zmq_connect (a, ack_endpoint) == 0);
        CHECK (zmq_send (a, "DONE", 4, 0) == 4);
        CHECK (zmq_close (a) == 0);
        CHECK (zmq_close (s) == 0);
        CHECK (zmq_ctx_term (ctx) == 0);
        printf ("OK %llu %llu %.0f %.1f\n", (unsigned long long) n, (unsigned long long) frames,
                dt > 0 ? (n - 1) / dt : 0.0, dt > 0 ? bytes / dt / 1e6 : 0.0);
        return 0;
    }
    //  the acknowledgement's receiver, as a CURVE server
    void *a = zmq_socket (ctx, ZMQ_PULL);
    CHECK (a);
    const int one = 1, acktimeo = 60000;
    CHECK (zmq_setsockopt (a, ZMQ_CURVE_SERVER, &one, sizeof one) == 0);
    CHECK (zmq_setsockopt (a, ZMQ_CURVE_SECRETKEY, server_secret, 40) == 0);
    CHECK (zmq_setsockopt (a, ZMQ_RCVTIMEO, &acktimeo, sizeof acktimeo) == 0);
    CHECK (zmq_bind (a, ack_endpoint) == 0);
    //  perf/remote_thr.cpp, as the CURVE client
    void *s = zmq_socket (ctx, ZMQ_PUSH);
    CHECK (s);
    CHECK (zmq_setsockopt (s, ZMQ_CURVE_SERVERKEY, server_public, 40) == 0);
    CHECK (zmq_setsockopt (s, ZMQ_CURVE_PUBLICKEY, client_public, 40) == 0);
    CHECK (zmq_setsockopt (s, ZMQ_CURVE_SECRETKEY, client_secret, 40) == 0);
    setup_heartbeats (s, ivl);
    CHECK (zmq_connect (s, endpoint) == 0);
    cpu_map_t c0;
    double t0 = 0;
    for (uint64_t i = 0; i < n; ++i) {
        if (i == 1) {
            //  (after the first send, which waits for the handshake)
            t0 = now_s ();
            c0 = thread_cpu ();
        }
        if (i == n / 5)
            sampler::start ();
        plan (seed, i, parts);
        for (size_t p = 0; p < parts.size (); ++p)
            CHECK (zmq_send (s, parts[p].empty () ? NULL : &parts[p][0], parts[p].size (),
                             p + 1 < parts.size () ? ZMQ_SNDMORE : 0)
                   == (int) parts[p].size ());
    }
    char ack[8];
    const int rc = zmq_recv (a, ack, sizeof ack, 0);
    if (rc != 4 || memcmp (ack, "DONE", 4) != 0) {
        fprintf (stderr, "FAIL: no acknowledgement (%d)\n", rc);
        return 1;
    }
    sampler::stop ();
    print_cpu (c0, thread_cpu (), now_s () - t0);
    CHECK (zmq_close (a) == 0);
    CHECK (zmq_close (s) == 0);
    CHECK (zmq_ctx_term (ctx) == 0);
    printf ("SENT %llu ACKED\n", (unsigned long long) n);
    return 0;
}
