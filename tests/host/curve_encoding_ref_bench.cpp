// CPU baseline on the reference's own CURVE MESSAGE codec: zmq::curve_encoding_t
// of the stock libzmq build (tests/host/build_libzmq.sh compiles
// src/curve_mechanism_base.cpp where it lies, over the image's libsodium
// 1.0.18), driven as the reference's unittests/unittest_curve_encoding.cpp:26-71
// drives it -- a client and a server encoding with precomputed keys from
// crypto_box_beforenm on fresh key pairs, msg_t::init_size for each message,
// encode on the client, decode on the server.  bench.py's cpu_baseline
// (kind "reference") runs it on the box's host cores.
//
//   curve_encoding_ref_bench <threads> <payload bytes> <seconds>
//
// Every thread owns one client/server pair (a connection lives on one I/O
// thread) and runs round trips until `seconds` have passed, checking every
// decoded payload against the input.  Prints
//   RATE threads <T> msgs <N> seconds <S> msgs_per_s <R> payload_GiB_per_s <G>
#include <precompiled.hpp> //  (platform.hpp, zmq.h: as every reference source starts)
#include <curve_mechanism_base.hpp>
#include <msg.hpp>

#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <vector>

static double now_s ()
{
    timespec t;
    clock_gettime (CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}

struct job_t
{
    size_t size;
    double seconds;
    unsigned long long msgs;
    int failed;
};

static void *run (void *arg_)
{
    job_t *j = static_cast<job_t *> (arg_);
    zmq::curve_encoding_t client ("CurveZMQMESSAGEC", "CurveZMQMESSAGES", false);
    zmq::curve_encoding_t server ("CurveZMQMESSAGES", "CurveZMQMESSAGEC", false);
    uint8_t cpub[32], csec[32], spub[32], ssec[32];
    if (crypto_box_keypair (cpub, csec) || crypto_box_keypair (spub, ssec)
        || crypto_box_beforenm (client.get_writable_precom_buffer (), spub, csec)
        || crypto_box_beforenm (server.get_writable_precom_buffer (), cpub, ssec)) {
        j->failed = 1;
        return NULL;
    }
    //  (unittest_curve_encoding.cpp:59: the client's first nonce is 1)
    server.set_peer_nonce (0);
    std::vector<uint8_t> payload (j->size);
    for (size_t i = 0; i < j->size; ++i)
        payload[i] = (uint8_t) (i * 131 + 7);
    const double t_end = now_s () + j->seconds;
    unsigned long long n = 0;
    while (true) {
        for (int k = 0; k < 64; ++k) {
            zmq::msg_t msg;
            if (msg.init_size (j->size) != 0) {
                j->failed = 1;
                return NULL;
            }
            if (j->size)
                memcpy (msg.data (), &payload[0], j->size);
            int code = 0;
            if (client.encode (&msg) != 0 || server.decode (&msg, &code) != 0
                || msg.size () != j->size
                || (j->size && memcmp (msg.data (), &payload[0], j->size) != 0)) {
                j->failed = 1;
                msg.close ();
                return NULL;
            }
            msg.close ();
            ++n;
        }
        if (now_s () >= t_end)
            break;
    }
    j->msgs = n;
    return NULL;
}

int main (int argc, char **argv)
{
    if (argc != 4) {
        fprintf (stderr, "usage: %s <threads> <payload bytes> <seconds>\n", argv[0]);
        return 2;
    }
    const int threads = atoi (argv[1]);
    const size_t size = (size_t) atol (argv[2]);
    const double seconds = atof (argv[3]);
    if (threads < 1 || sodium_init () < 0)
        return 2;
    std::vector<job_t> jobs (threads);
    std::vector<pthread_t> th (threads);
    const double t0 = now_s ();
    for (int t = 0; t < threads; ++t) {
        jobs[t].size = size;
        jobs[t].seconds = seconds;
        jobs[t].msgs = 0;
        jobs[t].failed = 0;
        pthread_create (&th[t], NULL, run, &jobs[t]);
    }
    unsigned long long msgs = 0;
    for (int t = 0; t < threads; ++t) {
        pthread_join (th[t], NULL);
        if (jobs[t].failed) {
            fprintf (stderr, "FAIL: thread %d\n", t);
            return 1;
        }
        msgs += jobs[t].msgs;
    }
    const double dt = now_s () - t0;
    printf ("RATE threads %d msgs %llu seconds %.3f msgs_per_s %.0f payload_GiB_per_s %.4f\n", threads, msgs, dt,
            msgs / dt, msgs * (double) size / dt / (1u << 30));
    return 0;
}
