// Per-message latency of the drop-in codec (curve_encoding_gpu_t), one
// message per device call as the reference engine calls its codec
// (src/stream_engine_base.cpp:281-291, :331-348):
//   msg   encode_msg / decode_msg (zmqg_encode_msg / zmqg_decode_msg: one
//         copy into the ctx's device-mapped message buffer, the frame kernel
//         in place over PCIe, one copy out)
//   many  encode_many / decode_many with n = 1 (descriptor vectors, staging
//         copy, hipMemcpy H2D, kernels, hipMemcpy D2H, copy out: round 2's
//         single-message path)
// Prints us per encode+decode round trip by payload size.
// Build: g++ -O2 -std=c++11 -Ilibzmq_amd/host tools/msg_latency.cpp
//        libzmq_amd/host/curve_encoding_gpu.cpp -Llibzmq_amd -lzmqg_curve
//        -Wl,-rpath,$PWD/libzmq_amd -o tools/bin/msg_latency
#include "curve_encoding_gpu.hpp"

#include <chrono>
#include <errno.h>
#include <stdio.h>
#include <string.h>
#include <vector>

static const char client_prefix[] = "CurveZMQMESSAGEC";
static const char server_prefix[] = "CurveZMQMESSAGES";

int main ()
{
    zmqg_ctx *ctx = zmqg::thread_ctx ();
    if (!ctx)
        return 1;
    uint32_t se = 0, sd = 0;
    if (zmqg::acquire_session (&se) || zmqg::acquire_session (&sd))
        return 1;
    zmqg::curve_encoding_gpu_t enc (ctx, se, client_prefix, server_prefix, false);
    zmqg::curve_encoding_gpu_t dec (ctx, sd, server_prefix, client_prefix, false);
    for (int i = 0; i < 32; ++i)
        enc.get_writable_precom_buffer ()[i] = dec.get_writable_precom_buffer ()[i] = (uint8_t) (i * 7 + 1);
    //  the handshake used nonces 1 (HELLO) and 2 (INITIATE), as in
    //  curve_client_t; the server saw INITIATE's
    enc.get_and_inc_nonce ();
    enc.get_and_inc_nonce ();
    dec.set_peer_nonce (2);
    const size_t sizes[] = {32, 1024, 4000, 65536, 1 << 20};
    for (size_t P : sizes) {
        std::vector<uint8_t> pay (P), wire (enc.wire_size (0, P)), back (P + 64);
        for (size_t i = 0; i < P; ++i)
            pay[i] = (uint8_t) (i * 13 + 5);
        const int iters = P >= (1u << 20) ? 50 : 500;
        for (int mode = 0; mode < 2; ++mode) {
            double us = 0;
            for (int it = -5; it < iters; ++it) {
                const auto t0 = std::chrono::steady_clock::now ();
                if (mode == 0) {
                    uint8_t fl = 0;
                    int ec = 0;
                    if (enc.encode_msg (&pay[0], P, 0, &wire[0]) != 0) {
                        perror ("encode_msg");
                        return 2;
                    }
                    if (dec.decode_msg (&wire[0], wire.size (), &back[0], &fl, &ec) != 0) {
                        fprintf (stderr, "decode_msg: errno %d event %d\n", errno, ec);
                        return 2;
                    }
                    if (memcmp (&back[0], &pay[0], P) != 0) {
                        fprintf (stderr, "payload mismatch at size %zu\n", P);
                        return 2;
                    }
                } else {
                    zmqg::msg_buf_t m;
                    m.bytes = pay;
                    zmqg::msg_buf_t *mp = &m;
                    zmqg::curve_encoding_gpu_t *ep = &enc, *dp = &dec;
                    int32_t st = 0;
                    if (zmqg::curve_encoding_gpu_t::encode_many (&ep, &mp, 1) != 0
                        || zmqg::curve_encoding_gpu_t::decode_many (&dp, &mp, 1, &st) != 0 || st != 0
                        || m.bytes != pay)
                        return 3;
                }
                const auto t1 = std::chrono::steady_clock::now ();
                if (it >= 0)
                    us += std::chrono::duration<double, std::micro> (t1 - t0).count ();
            }
            printf ("{\"path\": \"%s\", \"payload\": %zu, \"us_per_round_trip\": %.1f}\n", mode == 0 ? "msg" : "many",
                    P, us / iters);
            fflush (stdout);
        }
    }
    return 0;
}
