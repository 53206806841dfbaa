// Per-call time of zmqg_encode_msg / zmqg_decode_msg (results ignored, so
// diagnostic builds with parts of k_msg ablated can be timed; run under
// rocprofv3 --kernel-trace --stats for the kernel's own duration).
// Build: g++ -O2 -std=c++11 tools/msg_kernel_bench.cpp -Llibzmq_amd -lzmqg_curve
//        -Wl,-rpath,$PWD/libzmq_amd -o tools/bin/msg_kernel_bench   (ZMQG_CURVE_SO: none; link a build)
#include "../include/zmqg_curve.h"

#include <chrono>
#include <stdio.h>
#include <string.h>
#include <vector>

int main (int argc, char **argv)
{
    const char *tag = argc > 1 ? argv[1] : "default";
    zmqg_ctx *ctx = NULL;
    if (zmqg_ctx_create (0, 2, &ctx) != 0)
        return 1;
    uint8_t precom[32], pfx_c[16], pfx_s[16];
    for (int i = 0; i < 32; ++i)
        precom[i] = (uint8_t) (i * 7 + 1);
    memcpy (pfx_c, "CurveZMQMESSAGEC", 16);
    memcpy (pfx_s, "CurveZMQMESSAGES", 16);
    if (zmqg_session_set (ctx, 0, precom, pfx_c, pfx_s, 0, 1) || zmqg_session_set (ctx, 1, precom, pfx_s, pfx_c, 0, 2))
        return 2;
    const uint32_t sizes[] = {32, 1024, 4000};
    uint64_t nonce = 3;
    for (uint32_t P : sizes) {
        std::vector<uint8_t> pay (P, 0x5a), wire (P + 64), back (P + 64);
        double us_e = 0, us_d = 0;
        const int iters = 2000;
        for (int it = -50; it < iters; ++it) {
            const auto t0 = std::chrono::steady_clock::now ();
            zmqg_encode_msg (ctx, 0, nonce++, 0, &pay[0], P, &wire[0]);
            const auto t1 = std::chrono::steady_clock::now ();
            uint8_t fl;
            int32_t st;
            zmqg_decode_msg (ctx, 1, &wire[0], P + 33, &back[0], &fl, &st);
            const auto t2 = std::chrono::steady_clock::now ();
            if (it >= 0) {
                us_e += std::chrono::duration<double, std::micro> (t1 - t0).count ();
                us_d += std::chrono::duration<double, std::micro> (t2 - t1).count ();
            }
        }
        printf ("{\"tag\": \"%s\", \"payload\": %u, \"encode_us\": %.2f, \"decode_us\": %.2f}\n", tag, P, us_e / iters,
                us_d / iters);
    }
    zmqg_ctx_destroy (ctx);
    return 0;
}
