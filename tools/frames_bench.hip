// Frame kernel (libzmq_amd/csrc/curve_frames.hpp) against the library's
// head/body path: bit-exactness and timing at G = 1, 2, 4 lanes per frame.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/bin/frames_bench tools/frames_bench.hip -Llibzmq_amd -lzmqg_curve
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

#include "../libzmq_amd/csrc/curve_frames.hpp"

using namespace zmqg;

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__global__ void k_mksession(DevSession *s, const uint32_t *in)
{
    uint32_t k[8];
    for (int i = 0; i < 8; ++i)
        k[i] = in[i];
    hsalsa20(s->enc_key, k, in + 8);
    hsalsa20(s->dec_key, k, in + 8); // the decoder mirrors the encoder (client prefix)
    s->downgrade_sub = 0;
}

static uint64_t sm(uint64_t &s)
{
    uint64_t z = (s += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

int main(int argc, char **argv)
{
    const uint32_t n = argc > 1 ? atoi(argv[1]) : 65536, P = argc > 2 ? atoi(argv[2]) : 1024;
    const int reps = 20;
    const uint32_t W = P + 33;
    uint64_t seed = 1;
    std::vector<uint8_t> pay((size_t) n * P + 64), flags(n);
    for (auto &b : pay)
        b = (uint8_t) sm(seed);
    std::vector<uint32_t> sid(n, 0), len(n, P), wl(n, W);
    std::vector<uint64_t> nonce(n), ioff(n), ooff(n);
    for (uint32_t i = 0; i < n; ++i) {
        nonce[i] = 3 + i;
        flags[i] = (i % 16 == 0) ? 1 : 0;
        ioff[i] = (uint64_t) i * P;
        ooff[i] = (uint64_t) i * W;
    }
    uint8_t precom[32];
    for (int i = 0; i < 32; ++i)
        precom[i] = (uint8_t) sm(seed);
    const char *cp = "CurveZMQMESSAGEC", *sp = "CurveZMQMESSAGES";
    auto dev = [](const void *h, size_t b) {
        void *d;
        CHECK(hipMalloc(&d, b + 64));
        CHECK(hipMemcpy(d, h, b, hipMemcpyHostToDevice));
        return d;
    };
    uint32_t *d_sid = (uint32_t *) dev(sid.data(), 4 * n), *d_len = (uint32_t *) dev(len.data(), 4 * n),
             *d_wl = (uint32_t *) dev(wl.data(), 4 * n);
    uint64_t *d_nonce = (uint64_t *) dev(nonce.data(), 8 * n), *d_ioff = (uint64_t *) dev(ioff.data(), 8 * n),
             *d_ooff = (uint64_t *) dev(ooff.data(), 8 * n);
    uint8_t *d_flags = (uint8_t *) dev(flags.data(), n), *d_pay = (uint8_t *) dev(pay.data(), pay.size());
    const size_t wb = (size_t) n * W + 64;
    uint8_t *d_ref, *d_wire, *d_back, *d_fl;
    int32_t *d_st;
    unsigned long long *d_v;
    CHECK(hipMalloc(&d_ref, wb));
    CHECK(hipMalloc(&d_wire, wb));
    CHECK(hipMalloc(&d_back, pay.size()));
    CHECK(hipMalloc(&d_fl, n));
    CHECK(hipMalloc(&d_st, 4 * n));
    CHECK(hipMalloc(&d_v, 32 * n + 64));
    CHECK(hipMemset(d_v, 0, 32 * n + 64));
    CHECK(hipMemset(d_ref, 0, wb));
    zmqg_ctx *ctx;
    if (zmqg_ctx_create(0, 1, &ctx) || zmqg_session_set(ctx, 0, precom, (const uint8_t *) cp, (const uint8_t *) sp, 0, 0))
        return printf("ctx failed\n"), 1;
    DevSession *d_ses;
    CHECK(hipMalloc(&d_ses, sizeof(DevSession)));
    {
        uint32_t in[16];
        memcpy(in, precom, 32);
        memcpy(in + 8, cp, 16);
        uint32_t *d_in = (uint32_t *) dev(in, 64);
        hipLaunchKernelGGL(k_mksession, dim3(1), dim3(1), 0, 0, d_ses, d_in);
    }
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    auto timeit = [&](auto fn) {
        fn();
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(a, 0));
        for (int r = 0; r < reps; ++r)
            fn();
        CHECK(hipEventRecord(b, 0));
        CHECK(hipEventSynchronize(b));
        float ms;
        CHECK(hipEventElapsedTime(&ms, a, b));
        return ms * 1000.0 / reps;
    };
    double t_ref = timeit([&] { zmqg_encode_batch(ctx, n, d_sid, d_nonce, d_flags, d_ioff, d_len, d_pay, d_ooff, d_ref, 0); });
    std::vector<uint8_t> h_ref(wb), h_new(wb), h_back(pay.size());
    CHECK(hipMemcpy(h_ref.data(), d_ref, wb, hipMemcpyDeviceToHost));
    printf("n=%u P=%u library encode %.1f us\n", n, P, t_ref);
    ZState *d_zs;
    CHECK(hipMalloc(&d_zs, sizeof(ZState)));
    {
        ZState z0{};
        z0.epoch = 1;
        CHECK(hipMemcpy(d_zs, &z0, sizeof z0, hipMemcpyHostToDevice));
    }
    unsigned long long *d_clk;
    CHECK(hipMalloc(&d_clk, 32 * 4096));
    ReplayOut rpo{};
    rpo.clk = d_clk;
    rpo.vout = d_v;
    rpo.psnap = d_v + n;
    rpo.peer = d_v + 3 * n;
    int fails = 0;
    auto run = [&](auto kenc, auto kdec, int G) {
        CHECK(hipMemset(d_clk, 0, 32 * 4096));
        const uint32_t blocks = (uint32_t) (((uint64_t) n * G + 255) / 256);
        CHECK(hipMemset(d_wire, 0, wb));
        double te = timeit([&] {
            hipLaunchKernelGGL(kenc, dim3(blocks), dim3(256), 0, 0, n, d_sid, d_nonce, d_flags, d_ioff, d_len, d_pay,
                               d_ooff, d_wire, d_ses, 1u, 0xffffffffu, nullptr, nullptr, rpo, NoBigFrames{}, d_zs, FrameCtl{});
        });
        CHECK(hipMemcpy(h_new.data(), d_wire, wb, hipMemcpyDeviceToHost));
        size_t bad = 0, first = (size_t) -1;
        for (size_t k = 0; k < wb; ++k)
            if (h_ref[k] != h_new[k]) { ++bad; if (first == (size_t) -1) first = k; }
        CHECK(hipMemset(d_back, 0, pay.size()));
        CHECK(hipMemset(d_st, 0x7f, 4 * n));
        double td = timeit([&] {
            hipLaunchKernelGGL(kdec, dim3(blocks), dim3(256), 0, 0, n, d_sid, (const uint64_t *) nullptr,
                               (const uint8_t *) nullptr, d_ooff, d_wl, d_ref, d_ioff, d_back, d_ses, 1u, 0xffffffffu,
                               d_fl, d_st, rpo, NoBigFrames{}, d_zs, FrameCtl{});
        });
        CHECK(hipMemcpy(h_back.data(), d_back, pay.size(), hipMemcpyDeviceToHost));
        std::vector<int32_t> st(n);
        std::vector<uint8_t> fl(n);
        CHECK(hipMemcpy(st.data(), d_st, 4 * n, hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(fl.data(), d_fl, n, hipMemcpyDeviceToHost));
        size_t bad2 = 0, bads = 0;
        for (size_t k = 0; k < (size_t) n * P; ++k)
            bad2 += h_back[k] != pay[k];
        for (uint32_t k = 0; k < n; ++k)
            bads += st[k] != 0 || fl[k] != flags[k];
        {
            const uint32_t nwg = blocks;
            std::vector<unsigned long long> ck(4 * nwg);
            CHECK(hipMemcpy(ck.data(), d_clk, 32 * nwg, hipMemcpyDeviceToHost));
            unsigned long long t0 = ~0ull, t1 = 0;
            for (uint32_t w = 0; w < nwg; ++w) {
                t0 = ck[4 * w] < t0 ? ck[4 * w] : t0;
                t1 = ck[4 * w + 1] > t1 ? ck[4 * w + 1] : t1;
            }
            char fn[64];
            snprintf(fn, sizeof fn, "gpurun_out/wg_G%d.csv", G);
            FILE *f = fopen(fn, "w");
            double dsum = 0, dmax = 0, smax = 0;
            for (uint32_t w = 0; w < nwg; ++w) {
                const double st = (ck[4 * w] - t0) / 100.0, du = (ck[4 * w + 1] - ck[4 * w]) / 100.0;
                dsum += du;
                dmax = du > dmax ? du : dmax;
                smax = st > smax ? st : smax;
                if (f)
                    fprintf(f, "%u,%.2f,%.2f,%llu,%llu,%llu\n", w, st, du, ck[4 * w + 2], ck[4 * w + 3] >> 32,
                            ck[4 * w + 3] & 0xffffffffull);
            }
            if (f)
                fclose(f);
            printf("   decode workgroups: span %.1f us, mean %.1f us, max %.1f us, latest start %.1f us\n",
                   (t1 - t0) / 100.0, dsum / nwg, dmax, smax);
        }
        printf("G=%d encode %.1f us (%.0f GB/s payload) mismatched %zu (first %zd) | decode %.1f us (%.0f GB/s) payload mismatches %zu status/flag %zu\n",
               G, te, (double) n * P / te / 1e3, bad, (ssize_t) first, td, (double) n * P / td / 1e3, bad2, bads);
        fails += bad || bad2 || bads;
    };
    if (getenv("FB_ENC2_ONLY")) { // instruction-count experiments: the G = 2 encode kernel alone
        const uint32_t blocks = (uint32_t) (((uint64_t) n * 2 + 255) / 256);
        double te = timeit([&] {
            hipLaunchKernelGGL((k_frames<false, 2, NoBigFrames>), dim3(blocks), dim3(256), 0, 0, n, d_sid, d_nonce,
                               d_flags, d_ioff, d_len, d_pay, d_ooff, d_wire, d_ses, 1u, 0xffffffffu, nullptr, nullptr,
                               rpo, NoBigFrames{}, d_zs, FrameCtl{});
        });
        printf("G=2 encode only: %.1f us\n", te);
        return 0;
    }
    {
        // single-session replay in-kernel (decoupled look-back), G = 2
        unsigned long long *lbf, *lba, *lbi, *ex;
        uint32_t *tk;
        CHECK(hipMalloc(&lbf, 8 * n));
        CHECK(hipMalloc(&lba, 8 * n));
        CHECK(hipMalloc(&lbi, 8 * n));
        CHECK(hipMalloc(&ex, 8 * n));
        CHECK(hipMalloc(&tk, 8));
        CHECK(hipMemset(lbf, 0, 8 * n));
        CHECK(hipMemset(tk, 0, 8));
        const uint32_t blocks = (uint32_t) (((uint64_t) n * 2 + 255) / 256);
        for (uint32_t dbg : {3u, 2u, 1u, 0u}) {
        double td = timeit([&] {
            ReplayOut r = rpo;
            r.dbg = dbg;
            r.excl = ex;
            r.lb_flag = lbf;
            r.lb_agg = lba;
            r.lb_inc = lbi;
            hipLaunchKernelGGL((k_frames<true, 2, NoBigFrames>), dim3(blocks), dim3(256), 0, 0, n, d_sid,
                               (const uint64_t *) nullptr, (const uint8_t *) nullptr, d_ooff, d_wl, d_ref, d_ioff,
                               d_back, d_ses, 1u, 0xffffffffu, d_fl, d_st, r, NoBigFrames{}, d_zs, FrameCtl{});
        });
        printf("dbg=%u: %.1f us\n", dbg, td);
        }
        std::vector<int32_t> st(n);
        CHECK(hipMemcpy(st.data(), d_st, 4 * n, hipMemcpyDeviceToHost));
        unsigned long long pe = 0;
        CHECK(hipMemcpy(&pe, d_v + 3 * n, 8, hipMemcpyDeviceToHost));
        size_t bads = 0;
        for (uint32_t k = 0; k < n; ++k)
            bads += st[k] != 0;
        printf("G=2 decode with look-back replay: status errors %zu\n", bads);
        (void) pe;
    }
    run(k_frames<false, 1, NoBigFrames>, k_frames<true, 1, NoBigFrames>, 1);
    run(k_frames<false, 2, NoBigFrames>, k_frames<true, 2, NoBigFrames>, 2);
    run(k_frames<false, 4, NoBigFrames>, k_frames<true, 4, NoBigFrames>, 4);
    return fails ? 2 : 0;
}
