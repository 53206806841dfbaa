// Phase timing of k_frames_st (curve_frames_st.hpp), diagnostic build
// (-DZMQG_ST_STAMPS=1): per wave, s_memtime at entry (0), after the hand-off
// barrier (1), after window 0 / the first DMA (2), after barrier B_K (3+K),
// mid super-step (20+K: compute after window 2K, memory after its DMA and
// store issue), before B_K+1 (37+K: compute after window 2K+1, memory after
// its DMA wait), after B_KS (58), before B_fin (59), after it (60), end (61);
// s_memrealtime at entry (62) and end (63) for the clock.
// Config-2 shape: 65,536 frames of 1 KiB, encode then decode, third launch.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -DZMQG_ST_STAMPS=1 -o build/st_stamps tools/st_stamps.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <algorithm>
#include <vector>
#include "../libzmq_amd/csrc/curve_frames_st.hpp"
using namespace zmqg;

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

struct NoBig {
    __device__ void operator()(uint32_t, unsigned long long *, uint64_t) const {}
};

static long long med(std::vector<long long> v)
{
    if (v.empty())
        return -1;
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main()
{
    const uint32_t n = 65536, P = 1024, W = P + 33;
    std::vector<uint32_t> sid(n, 0), len(n, P), wl(n, W);
    std::vector<uint64_t> nonce(n), ioff(n), ooff(n);
    std::vector<uint8_t> flags(n, 0);
    for (uint32_t i = 0; i < n; ++i) {
        nonce[i] = 3 + i;
        ioff[i] = (uint64_t) i * P;
        ooff[i] = (uint64_t) i * W;
    }
    auto dev = [](const void *h, size_t b) {
        void *d = nullptr;
        if (hipMalloc(&d, b + 256) != hipSuccess || hipMemcpy(d, h, b, hipMemcpyHostToDevice) != hipSuccess)
            return (void *) nullptr;
        return d;
    };
    uint32_t *d_sid = (uint32_t *) dev(sid.data(), 4 * n), *d_len = (uint32_t *) dev(len.data(), 4 * n),
             *d_wl = (uint32_t *) dev(wl.data(), 4 * n);
    uint64_t *d_nonce = (uint64_t *) dev(nonce.data(), 8 * n), *d_ioff = (uint64_t *) dev(ioff.data(), 8 * n),
             *d_ooff = (uint64_t *) dev(ooff.data(), 8 * n);
    uint8_t *d_flags = (uint8_t *) dev(flags.data(), n);
    uint8_t *d_pay, *d_wire, *d_back, *d_fl;
    int32_t *d_st;
    CHECK(hipMalloc(&d_pay, (size_t) n * P + 256));
    CHECK(hipMemset(d_pay, 0x3c, (size_t) n * P + 256));
    CHECK(hipMalloc(&d_wire, (size_t) n * W + 256));
    CHECK(hipMalloc(&d_back, (size_t) n * P + 256));
    CHECK(hipMalloc(&d_fl, n));
    CHECK(hipMalloc(&d_st, 4 * n));
    DevSession *d_ses;
    CHECK(hipMalloc(&d_ses, sizeof(DevSession)));
    CHECK(hipMemset(d_ses, 0x11, sizeof(DevSession)));
    ZState *d_zs;
    CHECK(hipMalloc(&d_zs, sizeof(ZState)));
    ZState z0{};
    z0.epoch = 1;
    CHECK(hipMemcpy(d_zs, &z0, sizeof z0, hipMemcpyHostToDevice));
    unsigned long long *d_v, *d_clk;
    CHECK(hipMalloc(&d_v, 32ull * n + 64));
    CHECK(hipMemset(d_v, 0, 32ull * n + 64));
    const uint32_t nwg = n / kFramesBS, wpw = kSxThreads / 64;
    const size_t nwaves = (size_t) nwg * wpw;
    CHECK(hipMalloc(&d_clk, 8 * 64 * nwaves));
    ReplayOut rp{};
    rp.vout = d_v;
    rp.psnap = d_v + n;
    rp.peer = d_v + 3 * n;
    for (int dec = 0; dec < 2; ++dec) {
        for (int rep = 0; rep < 3; ++rep) {
            CHECK(hipMemset(d_clk, 0, 8 * 64 * nwaves));
            rp.clk = rep == 2 ? d_clk : nullptr;
            if (!dec)
                hipLaunchKernelGGL((k_frames_st<false, NoBig>), dim3(nwg), dim3(kSxThreads), 0, 0, n, d_sid, d_nonce,
                                   d_flags, d_ioff, d_len, d_pay, d_ooff, d_wire, d_ses, 1u, 0xffffffffu, nullptr,
                                   nullptr, rp, NoBig{}, d_zs, FrameCtl{});
            else
                hipLaunchKernelGGL((k_frames_st<true, NoBig>), dim3(nwg), dim3(kSxThreads), 0, 0, n, d_sid,
                                   (const uint64_t *) nullptr, (const uint8_t *) nullptr, d_ooff, d_wl, d_wire, d_ioff,
                                   d_back, d_ses, 1u, 0xffffffffu, d_fl, d_st, rp, NoBig{}, d_zs, FrameCtl{});
            CHECK(hipDeviceSynchronize());
        }
        std::vector<unsigned long long> c(64 * nwaves);
        CHECK(hipMemcpy(c.data(), d_clk, 8 * 64 * nwaves, hipMemcpyDeviceToHost));
        auto at = [&](size_t w, int sl) { return (long long) (c[64 * w + sl] - c[64 * w]); };
        printf("%s (cycles since the wave's entry, medians over waves)\n", dec ? "decode" : "encode");
        for (int role = 0; role < 2; ++role) {
            std::vector<size_t> ws;
            for (size_t w = 0; w < nwaves; ++w)
                if ((int) ((w % wpw) >= wpw / 2) == role && c[64 * w + 60])
                    ws.push_back(w);
            printf(" %s waves (%zu):", role ? "memory" : "compute", ws.size());
            for (int sl : {1, 2, 58, 59, 60, 61}) {
                std::vector<long long> v;
                for (size_t w : ws)
                    if (c[64 * w + sl])
                        v.push_back(at(w, sl));
                printf(" [%d] %lld", sl, med(v));
            }
            printf("\n  K: after B_K / mid / before B_K+1 / (next B release - arrival)\n");
            for (int K = 0; K < 10; ++K) {
                std::vector<long long> a, m, b, wt;
                for (size_t w : ws) {
                    if (!c[64 * w + 3 + K])
                        continue;
                    a.push_back(at(w, 3 + K));
                    m.push_back(at(w, 20 + K));
                    b.push_back(at(w, 37 + K));
                    const int nx = c[64 * w + 4 + K] ? 4 + K : 58;
                    wt.push_back(at(w, nx) - at(w, 37 + K));
                }
                if (a.empty())
                    break;
                printf("  %2d: %8lld %8lld %8lld  wait %6lld\n", K, med(a), med(m), med(b), med(wt));
            }
            // K = 3 detail (compute: window 6 -- 54 before the keystream (LDS reads issued),
            // 55 after keystream + MAC, 56 after the XOR, 57 after the ring writes;
            // memory: 54 after the DMA issue, 55 (super-group 2's) LDS reads landed, 56 stores issued)
            {
                std::vector<long long> v[4];
                for (size_t w : ws)
                    for (int q = 0; q < 4; ++q)
                        if (c[64 * w + 54 + q])
                            v[q].push_back(at(w, 54 + q) - at(w, 6));
                printf("  K=3 detail since B_3: %lld %lld %lld %lld\n", med(v[0]), med(v[1]), med(v[2]), med(v[3]));
            }
            std::vector<long long> dur, clk;
            for (size_t w : ws) {
                dur.push_back(at(w, 61));
                const double rt = (double) (c[64 * w + 63] - c[64 * w + 62]) * 10.0; // ns (100 MHz)
                if (rt > 0)
                    clk.push_back((long long) (1000.0 * at(w, 61) / rt));
            }
            std::sort(dur.begin(), dur.end());
            printf("  wave lifetime p10/p50/p90/max %lld %lld %lld %lld; clock MHz p50 %lld\n", dur[dur.size() / 10],
                   dur[dur.size() / 2], dur[dur.size() * 9 / 10], dur.back(), med(clk));
        }
    }
    return 0;
}
