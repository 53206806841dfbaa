// Phase timing of the one-lane-per-frame kernel (k_frames_seq), diagnostic
// build (-DZMQG_SEQ_STAMPS=1): per wave, s_memtime at entry (0), before
// window 0 (1), after it (2), at the start of step t (3+t) and after the
// wait for step t's input words (24+t), after the loop (60), at the end
// (61); for steps 1..7 also after the input words are in (44+t), before the
// stores (52+t) and after them (36+t); slot 62 holds the wave's placement
// (XCC_ID : HW_ID, k_frames_seq).  Default shape config 2 (65,536 frames of
// 1 KiB, one session), encode then decode; STAMP_N / STAMP_P / STAMP_S set
// another (config 4 below).  STAMP_REPS launches per direction back to back
// (the clock settles), the last two stamped: the second with every
// workgroup given the data of the one half a grid away, and the two
// compared (slow CU or slow data).
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -DZMQG_SEQ_STAMPS=1 -DSTAMP_REPS=400 -o tools/bin/seq_stamps tools/seq_stamps.hip
// (add -DSTAMP_LDS=1 for k_frames_lds: slots 3+t step start, 44+t after the
// wait, 52+t after the DMA and store issue, 24+t after keystream and MAC,
// 36+t after the ring write)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <vector>
#include <algorithm>
#include <math.h>
#include "../libzmq_amd/csrc/curve_frames_lds.hpp"
#ifndef STAMP_SHMEM_KB
#define STAMP_SHMEM_KB 0 // dynamic LDS requested per workgroup (unused; 84: one workgroup per CU)
#endif
#ifndef STAMP_N
#define STAMP_N 65536 // frames (config 4: -DSTAMP_N=16777216 -DSTAMP_P=256 -DSTAMP_S=1024 -DSTAMP_LDS=1)
#endif
#ifndef STAMP_P
#define STAMP_P 1024 // payload bytes per frame
#endif
#ifndef STAMP_S
#define STAMP_S 1 // sessions, frame i on session i mod STAMP_S
#endif
#ifndef STAMP_REPS
#define STAMP_REPS 3 // launches per direction; the last two are stamped (plain, then rotated offsets; more: the clock settles first)
#endif
#ifndef STAMP_LDS
#define STAMP_LDS 0 // 1: stamp k_frames_lds instead of k_frames_seq
#endif
#if STAMP_LDS
#define KFR k_frames_lds
#else
#define KFR k_frames_seq
#endif
using namespace zmqg;
// the frame kernels' BigOp without big frames (the library's NoBigFrames
// predates the decode's ZMTP hooks, which the kernels now read)
struct StampNoBig {
    const uint8_t *zflags = nullptr;
    const unsigned long long *res_src = nullptr;
    unsigned long long *res_dst = nullptr;
    __device__ void operator()(uint32_t, unsigned long long *, uint64_t) const {}
};

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main()
{
    const uint32_t n = STAMP_N, P = STAMP_P, W = P + 33, NS = STAMP_S;
    std::vector<uint32_t> sid(n, 0), len(n, P), wl(n, W);
    for (uint32_t i = 0; i < n; ++i)
        sid[i] = i % NS; // (config 4: frame i on session i mod 1,024)
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
    // the same frames, each workgroup given the data of the workgroup half a
    // grid away (frame i at frame (i + n/2) % n's offsets): a second stamped
    // launch with these tells a slow CU from slow data
    std::vector<uint64_t> ioff_r(n), ooff_r(n);
    for (uint32_t i = 0; i < n; ++i) {
        ioff_r[i] = ioff[(i + n / 2) % n];
        ooff_r[i] = ooff[(i + n / 2) % n];
    }
    uint64_t *d_ioff_r = (uint64_t *) dev(ioff_r.data(), 8 * n), *d_ooff_r = (uint64_t *) dev(ooff_r.data(), 8 * n);
    uint8_t *d_pay, *d_wire, *d_back, *d_fl;
    int32_t *d_st;
    CHECK(hipMalloc(&d_pay, (size_t) n * P + 256));
    CHECK(hipMemset(d_pay, 0x3c, (size_t) n * P + 256));
    CHECK(hipMalloc(&d_wire, (size_t) n * W + 256));
    CHECK(hipMalloc(&d_back, (size_t) n * P + 256));
    CHECK(hipMalloc(&d_fl, n));
    CHECK(hipMalloc(&d_st, 4 * n));
    DevSession *d_ses;
    CHECK(hipMalloc(&d_ses, NS * sizeof(DevSession)));
    CHECK(hipMemset(d_ses, 0x11, NS * sizeof(DevSession)));
    ZState *d_zs;
    CHECK(hipMalloc(&d_zs, sizeof(ZState)));
    ZState z0{};
    z0.epoch = 1;
    CHECK(hipMemcpy(d_zs, &z0, sizeof z0, hipMemcpyHostToDevice));
    unsigned long long *d_v, *d_clk;
    CHECK(hipMalloc(&d_v, 32ull * n + 64));
    CHECK(hipMemset(d_v, 0, 32ull * n + 64));
    const size_t nwaves = n / 64;
    CHECK(hipMalloc(&d_clk, 8 * 64 * nwaves));
    unsigned long long *d_clk2;
    CHECK(hipMalloc(&d_clk2, 8 * 64 * nwaves));
    ReplayOut rp{};
    rp.vout = d_v;
    rp.psnap = d_v + n;
    rp.peer = d_v + 3 * n;
    const dim3 grid(n / kFramesBS);
    for (int dec = 0; dec < 2; ++dec) {
        CHECK(hipMemset(d_clk, 0, 8 * 64 * nwaves));
        CHECK(hipMemset(d_clk2, 0, 8 * 64 * nwaves));
        for (int rep = 0; rep < STAMP_REPS; ++rep) { // back to back, one synchronise after
            // the last launch stamped with the rotated offsets, the one before with the plain ones
            const bool rot = rep == STAMP_REPS - 1;
            rp.clk = rep == STAMP_REPS - 2 ? d_clk : rot ? d_clk2 : nullptr;
            const uint64_t *io = rot ? d_ioff_r : d_ioff, *oo = rot ? d_ooff_r : d_ooff;
            if (!dec)
                hipLaunchKernelGGL((KFR<false, StampNoBig>), grid, dim3(kFramesBS), STAMP_SHMEM_KB * 1024, 0, n, d_sid, d_nonce,
                                   d_flags, io, d_len, d_pay, oo, d_wire, d_ses, NS, 0xffffffffu, nullptr,
                                   nullptr, rp, StampNoBig{}, d_zs, FrameCtl{});
            else
                hipLaunchKernelGGL((KFR<true, StampNoBig>), grid, dim3(kFramesBS), STAMP_SHMEM_KB * 1024, 0, n, d_sid,
                                   (const uint64_t *) nullptr, (const uint8_t *) nullptr, oo, d_wl, d_wire, io,
                                   d_back, d_ses, NS, 0xffffffffu, d_fl, d_st, rp, StampNoBig{}, d_zs, FrameCtl{});
        }
        CHECK(hipDeviceSynchronize());
        std::vector<unsigned long long> c(64 * nwaves), c2(64 * nwaves);
        CHECK(hipMemcpy(c.data(), d_clk, 8 * 64 * nwaves, hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(c2.data(), d_clk2, 8 * 64 * nwaves, hipMemcpyDeviceToHost));
        {
            // per workgroup: its slowest wave, in the plain launch (A) and the rotated one (B)
            const size_t nb = nwaves / kFramesWaves;
            std::vector<double> A(nb), B(nb);
            size_t same_cu = 0;
            for (size_t b = 0; b < nb; ++b) {
                double a = 0, bb = 0;
                for (uint32_t k = 0; k < kFramesWaves; ++k) {
                    const size_t w = b * kFramesWaves + k;
                    a = std::max(a, (double) (c[64 * w + 61] - c[64 * w]));
                    bb = std::max(bb, (double) (c2[64 * w + 61] - c2[64 * w]));
                }
                A[b] = a, B[b] = bb;
                same_cu += (c[64 * b * kFramesWaves + 62] & 0xffffff00ull) == (c2[64 * b * kFramesWaves + 62] & 0xffffff00ull);
            }
            auto corr = [&](int shift) {
                double ma = 0, mb = 0, sab = 0, saa = 0, sbb = 0;
                for (size_t b = 0; b < nb; ++b)
                    ma += A[(b + shift) % nb] / nb, mb += B[b] / nb;
                for (size_t b = 0; b < nb; ++b) {
                    const double x = A[(b + shift) % nb] - ma, y = B[b] - mb;
                    sab += x * y, saa += x * x, sbb += y * y;
                }
                return sab / sqrt(saa * sbb);
            };
            printf("  workgroups on the same CU in both launches: %zu of %zu; correlation of workgroup times, "
                   "same workgroup index (same CU) %.2f, same data %.2f\n", same_cu, nb, corr(0), corr((int) nb / 2));
        }
        // placement (slot 62: XCC_ID : HW_ID): workgroups per CU, waves per
        // SIMD, and the workgroups' durations by how many shared their CU
        {
            std::vector<unsigned long long> key(nwaves);
            for (size_t w = 0; w < nwaves; ++w) {
                const unsigned long long h = c[64 * w + 62];
                const unsigned hw = (unsigned) h, xcc = (unsigned) (h >> 32) & 0xfu;
                key[w] = ((unsigned long long) xcc << 16) | (((hw >> 13) & 7u) << 8) | (((hw >> 12) & 1u) << 4) |
                         ((hw >> 8) & 0xfu); // XCC, SE, SH, CU
            }
            std::vector<std::pair<unsigned long long, size_t>> cu;
            for (size_t b = 0; b < nwaves / kFramesWaves; ++b)
                cu.push_back({key[b * kFramesWaves], b});
            std::sort(cu.begin(), cu.end());
            std::vector<int> share(nwaves / kFramesWaves, 1);
            size_t ncu = 0;
            for (size_t j = 0; j < cu.size();) {
                size_t k = j;
                while (k < cu.size() && cu[k].first == cu[j].first)
                    ++k;
                for (size_t q = j; q < k; ++q)
                    share[cu[q].second] = (int) (k - j);
                ++ncu;
                j = k;
            }
            double sum[4] = {0}, cnt[4] = {0}, mx[4] = {0};
            for (size_t b = 0; b < nwaves / kFramesWaves; ++b) {
                double d = 0;
                for (uint32_t k = 0; k < kFramesWaves; ++k)
                    d = std::max(d, (double) (c[64 * (b * kFramesWaves + k) + 61] - c[64 * (b * kFramesWaves + k)]));
                const int s = std::min(share[b], 3);
                sum[s] += d, cnt[s] += 1, mx[s] = std::max(mx[s], d);
            }
            printf("  distinct CUs %zu for %zu workgroups; slowest wave of a workgroup by workgroups on its CU:", ncu,
                   nwaves / kFramesWaves);
            for (int s = 1; s < 4; ++s)
                if (cnt[s])
                    printf(" [%d%s: %.0f wg, mean %.0f, max %.0f]", s, s == 3 ? "+" : "", cnt[s], sum[s] / cnt[s], mx[s]);
            printf("\n");
        }
        // per slot: median over waves of (stamp - entry stamp), and of step deltas
        printf("%s: median cycles since entry per phase (min/median/max over waves)\n", dec ? "decode" : "encode");
        // every stamped slot, in order of its median time
        std::vector<std::pair<long long, int>> order;
        for (int sl = 1; sl < 64; ++sl) {
            if (sl == 62)
                continue; // (the wave's placement, not a time)
            std::vector<long long> v;
            for (size_t w = 0; w < nwaves; ++w)
                if (c[64 * w + sl])
                    v.push_back((long long) (c[64 * w + sl] - c[64 * w]));
            if (v.empty())
                continue;
            std::sort(v.begin(), v.end());
            order.push_back({v[v.size() / 2], sl});
        }
        std::sort(order.begin(), order.end());
        std::vector<int> slots;
        for (auto &o : order)
            slots.push_back(o.second);
        for (int sl : slots) {
            std::vector<long long> v;
            for (size_t w = 0; w < nwaves; ++w)
                if (c[64 * w + sl])
                    v.push_back((long long) (c[64 * w + sl] - c[64 * w]));
            if (v.empty())
                continue;
            std::sort(v.begin(), v.end());
            printf("  slot %2d: %8lld %8lld %8lld\n", sl, v.front(), v[v.size() / 2], v.back());
        }
        // wave durations (entry -> slot 61) by workgroup % 8 (the XCD of a
        // round-robin dispatch), by wave in workgroup, and by grid position
        {
            double sx[8] = {0}, nx[8] = {0}, sw[4] = {0}, nwv[4] = {0}, sq[8] = {0}, nq[8] = {0};
            std::vector<long long> all;
            for (size_t w = 0; w < nwaves; ++w) {
                if (!c[64 * w + 61])
                    continue;
                const double d = (double) (c[64 * w + 61] - c[64 * w]);
                const size_t b = w / kFramesWaves;
                sx[b % 8] += d, nx[b % 8] += 1;
                sw[w % kFramesWaves] += d, nwv[w % kFramesWaves] += 1;
                sq[b * 8 / (nwaves / kFramesWaves)] += d, nq[b * 8 / (nwaves / kFramesWaves)] += 1;
                all.push_back((long long) d);
            }
            std::sort(all.begin(), all.end());
            printf("  duration p10/p50/p90/p99/max: %lld %lld %lld %lld %lld\n", all[all.size() / 10],
                   all[all.size() / 2], all[all.size() * 9 / 10], all[all.size() * 99 / 100], all.back());
            printf("  mean by block%%8:");
            for (int k = 0; k < 8; ++k)
                printf(" %.0f", sx[k] / (nx[k] ? nx[k] : 1));
            printf("\n  mean by wave in block:");
            for (uint32_t k = 0; k < kFramesWaves; ++k)
                printf(" %.0f", sw[k] / (nwv[k] ? nwv[k] : 1));
            printf("\n  mean by grid eighth:");
            for (int k = 0; k < 8; ++k)
                printf(" %.0f", sq[k] / (nq[k] ? nq[k] : 1));
            printf("\n");
            // spread of the workgroup means (a CU-wide effect) against the
            // spread inside workgroups (a wave's own)
            double s1 = 0, s2 = 0, w2 = 0, mu = 0;
            size_t nb = nwaves / kFramesWaves;
            std::vector<double> bm(nb, 0.0);
            for (size_t b = 0; b < nb; ++b) {
                for (uint32_t k = 0; k < kFramesWaves; ++k)
                    bm[b] += (double) (c[64 * (b * kFramesWaves + k) + 61] - c[64 * (b * kFramesWaves + k)]);
                bm[b] /= kFramesWaves;
                mu += bm[b] / nb;
            }
            for (size_t b = 0; b < nb; ++b) {
                s1 += (bm[b] - mu) * (bm[b] - mu) / nb;
                for (uint32_t k = 0; k < kFramesWaves; ++k) {
                    const double d = (double) (c[64 * (b * kFramesWaves + k) + 61] - c[64 * (b * kFramesWaves + k)]);
                    w2 += (d - bm[b]) * (d - bm[b]) / (nb * kFramesWaves);
                    s2 += (d - mu) * (d - mu) / (nb * kFramesWaves);
                }
            }
            std::vector<double> sb = bm;
            std::sort(sb.begin(), sb.end());
            printf("  sd all %.0f, sd of workgroup means %.0f, sd within workgroups %.0f; workgroup means p50 %.0f "
                   "p90 %.0f max %.0f\n",
                   sqrt(s2), sqrt(s1), sqrt(w2), sb[nb / 2], sb[nb * 9 / 10], sb.back());
            // per-step time of the slowest and the median waves (slot 5 -> slot 19)
            std::vector<long long> st;
            for (size_t w = 0; w < nwaves; ++w)
                if (c[64 * w + 19] && c[64 * w + 5])
                    st.push_back((long long) (c[64 * w + 19] - c[64 * w + 5]));
            std::sort(st.begin(), st.end());
            if (!st.empty())
                printf("  steps 2..15 per step: p50 %lld p90 %lld max %lld\n", st[st.size() / 2] / 14,
                       st[st.size() * 9 / 10] / 14, st.back() / 14);
            // the slowest tenth of the waves against the middle fifth: per step
            // (2..15) keystream+MAC (slot 3+t -> 24+t) and the rest
            std::vector<std::pair<long long, size_t>> dw;
            for (size_t w = 0; w < nwaves; ++w)
                dw.push_back({(long long) (c[64 * w + 61] - c[64 * w]), w});
            std::sort(dw.begin(), dw.end());
            auto band = [&](size_t lo, size_t hi, const char *name) {
                double ks = 0, rest = 0, pro = 0, epi = 0;
                for (size_t j = lo; j < hi; ++j) {
                    const size_t w = dw[j].second;
                    for (int t = 2; t <= 15; ++t) {
                        ks += (double) (c[64 * w + 24 + t] - c[64 * w + 3 + t]);
                        rest += (double) (c[64 * w + 3 + t + 1] - c[64 * w + 24 + t]);
                    }
                    pro += (double) (c[64 * w + 5] - c[64 * w]);
                    epi += (double) (c[64 * w + 61] - c[64 * w + 18]);
                }
                const double m = (double) (hi - lo);
                printf("  %s: per step keystream+MAC %.0f, rest %.0f; entry->step 2 %.0f; step 15->end %.0f\n", name,
                       ks / m / 14, rest / m / 14, pro / m, epi / m);
            };
            band(nwaves * 2 / 5, nwaves * 3 / 5, "middle fifth ");
            band(nwaves * 9 / 10, nwaves, "slowest tenth");
        }
    }
    return 0;
}
