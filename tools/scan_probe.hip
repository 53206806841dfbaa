// scan_probe.hip -- the read floor under k_zmtp_scan:
// a 69.9 MB buffer (the config-2 framed stream's size) read with the scan's
// grid (one 256-thread workgroup per 16 KiB) by
//   plain    one 16-byte load per chunk, 4 chunk rounds per thread;
//   scan3    the scan's three loads per chunk (16 bytes before, the chunk,
//            8 bytes after);
//   wide     a persistent grid, 4 x CUs workgroups, looping over the buffer;
//   zscan    the library's k_zmtp_scan on a config-2-like stream (1,066-byte
//            LARGE frames of random bytes);
//   zscanpX  k_zmtp_scan_p, the persistent form, X x CUs workgroups;
//   vzV      variants of the signature tests (vz_scan_tile below), checked
//            candidate for candidate against zscan;
// each timed with hip events over 20 back-to-back launches (the buffer stays
// MALL-resident between them) and after a 1 GB sweep (HBM-fed).
//   hipcc -O3 --offload-arch=gfx950 -o tools/bin/scan_probe tools/scan_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <vector>

#include "../libzmq_amd/csrc/curve_frames.hpp"
#include "../libzmq_amd/csrc/curve_zmtp.hpp"

#define CK(x)                                                                                                    \
    do {                                                                                                         \
        hipError_t e_ = (x);                                                                                     \
        if (e_ != hipSuccess) {                                                                                  \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                                              \
            return 1;                                                                                            \
        }                                                                                                        \
    } while (0)

constexpr uint32_t kT = 256, kWg = 16384;

__global__ __launch_bounds__(kT) void k_plain(const uint8_t *b, uint64_t n, uint32_t *out)
{
    const uint64_t wg0 = (uint64_t) blockIdx.x * kWg;
    uint32_t x = 0;
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
        const uint64_t base = wg0 + 16ull * (k * kT + threadIdx.x);
        if (base + 16 <= n) {
            const uint4 v = *(const uint4 *) (b + base);
            x ^= v.x ^ v.y ^ v.z ^ v.w;
        }
    }
    if (x == 0x07070707u)
        out[blockIdx.x] = x;
}

__global__ __launch_bounds__(kT) void k_scan3(const uint8_t *b, uint64_t n, uint32_t *out)
{
    const uint64_t wg0 = (uint64_t) blockIdx.x * kWg;
    uint32_t x = 0;
    uint4 v0[4], v1[4];
    uint2 v2[4];
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
        const uint64_t base = wg0 + 16ull * (k * kT + threadIdx.x);
        const bool in = base >= 16 && base + 24 <= n;
        v0[k] = in ? *(const uint4 *) (b + base - 16) : uint4{0, 0, 0, 0};
        v1[k] = in ? *(const uint4 *) (b + base) : uint4{0, 0, 0, 0};
        v2[k] = in ? *(const uint2 *) (b + base + 16) : uint2{0, 0};
    }
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k)
        x ^= v0[k].x ^ v0[k].w ^ v1[k].x ^ v1[k].y ^ v1[k].z ^ v1[k].w ^ v2[k].x ^ v2[k].y;
    if (x == 0x07070707u)
        out[blockIdx.x] = x;
}

__global__ __launch_bounds__(kT) void k_wide(const uint8_t *b, uint64_t n, uint32_t *out)
{
    uint32_t x = 0;
    const uint64_t stride = (uint64_t) gridDim.x * kT * 16u;
    for (uint64_t p = ((uint64_t) blockIdx.x * kT + threadIdx.x) * 16u; p + 64u * stride / 16u <= n;) {
        uint4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
            v[k] = *(const uint4 *) (b + p + (uint64_t) k * stride);
#pragma unroll
        for (int k = 0; k < 4; ++k)
            x ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
        p += 4 * stride;
    }
    if (x == 0x07070707u)
        out[blockIdx.x] = x;
}

__global__ void k_sweep(uint4 *p, uint64_t n16)
{
    for (uint64_t i = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t) gridDim.x * blockDim.x)
        p[i] = uint4{(uint32_t) i, 1, 2, 3};
}

__global__ void k_fill_frames(uint8_t *b, uint64_t n)
{
    for (uint64_t i = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t) gridDim.x * blockDim.x) {
        const uint64_t f = i % 1066u;
        uint32_t x = (uint32_t) (i * 0x9E3779B1u);
        x ^= x >> 15;
        x *= 0x85EBCA77u;
        x ^= x >> 13;
        uint8_t v = (uint8_t) x;
        static const uint8_t hdr[17] = {2, 0, 0, 0, 0, 0, 0, 4, 33, 7, 'M', 'E', 'S', 'S', 'A', 'G', 'E'};
        if (f < 17)
            v = hdr[f];
        b[i] = v;
    }
}

// Variants of zmtp_scan_tile's signature tests, for
// timing against the library's: V = 1 one first-word compare per position
// and no per-word 0x07 filter; V = 2 the library's filter without the
// per-position bound (bytes past n load as zero and cannot match
// "\x07MESSAGE"); V = 3 = V1 with the header's size taken by byte swaps.
template <int O, int NW>
__device__ __forceinline__ uint32_t vz_word(const uint32_t (&w)[NW])
{ // bytes [O, O + 4) of the window, little-endian
    if constexpr (O % 4 == 0)
        return w[O / 4];
    else
        return __builtin_amdgcn_alignbyte(w[O / 4 + 1], w[O / 4], O % 4);
}
template <int O, int NW>
__device__ __forceinline__ uint64_t vz_cand_fast(const uint32_t (&w)[NW], uint64_t qq, uint64_t n, int64_t max_msg)
{
    if (qq >= 9 && (zmqg::zmtp_byte<O - 9>(w) & zmqg::kZmtpLarge)) {
        const uint64_t size = ((uint64_t) __builtin_bswap32(vz_word<O - 8>(w)) << 32) | __builtin_bswap32(vz_word<O - 4>(w));
        const uint64_t p = qq - 9;
        if (zmqg::zmtp_size_ok(size, max_msg) && size >= 8 && size <= n - p - 9)
            return p;
    }
    if (qq >= 2 && !(zmqg::zmtp_byte<O - 2>(w) & zmqg::kZmtpLarge)) {
        const uint64_t size = zmqg::zmtp_byte<O - 1>(w), p = qq - 2;
        if (zmqg::zmtp_size_ok(size, max_msg) && size >= 8 && size <= n - p - 2)
            return p;
    }
    return zmqg::kZmtpNone;
}

template <int V>
__device__ __forceinline__ void vz_scan_tile(uint64_t n, int64_t max_msg, uint64_t tile,
                                             const uint32_t (&w)[zmqg::kZmtpRounds][10], uint64_t *cand_wg,
                                             uint64_t *count_wg, uint16_t *count16)
{
    using namespace zmqg;
    constexpr uint32_t R = kZmtpRounds;
    const uint64_t wg0 = tile * kZmtpWgBytes;
    uint64_t *const dst0 = cand_wg + (size_t) tile * kZmtpWgCap;
    uint64_t f[R][2];
    uint32_t cnt[R];
#pragma unroll
    for (uint32_t k = 0; k < R; ++k) {
        const uint64_t base = wg0 + 16ull * (k * kZmtpThreads + threadIdx.x);
        uint64_t f0 = 0, f1 = 0;
        uint32_t c = 0;
        auto at = [&](uint64_t p) {
            if (p != kZmtpNone && c < 2u) {
                f1 = c ? p : f1;
                f0 = c ? f0 : p;
                ++c;
            }
        };
        const uint32_t(&wk)[10] = w[k];
#define VZ_CAND(O, q) (V == 3 ? vz_cand_fast<O>(wk, q, n, max_msg) : zmtp_cand_at<O>(wk, q, n, max_msg))
#define VZ_SIG1(Q, J)                                                                                            \
    if (__builtin_amdgcn_alignbyte(wk[5 + Q], wk[4 + Q], J) == 0x53454d07u)                                      \
        if (__builtin_amdgcn_alignbyte(wk[6 + Q], wk[5 + Q], J) == 0x45474153u)                                  \
            at(VZ_CAND(16 + 4 * Q + J, base + 4 * Q + J));
#define VZ_SIG2(Q, J)                                                                                            \
    if (__builtin_amdgcn_alignbyte(wk[5 + Q], wk[4 + Q], J) == 0x53454d07u &&                                    \
        __builtin_amdgcn_alignbyte(wk[6 + Q], wk[5 + Q], J) == 0x45474153u)                                      \
        at(zmtp_cand_at<16 + 4 * Q + J>(wk, base + 4 * Q + J, n, max_msg));
#define VZ_WORD(Q)                                                                                               \
    if constexpr (V == 2) {                                                                                      \
        const uint32_t x = wk[4 + Q] ^ 0x07070707u;                                                              \
        if ((x - 0x01010101u) & ~x & 0x80808080u) {                                                              \
            VZ_SIG2(Q, 0)                                                                                        \
            VZ_SIG2(Q, 1)                                                                                        \
            VZ_SIG2(Q, 2)                                                                                        \
            VZ_SIG2(Q, 3)                                                                                        \
        }                                                                                                        \
    } else {                                                                                                     \
        VZ_SIG1(Q, 0)                                                                                            \
        VZ_SIG1(Q, 1)                                                                                            \
        VZ_SIG1(Q, 2)                                                                                            \
        VZ_SIG1(Q, 3)                                                                                            \
    }
        VZ_WORD(0)
        VZ_WORD(1)
        VZ_WORD(2)
        VZ_WORD(3)
#undef VZ_WORD
#undef VZ_SIG1
#undef VZ_SIG2
#undef VZ_CAND
        f[k][0] = f0;
        f[k][1] = f1;
        cnt[k] = c;
    }
    uint64_t packed = 0;
#pragma unroll
    for (uint32_t k = 0; k < R; ++k)
        packed |= (uint64_t) cnt[k] << (16 * k);
    uint64_t tot;
    const uint64_t ex = zmtp_block_excl4(packed, tot);
    uint32_t base_out = 0;
#pragma unroll
    for (uint32_t k = 0; k < R; ++k) {
        const uint32_t off = base_out + (uint32_t) ((ex >> (16 * k)) & 0xffffu);
        if (cnt[k] > 0u)
            dst0[off] = f[k][0];
        if (cnt[k] > 1u)
            dst0[off + 1] = f[k][1];
        base_out += (uint32_t) ((tot >> (16 * k)) & 0xffffu);
    }
    if (threadIdx.x == 0) {
        count_wg[tile] = base_out;
        count16[tile] = (uint16_t) base_out;
    }
}

template <int V>
__global__ __launch_bounds__(zmqg::kZmtpThreads) void k_vz_scan(const uint8_t *b, uint64_t n, int64_t max_msg,
                                                                uint64_t *cand_wg, uint64_t *count_wg,
                                                                uint16_t *count16)
{
    uint32_t w[zmqg::kZmtpRounds][10];
    zmqg::zmtp_scan_load(b, n, blockIdx.x, w);
    vz_scan_tile<V>(n, max_msg, blockIdx.x, w, cand_wg, count_wg, count16);
}

int main()
{
    const uint64_t n = 65536ull * 1066ull;
    const uint32_t g = (uint32_t) ((n + kWg - 1) / kWg);
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    uint8_t *b = nullptr, *big = nullptr;
    uint32_t *out = nullptr;
    CK(hipMalloc(&b, n + 64));
    CK(hipMalloc(&big, 1ull << 30));
    CK(hipMalloc(&out, 4u * g));
    hipLaunchKernelGGL(k_sweep, dim3(4096), dim3(256), 0, 0, (uint4 *) b, (n + 64) / 16);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    uint64_t *cand_wg = nullptr, *count_wg = nullptr, *count_ref = nullptr, *cand_ref = nullptr;
    uint16_t *count16 = nullptr;
    CK(hipMalloc(&cand_wg, 8ull * g * zmqg::kZmtpWgCap));
    CK(hipMalloc(&count_wg, 8ull * (g + 1)));
    CK(hipMalloc(&cand_ref, 8ull * g * zmqg::kZmtpWgCap));
    CK(hipMalloc(&count_ref, 8ull * (g + 1)));
    CK(hipMalloc(&count16, 2ull * (g + 8)));
    for (int mode = 0; mode < 2; ++mode) {
        for (int kind = 0; kind < 10; ++kind) {
            if (kind == 3) { // the frame stream for the library's scans
                hipLaunchKernelGGL(k_fill_frames, dim3(4096), dim3(256), 0, 0, b, n);
                hipLaunchKernelGGL(zmqg::k_zmtp_scan, dim3(g), dim3(kT), 0, 0, b, n, (int64_t) -1, cand_ref, count_ref,
                                   count16);
                CK(hipDeviceSynchronize());
            }
            float best = 1e9f, sum = 0.f;
            const int reps = 20;
            for (int r = 0; r < reps; ++r) {
                if (mode == 1) // evict: a 1 GB sweep between launches
                    hipLaunchKernelGGL(k_sweep, dim3(4096), dim3(256), 0, 0, (uint4 *) big, (1ull << 30) / 16);
                CK(hipEventRecord(e0, 0));
                if (kind == 0)
                    hipLaunchKernelGGL(k_plain, dim3(g), dim3(kT), 0, 0, b, n, out);
                else if (kind == 1)
                    hipLaunchKernelGGL(k_scan3, dim3(g), dim3(kT), 0, 0, b, n, out);
                else if (kind == 2)
                    hipLaunchKernelGGL(k_wide, dim3(4 * cus), dim3(kT), 0, 0, b, n, out);
                else if (kind == 3)
                    hipLaunchKernelGGL(zmqg::k_zmtp_scan, dim3(g), dim3(kT), 0, 0, b, n, (int64_t) -1, cand_wg,
                                       count_wg, count16);
                else if (kind == 7)
                    hipLaunchKernelGGL(k_vz_scan<1>, dim3(g), dim3(kT), 0, 0, b, n, (int64_t) -1, cand_wg, count_wg,
                                       count16);
                else if (kind == 8)
                    hipLaunchKernelGGL(k_vz_scan<2>, dim3(g), dim3(kT), 0, 0, b, n, (int64_t) -1, cand_wg, count_wg,
                                       count16);
                else if (kind == 9)
                    hipLaunchKernelGGL(k_vz_scan<3>, dim3(g), dim3(kT), 0, 0, b, n, (int64_t) -1, cand_wg, count_wg,
                                       count16);
                else
                    hipLaunchKernelGGL(zmqg::k_zmtp_scan_p, dim3((kind == 4 ? 2 : kind == 5 ? 4 : 6) * cus), dim3(kT), 0,
                                       0, b, n, (int64_t) -1, (uint64_t) g, cand_wg, count_wg, count16);
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms = 0.f;
                CK(hipEventElapsedTime(&ms, e0, e1));
                best = ms < best ? ms : best;
                sum += ms;
            }
            if (kind >= 3) { // the same candidate counts as the reference launch
                std::vector<uint64_t> h1(g), h2(g);
                CK(hipMemcpy(h1.data(), count_ref, 8ull * g, hipMemcpyDeviceToHost));
                CK(hipMemcpy(h2.data(), count_wg, 8ull * g, hipMemcpyDeviceToHost));
                uint64_t tot = 0;
                for (uint32_t i = 0; i < g; ++i)
                    tot += h1[i];
                if (memcmp(h1.data(), h2.data(), 8ull * g) != 0 || tot < 65536) {
                    fprintf(stderr, "kind %d: counts differ (total %llu)\n", kind, (unsigned long long) tot);
                    return 1;
                }
                if (kind >= 7) { // and the same candidates
                    std::vector<uint64_t> c1((size_t) g * zmqg::kZmtpWgCap), c2((size_t) g * zmqg::kZmtpWgCap);
                    CK(hipMemcpy(c1.data(), cand_ref, 8ull * c1.size(), hipMemcpyDeviceToHost));
                    CK(hipMemcpy(c2.data(), cand_wg, 8ull * c2.size(), hipMemcpyDeviceToHost));
                    for (uint32_t i = 0; i < g; ++i)
                        if (memcmp(&c1[(size_t) i * zmqg::kZmtpWgCap], &c2[(size_t) i * zmqg::kZmtpWgCap], 8ull * h1[i])) {
                            fprintf(stderr, "kind %d: candidates differ in tile %u\n", kind, i);
                            return 1;
                        }
                }
            }
            static const char *names[] = {"plain", "scan3", "wide", "zscan", "zscanp2", "zscanp4", "zscanp6", "vz1", "vz2", "vz3"};
            printf("%-6s %-9s best %7.1f us  mean %7.1f us  %6.2f TB/s (best)\n", names[kind],
                   mode ? "hbm-fed" : "resident", best * 1e3, sum / reps * 1e3, n / (best * 1e-3) / 1e12);
        }
    }
    return 0;
}
