// Salsa20-shaped instruction mixes on gfx950: cycles per quarter-round step
// (t = a + b; x ^= rotl(t, k)) for different rotate encodings, and whole
// Salsa20 blocks one or two per lane.  8 waves per SIMD, >1 ms kernels.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include "../libzmq_amd/csrc/curve_device.hpp"
using namespace zmqg;

__device__ unsigned long long g_clk[2];

template <int V>
__device__ __forceinline__ uint32_t step(uint32_t x, uint32_t a, uint32_t b)
{
    uint32_t t = a + b, r;
    if (V == 0) { // alignbit rotate
        r = __builtin_amdgcn_alignbit(t, t, 25);
        return x ^ r;
    } else if (V == 1) { // shl + shr + xor3 via bitop3
        uint32_t hi = t << 7, lo = t >> 25, o;
        asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(o) : "v"(x), "v"(hi), "v"(lo));
        return o;
    } else if (V == 2) { // lshl_or rotate
        uint32_t lo = t >> 25, o;
        asm volatile("v_lshl_or_b32 %0, %1, 7, %2" : "=v"(o) : "v"(t), "v"(lo));
        return x ^ o;
    } else { // 64-bit shift of (t:t)
        uint64_t p = ((uint64_t) t << 32) | t;
        p <<= 7;
        return x ^ (uint32_t) (p >> 32);
    }
}

template <int V>
__global__ __launch_bounds__(256) void k_mix(uint32_t *out, int iters, uint32_t y)
{
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    uint32_t s[16];
    for (int u = 0; u < 16; ++u) s[u] = threadIdx.x * 16 + u + y;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int u = 0; u < 16; ++u) // 16 independent chains, 4 steps each
            s[u] = step<V>(s[u], s[(u + 1) & 15], s[(u + 5) & 15]);
#pragma unroll
        for (int u = 0; u < 16; ++u)
            s[u] = step<V>(s[u], s[(u + 3) & 15], s[(u + 7) & 15]);
    }
    uint32_t a = 0;
    for (int u = 0; u < 16; ++u) a ^= s[u];
    out[blockIdx.x * blockDim.x + threadIdx.x] = a;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        g_clk[0] = __builtin_amdgcn_s_memtime() - t0;
        g_clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
}

template <int NB>
__global__ __launch_bounds__(256) void k_salsa(uint32_t *out, int iters, uint32_t y)
{
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    uint32_t k8[8];
    for (int u = 0; u < 8; ++u) k8[u] = threadIdx.x * 8 + u + y;
    uint32_t acc = 0;
    for (int it = 0; it < iters; ++it) {
        uint32_t ks[NB][16];
#pragma unroll
        for (int b = 0; b < NB; ++b)
            salsa20_block(ks[b], k8, acc, it, b, 0);
#pragma unroll
        for (int b = 0; b < NB; ++b)
#pragma unroll
            for (int u = 0; u < 16; ++u)
                acc ^= ks[b][u];
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        g_clk[0] = __builtin_amdgcn_s_memtime() - t0;
        g_clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
}

typedef void (*KF)(uint32_t *, int, uint32_t);
int main()
{
    uint32_t *buf;
    hipMalloc(&buf, sizeof(uint32_t) * 256 * 16 * 256);
    struct { const char *name; KF k; double units_per_iter; int iters; } ks[] = {
        {"step alignbit", k_mix<0>, 32, 4000}, {"step bitop3", k_mix<1>, 32, 4000},
        {"step lshl_or", k_mix<2>, 32, 4000},   {"step shl64", k_mix<3>, 32, 4000},
        {"salsa x1", k_salsa<1>, 1, 200},       {"salsa x2", k_salsa<2>, 2, 100}};
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (auto &k : ks) {
        const int wps = 8, blocks = 256 * wps, iters = k.iters;
        hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, buf, iters / 10, 3u);
        hipDeviceSynchronize();
        hipEventRecord(a, 0);
        hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, buf, iters, 3u);
        hipEventRecord(b, 0);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        unsigned long long clk[2];
        hipMemcpyFromSymbol(clk, HIP_SYMBOL(g_clk), sizeof clk);
        const double ghz = (double) clk[0] / (double) clk[1] * 0.1;
        const double units = (double) wps * iters * k.units_per_iter; // per SIMD
        printf("%-16s %.3f ms  clk %.2f GHz  %.1f cyc per unit per SIMD\n", k.name, ms, ghz, ms * 1e6 * ghz / units);
    }
    return 0;
}
