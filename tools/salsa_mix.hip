// Salsa20 instruction-mix experiments on gfx950: the quarter-round step
// b ^= rotl(a + d, k) in different encodings, whole 20-round blocks, cycles
// per block per SIMD at 1, 2, 4 and 8 waves per SIMD (method as in
// tools/valu_rates.hip).  VOP3-encoded ops (v_alignbit_b32, v_bitop3_b32,
// v_lshl_or_b32) issue at about half the rate of VOP2 ops (v_add_u32,
// v_xor_b32, shifts): profiles/valu_rates_r02.md.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/bin/salsa_mix tools/salsa_mix.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__device__ unsigned long long g_clk[2];

__device__ __forceinline__ uint32_t shl(uint32_t x, int k)
{
    uint32_t r;
    asm("v_lshlrev_b32 %0, %1, %2" : "=v"(r) : "i"(k), "v"(x));
    return r;
}
__device__ __forceinline__ uint32_t shr(uint32_t x, int k)
{
    uint32_t r;
    asm("v_lshrrev_b32 %0, %1, %2" : "=v"(r) : "i"(k), "v"(x));
    return r;
}
__device__ __forceinline__ uint32_t xor2(uint32_t x, uint32_t y)
{
    uint32_t r;
    asm("v_xor_b32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
    return r;
}
__device__ __forceinline__ uint32_t or2(uint32_t x, uint32_t y)
{
    uint32_t r;
    asm("v_or_b32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
    return r;
}

// V: 0 alignbit (compiler rotate), 1 VOP2 only (shl, shr, xor, xor),
// 2 bitop3 xor3, 3 lshl_or, 4 VOP2 only with or, 5 half alignbit / half VOP2
template <int V, int Q>
__device__ __forceinline__ uint32_t qstep(uint32_t b, uint32_t t, int k)
{
    constexpr int VV = V == 5 ? ((Q & 1) ? 1 : 0) : V;
    if (VV == 0)
        return b ^ __builtin_rotateleft32(t, k);
    if (VV == 1)
        return xor2(xor2(b, shl(t, k)), shr(t, 32 - k));
    if (VV == 2) {
        uint32_t o;
        asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(o) : "v"(b), "v"(shl(t, k)), "v"(shr(t, 32 - k)));
        return o;
    }
    if (VV == 3) {
        uint32_t o;
        asm("v_lshl_or_b32 %0, %1, %2, %3" : "=v"(o) : "v"(t), "i"(k), "v"(shr(t, 32 - k)));
        return b ^ o;
    }
    return xor2(b, or2(shl(t, k), shr(t, 32 - k)));
}

#define QRV(Q, a, b, c, d)                   \
    b = qstep<V, Q>(b, a + d, 7);            \
    c = qstep<V, Q>(c, b + a, 9);            \
    d = qstep<V, Q>(d, c + b, 13);           \
    a = qstep<V, Q>(a, d + c, 18);

template <int V>
__device__ __forceinline__ void block(uint32_t out[16], const uint32_t k[8], uint32_t n0, uint32_t ctr)
{
    uint32_t x[16] = {0x61707865, k[0], k[1], k[2], k[3], 0x3320646e, n0, 7, ctr, 0, 0x79622d32, k[4], k[5], k[6], k[7],
                      0x6b206574};
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        QRV(0, x[0], x[4], x[8], x[12]);
        QRV(1, x[5], x[9], x[13], x[1]);
        QRV(2, x[10], x[14], x[2], x[6]);
        QRV(3, x[15], x[3], x[7], x[11]);
        QRV(0, x[0], x[1], x[2], x[3]);
        QRV(1, x[5], x[6], x[7], x[4]);
        QRV(2, x[10], x[11], x[8], x[9]);
        QRV(3, x[15], x[12], x[13], x[14]);
    }
#pragma unroll
    for (int i = 0; i < 16; ++i)
        out[i] = x[i] + (i == 8 ? ctr : i == 6 ? n0 : i);
}

template <int V, int NB>
__global__ __launch_bounds__(256) void k_salsa(uint32_t *out, int iters, uint32_t y)
{
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    uint32_t k8[8];
    for (int u = 0; u < 8; ++u)
        k8[u] = threadIdx.x * 8 + u + y;
    uint32_t acc = y;
    for (int it = 0; it < iters; ++it) {
        uint32_t ks[NB][16];
#pragma unroll
        for (int b = 0; b < NB; ++b)
            block<V>(ks[b], k8, acc, it * NB + b);
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

// independent mixes, 16 chains: P VOP2 (add/xor) per VOP3 (alignbit)
template <int P>
__global__ __launch_bounds__(256) void k_mix(uint32_t *out, int iters, uint32_t y)
{
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    uint32_t a[16];
    for (int u = 0; u < 16; ++u)
        a[u] = threadIdx.x * 16 + u + y;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            asm volatile("v_alignbit_b32 %0, %0, %0, 25" : "+v"(a[u]));
#pragma unroll
            for (int p = 0; p < P; ++p)
                asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[(u + 1 + p) & 15]) : "v"(y));
        }
    }
    uint32_t s = 0;
    for (int u = 0; u < 16; ++u)
        s ^= a[u];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        g_clk[0] = __builtin_amdgcn_s_memtime() - t0;
        g_clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
}

typedef void (*KF)(uint32_t *, int, uint32_t);
int main()
{
    uint32_t *buf;
    if (hipMalloc(&buf, sizeof(uint32_t) * 256 * 8 * 256) != hipSuccess)
        return 1;
    int cus = 0;
    (void) hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    struct {
        const char *name;
        KF k;
        double upi; // units per iteration per lane (blocks, or instructions)
        int iters1;
    } ks[] = {
        {"salsa alignbit", k_salsa<0, 1>, 1, 800},     {"salsa vop2 xor-xor", k_salsa<1, 1>, 1, 800},
        {"salsa bitop3", k_salsa<2, 1>, 1, 800},       {"salsa lshl_or", k_salsa<3, 1>, 1, 800},
        {"salsa vop2 or", k_salsa<4, 1>, 1, 800},      {"salsa half/half", k_salsa<5, 1>, 1, 800},
        {"salsa vop2 xor-xor x2", k_salsa<1, 2>, 2, 400}, {"salsa half/half x2", k_salsa<5, 2>, 2, 400},
        {"mix 1 vop2 : 1 vop3", k_mix<1>, 32, 30000},  {"mix 2 vop2 : 1 vop3", k_mix<2>, 48, 20000},
        {"mix 4 vop2 : 1 vop3", k_mix<4>, 80, 12000},
    };
    hipEvent_t a, b;
    (void) hipEventCreate(&a);
    (void) hipEventCreate(&b);
    for (auto &k : ks) {
        for (int wps : {1, 2, 4, 8}) {
            const int blocks = cus * wps;
            const int iters = k.iters1 * 2 / (wps + 1);
            hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, buf, iters / 4 + 1, 3u);
            if (hipDeviceSynchronize() != hipSuccess)
                return 2;
            (void) hipEventRecord(a, 0);
            hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, buf, iters, 3u);
            (void) hipEventRecord(b, 0);
            if (hipEventSynchronize(b) != hipSuccess)
                return 3;
            float ms = 0;
            (void) hipEventElapsedTime(&ms, a, b);
            unsigned long long clk[2];
            (void) hipMemcpyFromSymbol(clk, HIP_SYMBOL(g_clk), sizeof clk);
            const double ghz = (double) clk[0] / (double) clk[1] * 0.1;
            const double units = (double) wps * iters * k.upi;
            printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"clock_ghz\": %.3f, "
                   "\"cycles_per_unit_per_simd\": %.3f}\n",
                   k.name, wps, ms, ghz, ms * 1e6 * ghz / units);
            fflush(stdout);
        }
    }
    return 0;
}
