// VALU issue rate vs waves per SIMD on gfx950, kernels long enough (>1 ms)
// to reach steady clocks.  Reports cycles per wave-instruction per SIMD at
// 2.4 GHz and the in-kernel clock (s_memtime / s_memrealtime).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include "../libzmq_amd/csrc/curve_device.hpp"
using namespace zmqg;

__device__ unsigned long long g_clk[2];

template <int OP>
__global__ __launch_bounds__(256) void k_op(uint32_t *out, int iters, uint32_t y)
{
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    uint32_t a[16];
    for (int u = 0; u < 16; ++u) a[u] = threadIdx.x * 16 + u;
    for (int it = 0; it < iters; ++it) {
        if (OP == 0) { // VOP2 add
#pragma unroll
            for (int u = 0; u < 16; ++u) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[u]) : "v"(y));
        } else if (OP == 1) { // VOP2 xor
#pragma unroll
            for (int u = 0; u < 16; ++u) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[u]) : "v"(y));
        } else if (OP == 2) { // VOP3 alignbit
#pragma unroll
            for (int u = 0; u < 16; ++u) asm volatile("v_alignbit_b32 %0, %0, %0, 25" : "+v"(a[u]));
        } else if (OP == 3) { // VOP3 add (e64 encoding)
#pragma unroll
            for (int u = 0; u < 16; ++u) asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(a[u]) : "v"(y));
        } else if (OP == 4) { // mad64
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                uint64_t t = ((uint64_t) a[2 * u + 1] << 32) | a[2 * u];
                asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %1, %0" : "+v"(t) : "v"(y) : "s0", "s1");
                a[2 * u] = (uint32_t) t; a[2 * u + 1] = (uint32_t) (t >> 32);
            }
        } else if (OP == 5) { // salsa20 blocks (4 independent quarter-round chains)
            uint32_t k8[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) k8[u] = a[u];
            uint32_t ks[16];
            salsa20_block(ks, k8, a[8], a[9], it, 0);
#pragma unroll
            for (int u = 0; u < 16; ++u) a[u] ^= ks[u];
        } else if (OP == 6) { // VOP2 lshlrev
#pragma unroll
            for (int u = 0; u < 16; ++u) asm volatile("v_lshlrev_b32 %0, 3, %0" : "+v"(a[u]));
        } else if (OP == 7) { // v_perm_b32 (VOP3)
#pragma unroll
            for (int u = 0; u < 16; ++u) asm volatile("v_perm_b32 %0, %0, %1, %1" : "+v"(a[u]) : "v"(y));
        }
    }
    uint32_t s = 0;
    for (int u = 0; u < 16; ++u) s ^= a[u];
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
    hipMalloc(&buf, sizeof(uint32_t) * 256 * 16 * 256);
    struct { const char *name; KF k; double ipi; } ks[] = {
        {"v_add_u32 (VOP2)", k_op<0>, 16}, {"v_xor_b32 (VOP2)", k_op<1>, 16}, {"v_alignbit_b32", k_op<2>, 16},
        {"v_add_u32_e64 (VOP3)", k_op<3>, 16}, {"v_mad_u64_u32", k_op<4>, 8}, {"salsa20 block", k_op<5>, 1},
        {"v_lshlrev_b32 (VOP2)", k_op<6>, 16}, {"v_perm_b32", k_op<7>, 16}};
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (auto &k : ks) {
        for (int wps : {1, 2, 4, 8}) {
            const int blocks = 256 * wps;
            const int iters = (k.ipi == 1 ? 400 : 40000) / wps;
            hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, buf, iters, 3u);
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
            const double winstr = (double) wps * iters * k.ipi; // per SIMD (per-unit instrs)
            const double cyc = ms * 1e6 * ghz / winstr;
            printf("%-22s %d w/SIMD: %.3f ms  clk %.2f GHz  %.2f cyc per unit per SIMD\n", k.name, wps, ms, ghz, cyc);
        }
    }
    return 0;
}
