// Issue order of the Salsa20/20 rounds on gfx950 (round 4): the same 975
// VALU ops per block in different orders (tools/gen_salsa_sched.py), cycles
// per block per SIMD at 1, 2, 3 and 4 waves per SIMD.  The question: does a
// stream that spreads the VOP3 rotates evenly between the VOP2 adds/xors
// issue faster than the compiler's order once two waves share a SIMD
// (profiles/valu_rates_r02.md: an independent 2 VOP2 : 1 VOP3 mix issues at
// ~2.9 cycles per instruction at two waves, the compiler's Salsa20 block at ~4).
// Build: python3 tools/gen_salsa_sched.py tools/bin/salsa_sched_gen.hpp &&
//        python3 tools/gen_salsa_asm.py tools/bin/curve_salsa_asm.hpp &&
//        hipcc -O3 --offload-arch=gfx950 -Itools/bin -o tools/bin/salsa_sched tools/salsa_sched.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "salsa_sched_gen.hpp"
#include "../libzmq_amd/csrc/curve_device.hpp"
#include "curve_salsa_asm.hpp" // tools/gen_salsa_asm.py

__device__ unsigned long long g_clk[2];

#define QR(a, b, c, d)                        \
    b ^= __builtin_rotateleft32(a + d, 7);    \
    c ^= __builtin_rotateleft32(b + a, 9);    \
    d ^= __builtin_rotateleft32(c + b, 13);   \
    a ^= __builtin_rotateleft32(d + c, 18);

__device__ __forceinline__ void rounds_c(uint32_t (&x)[16])
{
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        QR(x[0], x[4], x[8], x[12]);
        QR(x[5], x[9], x[13], x[1]);
        QR(x[10], x[14], x[2], x[6]);
        QR(x[15], x[3], x[7], x[11]);
        QR(x[0], x[1], x[2], x[3]);
        QR(x[5], x[6], x[7], x[4]);
        QR(x[10], x[11], x[8], x[9]);
        QR(x[15], x[12], x[13], x[14]);
    }
}

// V: 0 compiler, 1 clump, 2 skew, 3 serial; B = 2: two blocks (V 0: compiler
// on both, V 2: skew2)
template <int V, int B>
__global__ __launch_bounds__(256) void k_blk(uint32_t *out, int iters, uint32_t y)
{
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    uint32_t x[16], z[16];
    for (int i = 0; i < 16; ++i) {
        x[i] = (threadIdx.x + blockIdx.x * 256) * 0x9e3779b9u + i * 0x85ebca6bu + y;
        z[i] = x[i] ^ 0x5bd1e995u;
    }
    for (int it = 0; it < iters; ++it) {
        uint32_t ix[16], iz[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            ix[i] = x[i];
            iz[i] = z[i];
        }
        if (B == 1) {
            if (V == 0) rounds_c(x);
            else if (V == 1) rounds_clump(x);
            else if (V == 2) rounds_skew(x);
            else rounds_serial(x);
        } else {
            if (V == 0) {
                rounds_c(x);
                rounds_c(z);
            } else {
                rounds_skew2(x, z);
            }
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            x[i] += ix[i];
            if (B == 2) z[i] += iz[i];
        }
    }
    uint32_t *o = out + (size_t) (blockIdx.x * 256 + threadIdx.x) * 32;
    for (int i = 0; i < 16; ++i) {
        o[i] = x[i];
        o[16 + i] = B == 2 ? z[i] : 0;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        g_clk[0] = __builtin_amdgcn_s_memtime() - t0;
        g_clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
}

// The product's pattern: one key and nonce per lane, the block counter
// stepping (curve_device.hpp's salsa20_block, where the compiler hoists the
// counter-free ops, against curve_salsa_asm.hpp's hoisted skewed block).
template <int V>
__global__ __launch_bounds__(256) void k_ctr(uint32_t *out, int iters, uint32_t y)
{
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    uint32_t key[8];
    for (int i = 0; i < 8; ++i)
        key[i] = (threadIdx.x + blockIdx.x * 256) * 0x9e3779b9u + i * 0x85ebca6bu + y;
    const uint32_t n0 = key[3] ^ 0x1234567u, n1 = key[5] + 77u;
    uint32_t acc[16] = {0};
    zmqg::SalsaHoist hs;
    if (V == 1)
        zmqg::salsa20_hoist(hs, key, n0, n1, 0);
    for (int it = 0; it < iters; ++it) {
        uint32_t ks[16];
        if (V == 0)
            zmqg::salsa20_block(ks, key, n0, n1, (uint32_t) it, 0);
        else
            zmqg::salsa20_block_hoisted(ks, hs, key, n0, n1, (uint32_t) it, 0);
#pragma unroll
        for (int i = 0; i < 16; ++i)
            acc[i] ^= ks[i];
    }
    uint32_t *o = out + (size_t) (blockIdx.x * 256 + threadIdx.x) * 32;
    for (int i = 0; i < 16; ++i) {
        o[i] = acc[i];
        o[16 + i] = 0;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        g_clk[0] = __builtin_amdgcn_s_memtime() - t0;
        g_clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
}

typedef void (*KF)(uint32_t *, int, uint32_t);
int main()
{
    int cus = 0;
    (void) hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const size_t words = (size_t) cus * 4 * 256 * 32;
    uint32_t *buf, *ref;
    if (hipMalloc(&buf, words * 4) != hipSuccess || hipMalloc(&ref, words * 4) != hipSuccess)
        return 1;
    struct {
        const char *name;
        KF k;
        int blocks;
    } ks[] = {
        {"compiler x1", k_blk<0, 1>, 1}, {"clump x1", k_blk<1, 1>, 1}, {"skew x1", k_blk<2, 1>, 1},
        {"serial x1", k_blk<3, 1>, 1},   {"compiler x2", k_blk<0, 2>, 2}, {"skew x2", k_blk<2, 2>, 2},
        {"ctr compiler", k_ctr<0>, 1},   {"ctr hoisted skew", k_ctr<1>, 1},
    };
    // parity: 3 iterations of each order equal the compiler's on the same inputs
    uint32_t *h0 = (uint32_t *) malloc(words * 4), *h1 = (uint32_t *) malloc(words * 4);
    for (auto &k : ks) {
        KF refk = k.k == (KF) k_ctr<1> ? (KF) k_ctr<0> : k.blocks == 1 ? (KF) k_blk<0, 1> : (KF) k_blk<0, 2>;
        hipLaunchKernelGGL(refk, dim3(cus), dim3(256), 0, 0, ref, 3, 7u);
        hipLaunchKernelGGL(k.k, dim3(cus), dim3(256), 0, 0, buf, 3, 7u);
        if (hipDeviceSynchronize() != hipSuccess)
            return 2;
        (void) hipMemcpy(h0, ref, (size_t) cus * 256 * 32 * 4, hipMemcpyDeviceToHost);
        (void) hipMemcpy(h1, buf, (size_t) cus * 256 * 32 * 4, hipMemcpyDeviceToHost);
        printf("{\"parity\": \"%s\", \"equal\": %s}\n", k.name,
               memcmp(h0, h1, (size_t) cus * 256 * 32 * 4) == 0 ? "true" : "false");
    }
    hipEvent_t a, b;
    (void) hipEventCreate(&a);
    (void) hipEventCreate(&b);
    for (int rep = 0; rep < 2; ++rep)
        for (auto &k : ks)
            for (int wps : {1, 2, 3, 4}) {
                const int iters = 1600 / k.blocks / wps;
                hipLaunchKernelGGL(k.k, dim3(cus * wps), dim3(256), 0, 0, buf, iters / 4 + 1, 3u);
                if (hipDeviceSynchronize() != hipSuccess)
                    return 3;
                (void) hipEventRecord(a, 0);
                hipLaunchKernelGGL(k.k, dim3(cus * wps), dim3(256), 0, 0, buf, iters, 3u);
                (void) hipEventRecord(b, 0);
                if (hipEventSynchronize(b) != hipSuccess)
                    return 4;
                float ms = 0;
                (void) hipEventElapsedTime(&ms, a, b);
                unsigned long long clk[2];
                (void) hipMemcpyFromSymbol(clk, HIP_SYMBOL(g_clk), sizeof clk);
                const double ghz = (double) clk[0] / (double) clk[1] * 0.1;
                const double blocks = (double) wps * iters * k.blocks;
                printf("{\"order\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"clock_ghz\": %.3f, "
                       "\"cycles_per_block_per_simd\": %.1f, \"cycles_per_instr\": %.3f}\n",
                       k.name, wps, ms, ghz, ms * 1e6 * ghz / blocks, ms * 1e6 * ghz / blocks / 976.0);
                fflush(stdout);
            }
    return 0;
}
