// Microbenchmarks for the VALU costs that bound the CURVE path on gfx950:
// Salsa20 block rate, Poly1305 field-multiply rate (radix 2^26) and raw
// v_mad_u64_u32 / 32-bit op rates.  Build: hipcc -O3 --offload-arch=gfx950.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>

#include "../libzmq_amd/csrc/curve_device.hpp"

using namespace zmqg;

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void k_salsa(uint32_t *out, int iters)
{
    uint32_t k[8];
    for (int i = 0; i < 8; ++i)
        k[i] = threadIdx.x * 8 + i;
    uint32_t acc = 0;
    for (int it = 0; it < iters; ++it) {
        uint32_t ks[16];
        salsa20_block(ks, k, blockIdx.x, it, it, 0);
        for (int i = 0; i < 16; ++i)
            acc ^= ks[i];
        k[it & 7] ^= acc;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

__global__ void k_fe_mul(uint32_t *out, int iters)
{
    fe r, h0, h1, h2, h3;
    for (int i = 0; i < 5; ++i) {
        r.l[i] = (threadIdx.x * 977 + i * 131) & 0x3ffffff;
        h0.l[i] = (threadIdx.x + i) & 0x3ffffff;
        h1.l[i] = h0.l[i] ^ 1;
        h2.l[i] = h0.l[i] ^ 2;
        h3.l[i] = h0.l[i] ^ 3;
    }
    const uint32_t s1 = r.l[1] * 5, s2 = r.l[2] * 5, s3 = r.l[3] * 5, s4 = r.l[4] * 5;
    for (int it = 0; it < iters; ++it) {
        // four independent chains (ILP), like 4 lanes' worth of Horner
        fe_add_block(h0, it, 1, 2, 3, 1u << 24);
        fe_mul_s(h0, r, s1, s2, s3, s4);
        fe_add_block(h1, it, 1, 2, 3, 1u << 24);
        fe_mul_s(h1, r, s1, s2, s3, s4);
        fe_add_block(h2, it, 1, 2, 3, 1u << 24);
        fe_mul_s(h2, r, s1, s2, s3, s4);
        fe_add_block(h3, it, 1, 2, 3, 1u << 24);
        fe_mul_s(h3, r, s1, s2, s3, s4);
    }
    uint32_t a = 0;
    for (int i = 0; i < 5; ++i)
        a ^= h0.l[i] ^ h1.l[i] ^ h2.l[i] ^ h3.l[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = a;
}

__global__ void k_mad64(uint32_t *out, int iters)
{
    uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = threadIdx.x * 3 + 1, y = blockIdx.x * 5 + 7;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            a0 = (uint64_t) (uint32_t) a1 * y + a0;
            a1 = (uint64_t) (uint32_t) a2 * y + a1;
            a2 = (uint64_t) (uint32_t) a3 * y + a2;
            a3 = (uint64_t) (uint32_t) a4 * y + a3;
            a4 = (uint64_t) (uint32_t) a5 * y + a4;
            a5 = (uint64_t) (uint32_t) a6 * y + a5;
            a6 = (uint64_t) (uint32_t) a7 * y + a6;
            a7 = (uint64_t) (uint32_t) a0 * y + a7;
        }
        y ^= (uint32_t) a0;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t) (a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}

__global__ void k_mul24(uint32_t *out, int iters)
{
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = threadIdx.x * 3 + 1, y = blockIdx.x * 5 + 7;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            a0 = __umul24(a1, y) + a0;
            a1 = __umul24(a2, y) + a1;
            a2 = __umul24(a3, y) + a2;
            a3 = __umul24(a4, y) + a3;
            a4 = __umul24(a5, y) + a4;
            a5 = __umul24(a6, y) + a5;
            a6 = __umul24(a7, y) + a6;
            a7 = __umul24(a0, y) + a7;
        }
        y ^= a0;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void k_mullo32(uint32_t *out, int iters)
{
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = threadIdx.x * 3 + 1, y = blockIdx.x * 5 + 7;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            a0 = a1 * y + a0;
            a1 = a2 * y + a1;
            a2 = a3 * y + a2;
            a3 = a4 * y + a3;
            a4 = a5 * y + a4;
            a5 = a6 * y + a5;
            a6 = a7 * y + a6;
            a7 = a0 * y + a7;
        }
        y ^= a0;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void k_addxor(uint32_t *out, int iters)
{
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t y = blockIdx.x * 5 + 7;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            a0 = rotl32(a0 + y, 7) ^ a1;
            a1 = rotl32(a1 + y, 9) ^ a2;
            a2 = rotl32(a2 + y, 13) ^ a3;
            a3 = rotl32(a3 + y, 18) ^ a4;
            a4 = rotl32(a4 + y, 7) ^ a5;
            a5 = rotl32(a5 + y, 9) ^ a6;
            a6 = rotl32(a6 + y, 13) ^ a7;
            a7 = rotl32(a7 + y, 18) ^ a0;
        }
        y ^= a0;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

template <typename K>
float timeit(K kern, uint32_t *buf, int blocks, int threads, int iters)
{
    hipEvent_t a, b;
    (void) hipEventCreate(&a);
    (void) hipEventCreate(&b);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, buf, 2);
    (void) hipDeviceSynchronize();
    (void) hipEventRecord(a, 0);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, buf, iters);
    (void) hipEventRecord(b, 0);
    (void) hipEventSynchronize(b);
    float ms = 0;
    (void) hipEventElapsedTime(&ms, a, b);
    return ms;
}

int main()
{
    uint32_t *buf;
    const int blocks = 256 * 8, threads = 256;
    CHECK(hipMalloc(&buf, sizeof(uint32_t) * blocks * threads));
    const double lanes = (double) blocks * threads;
    for (int wps = 1; wps <= 8; wps *= 2) { // waves per SIMD
        int it = 200;
        const int b = 256 * wps; // 256-thread blocks: 4 waves = one per SIMD
        float ms = timeit(k_salsa, buf, b, threads, it);
        double blk = (double) b * threads * it;
        printf("salsa20 @%d waves/SIMD: %.3f ms, %.3f G blocks/s = %.1f GB/s keystream\n", wps, ms, blk / ms / 1e6,
               blk * 64 / ms / 1e6);
    }
    {
        int it = 200;
        float ms = timeit(k_fe_mul, buf, blocks, threads, it);
        double m = lanes * it * 4;
        printf("poly add+mul (r26): %.3f ms, %.3f G blocks/s = %.1f GB/s absorbed\n", ms, m / ms / 1e6, m * 16 / ms / 1e6);
    }
    {
        int it = 200;
        float ms = timeit(k_mad64, buf, blocks, threads, it);
        double ops = lanes * it * 64;
        printf("v_mad_u64_u32: %.3f ms, %.2f T lane-ops/s\n", ms, ops / ms / 1e9);
    }
    {
        int it = 200;
        float ms = timeit(k_mul24, buf, blocks, threads, it);
        double ops = lanes * it * 64;
        printf("mul_u24+add: %.3f ms, %.2f T (mul,add) pairs/s\n", ms, ops / ms / 1e9);
    }
    {
        int it = 200;
        float ms = timeit(k_mullo32, buf, blocks, threads, it);
        double ops = lanes * it * 64;
        printf("mul_lo_u32+add: %.3f ms, %.2f T pairs/s\n", ms, ops / ms / 1e9);
    }
    {
        int it = 200;
        float ms = timeit(k_addxor, buf, blocks, threads, it);
        double ops = lanes * it * 64 * 3;
        printf("add+alignbit+xor: %.3f ms, %.2f T lane-ops/s\n", ms, ops / ms / 1e9);
    }
    return 0;
}
