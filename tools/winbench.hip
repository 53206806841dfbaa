// VALU efficiency of the body kernel's per-window work (Salsa20 block +
// 4 Poly1305 blocks + XOR) versus occupancy, with one or two independent
// windows in flight per lane (ILP).  Data stays in registers; occupancy is
// set with a dynamic LDS allocation.  Build: hipcc -O3 --offload-arch=gfx950.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#include "../libzmq_amd/csrc/curve_device.hpp"

using namespace zmqg;

__global__ __launch_bounds__(256) void k_win1(uint32_t *out, int iters)
{
    extern __shared__ char pad[];
    uint32_t k[8];
    for (int i = 0; i < 8; ++i)
        k[i] = threadIdx.x * 8 + i + blockIdx.x;
    fe r, h = fe_zero();
    for (int i = 0; i < 5; ++i)
        r.l[i] = (threadIdx.x * 977 + i * 131) & 0x3ffffff;
    const uint32_t s1 = r.l[1] * 5, s2 = r.l[2] * 5, s3 = r.l[3] * 5, s4 = r.l[4] * 5;
    uint32_t w[16];
    for (int q = 0; q < 16; ++q)
        w[q] = threadIdx.x ^ q;
    for (int it = 0; it < iters; ++it) {
        uint32_t ks[16];
        salsa20_block(ks, k, 7, 9, it, 0);
        poly_absorb64(h, r, s1, s2, s3, s4, w, 64);
#pragma unroll
        for (int q = 0; q < 16; ++q)
            w[q] ^= ks[q];
    }
    uint32_t a = 0;
    for (int q = 0; q < 16; ++q)
        a ^= w[q];
    for (int i = 0; i < 5; ++i)
        a ^= h.l[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = a;
    if (a == 0x12345678)
        pad[0] = 1;
}

// two independent windows per iteration: blocks ctr and ctr+1, MAC as two
// interleaved Horner chains in r^2 (even / odd blocks)
__global__ __launch_bounds__(256) void k_win2(uint32_t *out, int iters)
{
    extern __shared__ char pad[];
    uint32_t k[8];
    for (int i = 0; i < 8; ++i)
        k[i] = threadIdx.x * 8 + i + blockIdx.x;
    fe r, ha = fe_zero(), hb = fe_zero();
    for (int i = 0; i < 5; ++i)
        r.l[i] = (threadIdx.x * 977 + i * 131) & 0x3ffffff;
    const uint32_t s1 = r.l[1] * 5, s2 = r.l[2] * 5, s3 = r.l[3] * 5, s4 = r.l[4] * 5;
    uint32_t wa[16], wb[16];
    for (int q = 0; q < 16; ++q) {
        wa[q] = threadIdx.x ^ q;
        wb[q] = threadIdx.x ^ (q * 3);
    }
    for (int it = 0; it < iters; it += 2) {
        uint32_t ka[16], kb[16];
        salsa20_block(ka, k, 7, 9, it, 0);
        salsa20_block(kb, k, 7, 9, it + 1, 0);
        poly_absorb64(ha, r, s1, s2, s3, s4, wa, 64);
        poly_absorb64(hb, r, s1, s2, s3, s4, wb, 64);
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            wa[q] ^= ka[q];
            wb[q] ^= kb[q];
        }
    }
    uint32_t a = 0;
    for (int q = 0; q < 16; ++q)
        a ^= wa[q] ^ wb[q];
    for (int i = 0; i < 5; ++i)
        a ^= ha.l[i] ^ hb.l[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = a;
    if (a == 0x12345678)
        pad[0] = 1;
}

__global__ __launch_bounds__(256) void k_salsa_only(uint32_t *out, int iters)
{
    extern __shared__ char pad[];
    uint32_t k[8];
    for (int i = 0; i < 8; ++i)
        k[i] = threadIdx.x * 8 + i + blockIdx.x;
    uint32_t w[16];
    for (int q = 0; q < 16; ++q)
        w[q] = threadIdx.x ^ q;
    for (int it = 0; it < iters; ++it) {
        uint32_t ks[16];
        salsa20_block(ks, k, 7, 9, it, 0);
#pragma unroll
        for (int q = 0; q < 16; ++q)
            w[q] ^= ks[q];
    }
    uint32_t a = 0;
    for (int q = 0; q < 16; ++q)
        a ^= w[q];
    out[blockIdx.x * blockDim.x + threadIdx.x] = a;
    if (a == 0x12345678)
        pad[0] = 1;
}

__global__ __launch_bounds__(256) void k_poly_only(uint32_t *out, int iters)
{
    extern __shared__ char pad[];
    fe r, h = fe_zero();
    for (int i = 0; i < 5; ++i)
        r.l[i] = (threadIdx.x * 977 + i * 131) & 0x3ffffff;
    const uint32_t s1 = r.l[1] * 5, s2 = r.l[2] * 5, s3 = r.l[3] * 5, s4 = r.l[4] * 5;
    uint32_t w[16];
    for (int q = 0; q < 16; ++q)
        w[q] = threadIdx.x ^ q;
    for (int it = 0; it < iters; ++it) {
        poly_absorb64(h, r, s1, s2, s3, s4, w, 64);
        w[it & 15] ^= h.l[0];
    }
    uint32_t a = 0;
    for (int i = 0; i < 5; ++i)
        a ^= h.l[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = a;
    if (a == 0x12345678)
        pad[0] = 1;
}

template <typename K>
float timeit(K kern, uint32_t *buf, int blocks, size_t lds, int iters)
{
    hipEvent_t a, b;
    (void) hipEventCreate(&a);
    (void) hipEventCreate(&b);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), lds, 0, buf, 4);
    (void) hipDeviceSynchronize();
    (void) hipEventRecord(a, 0);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), lds, 0, buf, iters);
    (void) hipEventRecord(b, 0);
    (void) hipEventSynchronize(b);
    float ms = 0;
    (void) hipEventElapsedTime(&ms, a, b);
    return ms;
}

int main()
{
    uint32_t *buf;
    if (hipMalloc(&buf, sizeof(uint32_t) * 256 * 256 * 8) != hipSuccess)
        return 1;
    int cus = 256;
    (void) hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int iters = 256;
    const char *names[] = {"window x1", "window x2 (ILP)", "salsa only", "poly only (4 blocks)"};
    for (int kind = 0; kind < 4; ++kind) {
        for (int wps = 1; wps <= 8; wps *= 2) { // waves per SIMD: one 256-thread block per SIMD set
            const int blocks = cus * wps;
            const size_t lds = (160 * 1024) / wps - 1024; // at most wps blocks per CU
            float ms = kind == 0 ? timeit(k_win1, buf, blocks, lds, iters)
                     : kind == 1 ? timeit(k_win2, buf, blocks, lds, iters)
                     : kind == 2 ? timeit(k_salsa_only, buf, blocks, lds, iters)
                                 : timeit(k_poly_only, buf, blocks, lds, iters);
            const double wave_windows = (double) blocks * 4 * iters; // per-wave windows
            const double per_simd = wave_windows / (cus * 4);
            printf("%-22s %d waves/SIMD: %.3f ms, %.1f ns per wave-window per SIMD, %.2f G windows/s\n", names[kind],
                   wps, ms, ms * 1e6 / per_simd, wave_windows * 64 / ms / 1e6);
        }
    }
    return 0;
}
