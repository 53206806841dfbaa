// Unaligned LDS access on gfx950: correctness of ds_read/ds_write b32/b128 at
// byte offsets 0..3 (and 4..15 for b128), and cycles per wave-instruction
// (one wave per SIMD, 16 independent accesses per iteration), aligned vs not.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/bin/lds_ua_rate tools/lds_ua_rate.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ unsigned long long g_clk[2];

__global__ void k_check(uint32_t *out, int sh)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[64 * 96 + 64];
    const int lane = threadIdx.x;
    for (int b = lane; b < 64 * 96 + 64; b += 64)
        lds[b] = (uint8_t) (b * 7 + 3);
    __syncthreads();
    const uint32_t a = lane * 80 + sh;
    uint32_t r32;
    u32x4 v;
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(r32) : "v"(a));
    asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a));
    uint32_t bad = 0, e = 0;
    for (int t = 0; t < 4; ++t)
        e |= (uint32_t) (uint8_t) ((a + t) * 7 + 3) << (8 * t);
    bad += r32 != e;
    const uint32_t r128[4] = {v.x, v.y, v.z, v.w};
    for (int q = 0; q < 4; ++q) {
        uint32_t eq = 0;
        for (int t = 0; t < 4; ++t)
            eq |= (uint32_t) (uint8_t) ((a + 4 * q + t) * 7 + 3) << (8 * t);
        bad += (r128[q] != eq) << 4;
    }
    __syncthreads();
    const uint32_t wa = lane * 80 + sh;
    const uint32_t w32 = 0xa1b2c3d4u ^ lane;
    asm volatile("ds_write_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" ::"v"(wa), "v"(w32) : "memory");
    __syncthreads();
    uint32_t g = 0;
    for (int t = 0; t < 4; ++t)
        g |= (uint32_t) lds[wa + t] << (8 * t);
    bad += (g != w32) << 8;
    bad += (lds[wa + 4] != (uint8_t) ((wa + 4) * 7 + 3)) << 9;
    if (wa > 0)
        bad += (lds[wa - 1] != (uint8_t) ((wa - 1) * 7 + 3)) << 10;
    __syncthreads();
    const u32x4 wv = {0x11111111u * (lane & 15), 0x22222222u ^ lane, 0x33333333u, 0x44444444u};
    const uint32_t wb = lane * 80 + 32 + sh;
    asm volatile("ds_write_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" ::"v"(wb), "v"(wv) : "memory");
    __syncthreads();
    uint32_t got[4];
    for (int q = 0; q < 4; ++q) {
        uint32_t gg = 0;
        for (int t = 0; t < 4; ++t)
            gg |= (uint32_t) lds[wb + 4 * q + t] << (8 * t);
        got[q] = gg;
    }
    bad += ((got[0] != wv.x) + (got[1] != wv.y) + (got[2] != wv.z) + (got[3] != wv.w)) << 12;
    out[lane] = bad;
}

// OP 0 ds_read_b32, 1 ds_read_b128, 2 ds_write_b32, 3 ds_write_b128; address offset off
template <int OP>
__global__ __launch_bounds__(256) void k_rate(uint32_t *out, int iters, int off)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[256 * 160];
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    const uint32_t base = threadIdx.x * 160 + off;
    uint32_t acc = 0;
    u32x4 va = {threadIdx.x, 1, 2, 3};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const uint32_t a = base + 16 * u;
            if (OP == 0) {
                uint32_t r;
                asm volatile("ds_read_b32 %0, %1" : "=v"(r) : "v"(a));
                acc += r;
            } else if (OP == 1) {
                u32x4 r;
                asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"(a));
                acc += r.x ^ r.w;
            } else if (OP == 2) {
                asm volatile("ds_write_b32 %0, %1" ::"v"(a), "v"(acc + u) : "memory");
            } else {
                asm volatile("ds_write_b128 %0, %1" ::"v"(a), "v"(va) : "memory");
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    (void) lds;
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        g_clk[0] = __builtin_amdgcn_s_memtime() - t0;
        g_clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
}

typedef void (*KF)(uint32_t *, int, int);
int main()
{
    uint32_t *d;
    if (hipMalloc(&d, 4 << 20) != hipSuccess)
        return 1;
    for (int sh = 0; sh < 16; ++sh) {
        hipLaunchKernelGGL(k_check, dim3(1), dim3(64), 0, 0, d, sh);
        uint32_t h[64];
        hipError_t e = hipMemcpy(h, d, 256, hipMemcpyDeviceToHost);
        uint32_t tot = 0;
        for (int i = 0; i < 64; ++i)
            tot |= h[i];
        printf("{\"check\": \"offset %d\", \"status\": \"%s\", \"bad_bits\": %u}\n", sh,
               e == hipSuccess ? "ran" : hipGetErrorString(e), tot);
        if (e != hipSuccess)
            return 2;
    }
    int cus = 0;
    (void) hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    struct { const char *n; KF k; } ks[] = {{"ds_read_b32", k_rate<0>}, {"ds_read_b128", k_rate<1>},
                                           {"ds_write_b32", k_rate<2>}, {"ds_write_b128", k_rate<3>}};
    hipEvent_t a, b;
    (void) hipEventCreate(&a);
    (void) hipEventCreate(&b);
    for (auto &k : ks)
        for (int off : {0, 1, 2, 4, 8})
            for (int wps : {1, 2}) {
                const int iters = 20000 / wps;
                hipLaunchKernelGGL(k.k, dim3(cus * wps), dim3(256), 0, 0, d, iters / 4, off);
                if (hipDeviceSynchronize() != hipSuccess)
                    return 3;
                (void) hipEventRecord(a, 0);
                hipLaunchKernelGGL(k.k, dim3(cus * wps), dim3(256), 0, 0, d, iters, off);
                (void) hipEventRecord(b, 0);
                if (hipEventSynchronize(b) != hipSuccess)
                    return 4;
                float ms = 0;
                (void) hipEventElapsedTime(&ms, a, b);
                unsigned long long clk[2];
                (void) hipMemcpyFromSymbol(clk, HIP_SYMBOL(g_clk), sizeof clk);
                const double ghz = (double) clk[0] / (double) clk[1] * 0.1;
                printf("{\"op\": \"%s\", \"offset\": %d, \"waves_per_simd\": %d, \"cycles_per_instr_per_simd\": %.2f}\n",
                       k.n, off, wps, ms * 1e6 * ghz / ((double) wps * iters * 8));
                fflush(stdout);
            }
    return 0;
}
