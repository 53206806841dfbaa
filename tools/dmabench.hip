// Throughput of the body kernel's staging path on gfx950: a wave copies
// contiguous 9 KiB tiles (a) with plain global_load_dwordx4 -> global_store,
// (b) through LDS with global_load_lds_dwordx4 (LDS-DMA) -> ds_read_b128 ->
// global_store, (c) as (b) but double-buffered (the next tile's DMA is
// issued before the current tile is stored).  Occupancy = waves per SIMD.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void LdsVoid;
typedef __attribute__((address_space(1))) void GVoid;
constexpr int kG = 9; // granules per lane per tile

__global__ __launch_bounds__(256) void k_plain(const u32x4 *__restrict__ in, u32x4 *__restrict__ out, size_t tiles)
{
    extern __shared__ char pad[];
    const size_t lane = threadIdx.x & 63;
    const size_t wave = (blockIdx.x * (size_t) blockDim.x + threadIdx.x) >> 6;
    const size_t nwaves = (gridDim.x * (size_t) blockDim.x) >> 6;
    for (size_t t = wave; t < tiles; t += nwaves) {
        const size_t g0 = t * 64 * kG;
        u32x4 v[kG];
#pragma unroll
        for (int k = 0; k < kG; ++k)
            v[k] = in[g0 + k * 64 + lane];
#pragma unroll
        for (int k = 0; k < kG; ++k)
            out[g0 + k * 64 + lane] = v[k];
    }
    if (lane == 999)
        pad[0] = 0;
}

__global__ __launch_bounds__(256) void k_lds(const u32x4 *__restrict__ in, u32x4 *__restrict__ out, size_t tiles)
{
    extern __shared__ __attribute__((aligned(16))) char dyn[];
    const size_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    char *buf = dyn + wv * (64 * 16 * kG);
    const size_t wave = (blockIdx.x * (size_t) blockDim.x + threadIdx.x) >> 6;
    const size_t nwaves = (gridDim.x * (size_t) blockDim.x) >> 6;
    for (size_t t = wave; t < tiles; t += nwaves) {
        const size_t g0 = t * 64 * kG;
#pragma unroll
        for (int k = 0; k < kG; ++k)
            __builtin_amdgcn_global_load_lds((GVoid *) (in + g0 + k * 64 + lane), (LdsVoid *) (buf + 1024 * k), 16, 0,
                                             0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int k = 0; k < kG; ++k)
            out[g0 + k * 64 + lane] = *(const u32x4 *) (buf + 1024 * k + 16 * lane);
    }
}

__global__ __launch_bounds__(256) void k_lds2(const u32x4 *__restrict__ in, u32x4 *__restrict__ out, size_t tiles)
{
    extern __shared__ __attribute__((aligned(16))) char dyn[];
    const size_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    char *bufs = dyn + wv * 2 * (64 * 16 * kG);
    const size_t wave = (blockIdx.x * (size_t) blockDim.x + threadIdx.x) >> 6;
    const size_t nwaves = (gridDim.x * (size_t) blockDim.x) >> 6;
    size_t t = wave;
    int b = 0;
    if (t < tiles) {
#pragma unroll
        for (int k = 0; k < kG; ++k)
            __builtin_amdgcn_global_load_lds((GVoid *) (in + t * 64 * kG + k * 64 + lane), (LdsVoid *) (bufs + 1024 * k),
                                             16, 0, 0);
    }
    for (; t < tiles; t += nwaves, b ^= 1) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        char *cb = bufs + b * (64 * 16 * kG), *nb = bufs + (b ^ 1) * (64 * 16 * kG);
        const size_t tn = t + nwaves;
        if (tn < tiles) {
#pragma unroll
            for (int k = 0; k < kG; ++k)
                __builtin_amdgcn_global_load_lds((GVoid *) (in + tn * 64 * kG + k * 64 + lane),
                                                 (LdsVoid *) (nb + 1024 * k), 16, 0, 0);
        }
        const size_t g0 = t * 64 * kG;
#pragma unroll
        for (int k = 0; k < kG; ++k)
            out[g0 + k * 64 + lane] = *(const u32x4 *) (cb + 1024 * k + 16 * lane);
    }
}

template <typename K>
float run(K k, const u32x4 *in, u32x4 *out, size_t tiles, int wgs, size_t lds)
{
    hipEvent_t a, b;
    (void) hipEventCreate(&a);
    (void) hipEventCreate(&b);
    hipLaunchKernelGGL(k, dim3(wgs), dim3(256), lds, 0, in, out, tiles);
    (void) hipDeviceSynchronize();
    float best = 1e9;
    for (int r = 0; r < 5; ++r) {
        (void) hipEventRecord(a, 0);
        hipLaunchKernelGGL(k, dim3(wgs), dim3(256), lds, 0, in, out, tiles);
        (void) hipEventRecord(b, 0);
        (void) hipEventSynchronize(b);
        float ms;
        (void) hipEventElapsedTime(&ms, a, b);
        best = ms < best ? ms : best;
    }
    return best;
}

int main()
{
    const size_t tiles = 8192; // 8192 x 9 KiB = 72 MiB, like one body's input
    const size_t bytes = tiles * 64 * 16 * kG;
    u32x4 *in, *out;
    if (hipMalloc(&in, bytes) != hipSuccess || hipMalloc(&out, bytes) != hipSuccess)
        return 1;
    (void) hipMemset(in, 1, bytes);
    int cus = 256;
    (void) hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    for (int wps = 1; wps <= 4; wps *= 2) {
        const int wgs = cus * wps;
        const size_t lds1 = 4 * 64 * 16 * kG, lds2 = 2 * lds1;
        const float tp = run(k_plain, in, out, tiles, wgs, (160 * 1024) / wps - 1024);
        const float tl = run(k_lds, in, out, tiles, wgs, lds1);
        float t2 = -1;
        if (lds2 * wps <= 160 * 1024)
            t2 = run(k_lds2, in, out, tiles, wgs, lds2);
        printf("%d waves/SIMD: plain %6.1f us %5.0f GB/s | LDS-DMA %6.1f us %5.0f GB/s | LDS-DMA x2 %6.1f us %5.0f GB/s\n",
               wps, tp * 1e3, 2.0 * bytes / tp / 1e6, tl * 1e3, 2.0 * bytes / tl / 1e6, t2 * 1e3,
               t2 > 0 ? 2.0 * bytes / t2 / 1e6 : 0.0);
    }
    return 0;
}
