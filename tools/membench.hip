// Memory-pattern microbenchmark for the CURVE body kernels on gfx950:
// how fast can a wave move 256-byte per-lane chunks (lane = chunk) versus a
// fully coalesced stream, at different occupancies?
//   P1 coalesced copy: lane i moves granules i, i+64, ... of the wave's 16 KiB
//   P2 lane-chunk copy: lane i moves its own 256-byte chunk (16 granules)
//   P3 lane-chunk copy, all 16 loads issued before any store
//   occupancy is set with a dynamic LDS allocation per workgroup.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ void p1_coalesced(const u32x4 *__restrict__ in, u32x4 *__restrict__ out, size_t chunks)
{
    extern __shared__ char pad[];
    const size_t lane = threadIdx.x & 63;
    const size_t wave = (blockIdx.x * (size_t) blockDim.x + threadIdx.x) >> 6;
    const size_t nwaves = (gridDim.x * (size_t) blockDim.x) >> 6;
    for (size_t w = wave; w * 64 < chunks; w += nwaves) {
        const size_t g0 = w * 64 * 16; // granule base of the wave's 64 chunks
        u32x4 v[16];
#pragma unroll
        for (int k = 0; k < 16; ++k)
            v[k] = in[g0 + k * 64 + lane];
#pragma unroll
        for (int k = 0; k < 16; ++k)
            out[g0 + k * 64 + lane] = v[k] ^ (u32x4){1, 2, 3, 4};
    }
    if (lane == 999)
        pad[0] = 0;
}

__global__ void p2_lanechunk(const u32x4 *__restrict__ in, u32x4 *__restrict__ out, size_t chunks)
{
    extern __shared__ char pad[];
    const size_t lane = threadIdx.x & 63;
    const size_t wave = (blockIdx.x * (size_t) blockDim.x + threadIdx.x) >> 6;
    const size_t nwaves = (gridDim.x * (size_t) blockDim.x) >> 6;
    for (size_t w = wave; w * 64 < chunks; w += nwaves) {
        const size_t c = w * 64 + lane;
#pragma unroll
        for (int t = 0; t < 4; ++t) { // 4 windows of 4 granules, like the body kernel
            u32x4 v[4];
#pragma unroll
            for (int k = 0; k < 4; ++k)
                v[k] = in[c * 16 + 4 * t + k];
#pragma unroll
            for (int k = 0; k < 4; ++k)
                out[c * 16 + 4 * t + k] = v[k] ^ (u32x4){1, 2, 3, 4};
        }
    }
    if (lane == 999)
        pad[0] = 0;
}

__global__ void p3_lanechunk_batched(const u32x4 *__restrict__ in, u32x4 *__restrict__ out, size_t chunks)
{
    extern __shared__ char pad[];
    const size_t lane = threadIdx.x & 63;
    const size_t wave = (blockIdx.x * (size_t) blockDim.x + threadIdx.x) >> 6;
    const size_t nwaves = (gridDim.x * (size_t) blockDim.x) >> 6;
    for (size_t w = wave; w * 64 < chunks; w += nwaves) {
        const size_t c = w * 64 + lane;
        u32x4 v[16];
#pragma unroll
        for (int k = 0; k < 16; ++k)
            v[k] = in[c * 16 + k];
#pragma unroll
        for (int k = 0; k < 16; ++k)
            out[c * 16 + k] = v[k] ^ (u32x4){1, 2, 3, 4};
    }
    if (lane == 999)
        pad[0] = 0;
}

template <typename K>
float run(K k, const u32x4 *in, u32x4 *out, size_t chunks, int wgs, int threads, size_t lds)
{
    hipEvent_t a, b;
    (void) hipEventCreate(&a);
    (void) hipEventCreate(&b);
    hipLaunchKernelGGL(k, dim3(wgs), dim3(threads), lds, 0, in, out, chunks);
    (void) hipDeviceSynchronize();
    float best = 1e9;
    for (int r = 0; r < 5; ++r) {
        (void) hipEventRecord(a, 0);
        hipLaunchKernelGGL(k, dim3(wgs), dim3(threads), lds, 0, in, out, chunks);
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
    const size_t chunks = 262144; // 64 MiB, the config-2 body payload
    u32x4 *in, *out;
    if (hipMalloc(&in, chunks * 256) != hipSuccess || hipMalloc(&out, chunks * 256) != hipSuccess)
        return 1;
    (void) hipMemset(in, 1, chunks * 256);
    const double bytes = 2.0 * chunks * 256;
    struct Occ {
        int threads, wgs_per_cu;
        size_t lds;
        const char *name;
    } occ[] = {{128, 4, 40960, "2 waves/SIMD"}, {128, 8, 16384, "4 waves/SIMD"}, {256, 8, 8192, "8 waves/SIMD"}};
    for (auto &o : occ) {
        const int wgs = 256 * o.wgs_per_cu;
        float t1 = run(p1_coalesced, in, out, chunks, wgs, o.threads, o.lds);
        float t2 = run(p2_lanechunk, in, out, chunks, wgs, o.threads, o.lds);
        float t3 = run(p3_lanechunk_batched, in, out, chunks, wgs, o.threads, o.lds);
        printf("%-13s coalesced %7.1f us %6.0f GB/s | lane-chunk %7.1f us %6.0f GB/s | lane-chunk batched %7.1f us %6.0f GB/s\n",
               o.name, t1 * 1e3, bytes / t1 / 1e6, t2 * 1e3, bytes / t2 / 1e6, t3 * 1e3, bytes / t3 / 1e6);
    }
    return 0;
}
