// Unaligned 16-byte global access on gfx950: correctness and speed of
// lane-chunk copies (lane = 256-byte chunk) at byte offsets 0, 1, 5, 15.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 u32x4_a1 __attribute__((aligned(1)));

__global__ void lanechunk_ua(const uint8_t *__restrict__ in, uint8_t *__restrict__ out, size_t chunks, int ioff,
                             int ooff)
{
    const size_t lane = threadIdx.x & 63;
    const size_t wave = (blockIdx.x * (size_t) blockDim.x + threadIdx.x) >> 6;
    const size_t nwaves = (gridDim.x * (size_t) blockDim.x) >> 6;
    for (size_t w = wave; w * 64 < chunks; w += nwaves) {
        const size_t c = w * 64 + lane;
        const u32x4_a1 *p = (const u32x4_a1 *) (in + ioff + c * 256);
        u32x4_a1 *q = (u32x4_a1 *) (out + ooff + c * 256);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            u32x4 v[4];
#pragma unroll
            for (int k = 0; k < 4; ++k)
                v[k] = p[4 * t + k];
#pragma unroll
            for (int k = 0; k < 4; ++k)
                q[4 * t + k] = v[k] ^ (u32x4){0x01010101u, 0x01010101u, 0x01010101u, 0x01010101u};
        }
    }
}

int main()
{
    const size_t chunks = 262144, bytes = chunks * 256 + 64;
    uint8_t *in, *out;
    if (hipMalloc(&in, bytes) != hipSuccess || hipMalloc(&out, bytes) != hipSuccess)
        return 1;
    uint8_t *h = (uint8_t *) malloc(bytes), *g = (uint8_t *) malloc(bytes);
    for (size_t i = 0; i < bytes; ++i)
        h[i] = (uint8_t) (i * 131 + (i >> 9));
    (void) hipMemcpy(in, h, bytes, hipMemcpyHostToDevice);
    int offs[][2] = {{0, 0}, {1, 0}, {0, 1}, {5, 13}, {15, 15}, {31, 3}};
    for (auto &o : offs) {
        (void) hipMemset(out, 0, bytes);
        hipEvent_t a, b;
        (void) hipEventCreate(&a);
        (void) hipEventCreate(&b);
        hipLaunchKernelGGL(lanechunk_ua, dim3(1024), dim3(256), 0, 0, in, out, chunks, o[0], o[1]);
        (void) hipDeviceSynchronize();
        (void) hipMemcpy(g, out, bytes, hipMemcpyDeviceToHost);
        size_t bad = 0;
        for (size_t i = 0; i < chunks * 256; ++i)
            bad += g[o[1] + i] != (uint8_t) (h[o[0] + i] ^ 1);
        for (int i = 0; i < o[1]; ++i)
            bad += g[i] != 0;
        float best = 1e9;
        for (int r = 0; r < 5; ++r) {
            (void) hipEventRecord(a, 0);
            hipLaunchKernelGGL(lanechunk_ua, dim3(1024), dim3(256), 0, 0, in, out, chunks, o[0], o[1]);
            (void) hipEventRecord(b, 0);
            (void) hipEventSynchronize(b);
            float ms;
            (void) hipEventElapsedTime(&ms, a, b);
            best = ms < best ? ms : best;
        }
        printf("in+%2d out+%2d: %s, %.1f us, %.0f GB/s\n", o[0], o[1], bad ? "WRONG" : "ok", best * 1e3,
               2.0 * chunks * 256 / best / 1e6);
    }
    return 0;
}
