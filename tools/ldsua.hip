// Does gfx950 LDS serve unaligned ds_read_b32/b64/b128 and ds_write_b32/b128
// correctly, and at what cost?  Build: hipcc -O3 --offload-arch=gfx950.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ void k_test(uint32_t *out, int sh)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[64 * 96];
    const int lane = threadIdx.x;
    for (int b = lane; b < 64 * 96; b += 64)
        lds[b] = (uint8_t) (b * 7 + 3);
    __syncthreads();
    const uint32_t a = lane * 80 + sh + (lane & 7);
    uint32_t r32, r128[4];
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(r32) : "v"(a));
    u32x4 v;
    asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a));
    r128[0] = v.x; r128[1] = v.y; r128[2] = v.z; r128[3] = v.w;
    uint32_t bad = 0;
    uint32_t e = 0;
    for (int t = 0; t < 4; ++t)
        e |= (uint32_t) (uint8_t) ((a + t) * 7 + 3) << (8 * t);
    bad += r32 != e;
    for (int q = 0; q < 4; ++q) {
        uint32_t eq = 0;
        for (int t = 0; t < 4; ++t)
            eq |= (uint32_t) (uint8_t) ((a + 4 * q + t) * 7 + 3) << (8 * t);
        bad += r128[q] != eq;
    }
    // unaligned write then aligned read-back
    __syncthreads();
    const u32x4 wv = {0x11111111u * (lane & 15), 0x22222222u, 0x33333333u, 0x44444444u};
    const uint32_t wa = lane * 80 + 3 + sh;
    asm volatile("ds_write_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" ::"v"(wa), "v"(wv) : "memory");
    __syncthreads();
    uint32_t got[4];
    for (int q = 0; q < 4; ++q) {
        uint32_t g = 0;
        for (int t = 0; t < 4; ++t)
            g |= (uint32_t) lds[wa + 4 * q + t] << (8 * t);
        got[q] = g;
    }
    bad += (got[0] != wv.x) + (got[1] != wv.y) + (got[2] != wv.z) + (got[3] != wv.w);
    out[lane] = bad;
}

int main()
{
    uint32_t *d;
    hipMalloc(&d, 256);
    for (int sh = 0; sh < 4; ++sh) {
        hipLaunchKernelGGL(k_test, dim3(1), dim3(64), 0, 0, d, sh);
        uint32_t h[64];
        hipError_t e = hipMemcpy(h, d, 256, hipMemcpyDeviceToHost);
        uint32_t tot = 0;
        for (int i = 0; i < 64; ++i)
            tot += h[i];
        printf("sh=%d: %s, mismatched words %u\n", sh, e == hipSuccess ? "ran" : hipGetErrorString(e), tot);
    }
    return 0;
}
