// Memory-pattern experiment for lane-per-frame CURVE kernels: copy n frames
// of F bytes (in stride SI, out stride SO, arbitrary alignment) window by
// window (64 B), with D windows of loads in flight, in two access shapes:
//   LANE  lane = frame, each lane loads its own 4 x 16 B per window
//   COOP  4 lanes per frame-window (16 frames per instruction)
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/bin/framecopy tools/framecopy.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 u32x4_u __attribute__((aligned(1)));

template <bool COOP, int D>
__global__ __launch_bounds__(256) void k_copy(uint32_t n, uint32_t F, uint64_t SI, uint64_t SO,
                                              const uint8_t *__restrict__ in, uint8_t *__restrict__ out)
{
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t f0 = (blockIdx.x * 256 + (threadIdx.x & ~63u)); // wave's first frame
    const uint32_t nw = F / 64;
    uint64_t ib[4], ob[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (COOP) {
            const uint32_t fr = f0 + 16 * k + (lane >> 2);
            ib[k] = (uint64_t) fr * SI + 16 * (lane & 3);
            ob[k] = (uint64_t) fr * SO + 16 * (lane & 3);
        } else {
            ib[k] = (uint64_t) (f0 + lane) * SI + 16 * k;
            ob[k] = (uint64_t) (f0 + lane) * SO + 16 * k;
        }
    }
    if (f0 >= n)
        return;
    u32x4 buf[D][4];
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
        for (int k = 0; k < 4; ++k)
            buf[d][k] = *(const u32x4_u *) (in + ib[k] + 64 * d);
    for (uint32_t w = 0; w < nw; w += D) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
#pragma unroll
            for (int k = 0; k < 4; ++k)
                *(u32x4_u *) (out + ob[k] + 64 * (w + d)) = buf[d][k] ^ (u32x4){1, 2, 3, 4};
            if (w + d + D < nw) {
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    buf[d][k] = *(const u32x4_u *) (in + ib[k] + 64 * (w + d + D));
            }
        }
    }
}

int main(int argc, char **argv)
{
    const uint32_t n = argc > 1 ? atoi(argv[1]) : 65536;
    const uint32_t F = 1024;
    uint8_t *in, *out;
    const size_t maxb = (size_t) n * 1100 + 4096;
    CHECK(hipMalloc(&in, maxb));
    CHECK(hipMalloc(&out, maxb));
    CHECK(hipMemset(in, 1, maxb));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    struct Case { uint64_t si, so; int ioff, ooff; } cases[] = {
        {1024, 1024, 0, 0}, {1024, 1057, 0, 0}, {1024, 1088, 0, 0}, {1024, 1057, 33, 0}, {1088, 1088, 0, 0}};
    for (auto &c : cases) {
        auto run = [&](auto kern, const char *name) {
            const uint32_t blocks = (n + 255) / 256;
            hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, n, F, c.si, c.so, in + c.ioff, out + c.ooff);
            CHECK(hipDeviceSynchronize());
            float best = 1e9;
            for (int r = 0; r < 5; ++r) {
                CHECK(hipEventRecord(a, 0));
                hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, n, F, c.si, c.so, in + c.ioff, out + c.ooff);
                CHECK(hipEventRecord(b, 0));
                CHECK(hipEventSynchronize(b));
                float ms;
                CHECK(hipEventElapsedTime(&ms, a, b));
                best = ms < best ? ms : best;
            }
            printf("n=%u SI=%4lu SO=%4lu ioff=%2d %-9s %7.1f us  %6.0f GB/s (in+out)\n", n, (unsigned long) c.si,
                   (unsigned long) c.so, c.ioff, name, best * 1e3, 2.0 * n * F / best / 1e6);
        };
        run(k_copy<false, 1>, "LANE D=1");
        run(k_copy<false, 4>, "LANE D=4");
        run(k_copy<true, 1>, "COOP D=1");
        run(k_copy<true, 4>, "COOP D=4");
    }
    return 0;
}
