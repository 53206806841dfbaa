// Round 4: the floor under a per-message call -- one kernel launch that
// only sets a completion word in mapped host memory, the host polling it
// (the shape of zmqg_encode_msg's wait), against hipStreamSynchronize.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/bin/launch_floor tools/launch_floor.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <chrono>

template <int ARGB>
struct Args {
    uint32_t w[ARGB / 4];
};

template <int ARGB>
__global__ void k_done(uint32_t *done, Args<ARGB> a)
{
    if (threadIdx.x == 0) {
        __threadfence_system();
        __hip_atomic_store(done, a.w[0] + 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

template <int ARGB>
static void run(hipStream_t st, uint32_t *h, uint32_t *d, int threads)
{
    Args<ARGB> a{};
    const int iters = 2000;
    for (int mode = 0; mode < 2; ++mode) {
        double tot = 0;
        for (int i = 0; i < iters + 50; ++i) {
            a.w[0] = (uint32_t) i;
            __atomic_store_n(h, 0u, __ATOMIC_RELEASE);
            const auto t0 = std::chrono::steady_clock::now();
            hipLaunchKernelGGL(k_done<ARGB>, dim3(1), dim3(threads), 0, st, d, a);
            if (mode == 0) {
                while (__atomic_load_n(h, __ATOMIC_ACQUIRE) != (uint32_t) i + 1u) {
                }
            } else {
                (void) hipStreamSynchronize(st);
            }
            const auto t1 = std::chrono::steady_clock::now();
            if (i >= 50)
                tot += std::chrono::duration<double, std::micro>(t1 - t0).count();
        }
        printf("{\"arg_bytes\": %d, \"threads\": %d, \"wait\": \"%s\", \"us_per_call\": %.2f}\n", ARGB, threads,
               mode == 0 ? "poll" : "stream_sync", tot / iters);
    }
}

int main()
{
    uint32_t *h = nullptr, *d = nullptr;
    if (hipHostMalloc((void **) &h, 64, hipHostMallocMapped) != hipSuccess ||
        hipHostGetDevicePointer((void **) &d, h, 0) != hipSuccess)
        return 1;
    hipStream_t st;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess)
        return 2;
    run<16>(st, h, d, 64);
    run<256>(st, h, d, 64);
    run<1024>(st, h, d, 256);
    run<3968>(st, h, d, 256);
    return 0;
}
