// The floor of a resident per-message kernel (verdict
// round 4 item 6): instead of one launch per zmqg_encode_msg call, one
// workgroup stays resident and polls a doorbell the host writes in
// page-locked coherent host memory; per request it reads the request's bytes
// from host memory, writes a result of the same size back, and sets a
// completion word the host polls.  Prints the host-timed round trip per
// request size (median and 90th percentile of 2,000 requests) -- the part of
// a call such a kernel would cost before any crypto, to set against the
// launch path's 6.1-7.0 us floor (tools/launch_floor.hip).
//
// Exit conditions: the host's stop value, and a 20 s bound on the kernel's
// own clock (s_memrealtime, 100 MHz), so the grid always drains.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/bin/resident_probe tools/resident_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <chrono>
#include <vector>

#define CK(x)                                                                                    \
    do {                                                                                         \
        hipError_t e = (x);                                                                      \
        if (e != hipSuccess) {                                                                   \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e));     \
            exit(1);                                                                             \
        }                                                                                        \
    } while (0)

struct Ctl {
    uint32_t door;  // host -> device: request number (0xffffffff: stop)
    uint32_t bytes; // request size
    uint32_t done;  // device -> host: last request completed
    uint32_t pad;
};

__global__ __launch_bounds__(64) void k_resident(Ctl *ctl, const uint32_t *req, uint32_t *resp)
{
    const uint32_t lane = threadIdx.x;
    uint32_t last = 0;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        uint32_t d = 0;
        if (lane == 0)
            d = __hip_atomic_load(&ctl->door, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
        d = __builtin_amdgcn_readfirstlane(d);
        if (d == 0xffffffffu)
            break;
        if (d != last) {
            last = d;
            const uint32_t bytes = __hip_atomic_load(&ctl->bytes, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            // the request's bytes over PCIe, the result back: 16 bytes per
            // lane per round, every round's loads issued before any is used
            // (coherent host memory is not cached by the GPU, so plain loads
            // after the doorbell's acquire see the host's writes)
            typedef uint32_t u4 __attribute__((ext_vector_type(4)));
            const u4 *rq = (const u4 *) req;
            u4 *rs = (u4 *) resp;
            u4 v[4];
#pragma unroll
            for (uint32_t j = 0; j < 4; ++j)
                if (16u * (lane + 64u * j) < bytes)
                    v[j] = rq[lane + 64u * j];
#pragma unroll
            for (uint32_t j = 0; j < 4; ++j)
                if (16u * (lane + 64u * j) < bytes)
                    rs[lane + 64u * j] = v[j] ^ d;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            if (lane == 0)
                __hip_atomic_store(&ctl->done, d, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        if (__builtin_amdgcn_s_memrealtime() - t0 > 2000000000ull) // 20 s at 100 MHz
            break;
    }
}

int main()
{
    Ctl *ctl = nullptr;
    uint32_t *req = nullptr, *resp = nullptr;
    const size_t maxb = 4096;
    CK(hipHostMalloc((void **) &ctl, sizeof(Ctl), hipHostMallocMapped | hipHostMallocCoherent));
    CK(hipHostMalloc((void **) &req, maxb, hipHostMallocMapped | hipHostMallocCoherent));
    CK(hipHostMalloc((void **) &resp, maxb, hipHostMallocMapped | hipHostMallocCoherent));
    Ctl *dctl;
    uint32_t *dreq, *dresp;
    CK(hipHostGetDevicePointer((void **) &dctl, ctl, 0));
    CK(hipHostGetDevicePointer((void **) &dreq, req, 0));
    CK(hipHostGetDevicePointer((void **) &dresp, resp, 0));
    *ctl = Ctl{0, 0, 0, 0};
    for (size_t k = 0; k < maxb / 4; ++k)
        req[k] = (uint32_t) (k * 2654435761u);
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipLaunchKernelGGL(k_resident, dim3(1), dim3(64), 0, st, dctl, dreq, dresp);
    CK(hipGetLastError());
    uint32_t seq = 0;
    bool ok = true;
    for (uint32_t bytes : {16u, 256u, 1024u, 4096u}) {
        std::vector<double> us;
        for (int r = 0; r < 2200; ++r) {
            ++seq;
            __atomic_store_n(&ctl->bytes, bytes, __ATOMIC_RELAXED);
            const auto t0 = std::chrono::steady_clock::now();
            __atomic_store_n(&ctl->door, seq, __ATOMIC_RELEASE);
            bool seen = false;
            while (!seen) {
                if (__atomic_load_n(&ctl->done, __ATOMIC_ACQUIRE) == seq)
                    seen = true;
                else if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2))
                    break;
            }
            const auto t1 = std::chrono::steady_clock::now();
            if (!seen) {
                fprintf(stderr, "request %u not completed within 2 s\n", seq);
                ok = false;
                break;
            }
            if (r >= 200)
                us.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
            for (uint32_t k = 0; k < (bytes < 16 ? 4 : bytes / 4); k += 97)
                if (resp[k] != (req[k] ^ seq)) {
                    fprintf(stderr, "request %u: word %u wrong\n", seq, k);
                    ok = false;
                }
        }
        if (!ok)
            break;
        std::sort(us.begin(), us.end());
        printf("{\"bytes\": %u, \"median_us\": %.2f, \"p90_us\": %.2f, \"min_us\": %.2f}\n", bytes,
               us[us.size() / 2], us[us.size() * 9 / 10], us[0]);
    }
    __atomic_store_n(&ctl->door, 0xffffffffu, __ATOMIC_RELEASE);
    CK(hipStreamSynchronize(st));
    CK(hipStreamDestroy(st));
    CK(hipHostFree(ctl));
    CK(hipHostFree(req));
    CK(hipHostFree(resp));
    return ok ? 0 : 1;
}
