// Per-instruction VALU throughput on gfx950: 16 independent chains per lane,
// 8 waves per SIMD, cycles per wave-instruction per SIMD (from s_memtime)
// and chip-wide lane-ops/s.  Build: hipcc -O3 --offload-arch=gfx950.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

#define CH 16
#define BODY(OPSTR, ...)                                                      \
    for (int it = 0; it < iters; ++it) {                                      \
        _Pragma("unroll") for (int u = 0; u < CH; ++u)                        \
            asm volatile(OPSTR : __VA_ARGS__);                                \
    }

__global__ void k_add(uint32_t *out, int iters, uint32_t y)
{
    uint32_t a[CH];
    for (int u = 0; u < CH; ++u) a[u] = threadIdx.x + u;
    BODY("v_add_u32 %0, %0, %1", "+v"(a[u]) : "v"(y))
    uint32_t s = 0; for (int u = 0; u < CH; ++u) s ^= a[u];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_xor(uint32_t *out, int iters, uint32_t y)
{
    uint32_t a[CH];
    for (int u = 0; u < CH; ++u) a[u] = threadIdx.x + u;
    BODY("v_xor_b32 %0, %0, %1", "+v"(a[u]) : "v"(y))
    uint32_t s = 0; for (int u = 0; u < CH; ++u) s ^= a[u];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_alignbit(uint32_t *out, int iters, uint32_t y)
{
    uint32_t a[CH];
    for (int u = 0; u < CH; ++u) a[u] = threadIdx.x + u;
    BODY("v_alignbit_b32 %0, %0, %0, 25", "+v"(a[u]) :)
    uint32_t s = 0; for (int u = 0; u < CH; ++u) s ^= a[u];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_add3(uint32_t *out, int iters, uint32_t y)
{
    uint32_t a[CH];
    for (int u = 0; u < CH; ++u) a[u] = threadIdx.x + u;
    BODY("v_add3_u32 %0, %0, %1, %1", "+v"(a[u]) : "v"(y))
    uint32_t s = 0; for (int u = 0; u < CH; ++u) s ^= a[u];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_mullo(uint32_t *out, int iters, uint32_t y)
{
    uint32_t a[CH];
    for (int u = 0; u < CH; ++u) a[u] = threadIdx.x + u;
    BODY("v_mul_lo_u32 %0, %0, %1", "+v"(a[u]) : "v"(y))
    uint32_t s = 0; for (int u = 0; u < CH; ++u) s ^= a[u];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_mulhi(uint32_t *out, int iters, uint32_t y)
{
    uint32_t a[CH];
    for (int u = 0; u < CH; ++u) a[u] = threadIdx.x + u;
    BODY("v_mul_hi_u32 %0, %0, %1", "+v"(a[u]) : "v"(y))
    uint32_t s = 0; for (int u = 0; u < CH; ++u) s ^= a[u];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_mul24(uint32_t *out, int iters, uint32_t y)
{
    uint32_t a[CH];
    for (int u = 0; u < CH; ++u) a[u] = threadIdx.x + u;
    BODY("v_mul_u32_u24 %0, %0, %1", "+v"(a[u]) : "v"(y))
    uint32_t s = 0; for (int u = 0; u < CH; ++u) s ^= a[u];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_mad24(uint32_t *out, int iters, uint32_t y)
{
    uint32_t a[CH];
    for (int u = 0; u < CH; ++u) a[u] = threadIdx.x + u;
    BODY("v_mad_u32_u24 %0, %0, %1, %0", "+v"(a[u]) : "v"(y))
    uint32_t s = 0; for (int u = 0; u < CH; ++u) s ^= a[u];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_mulhi24(uint32_t *out, int iters, uint32_t y)
{
    uint32_t a[CH];
    for (int u = 0; u < CH; ++u) a[u] = threadIdx.x + u;
    BODY("v_mul_hi_u32_u24 %0, %0, %1", "+v"(a[u]) : "v"(y))
    uint32_t s = 0; for (int u = 0; u < CH; ++u) s ^= a[u];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_mad64(uint32_t *out, int iters, uint32_t y)
{
    uint64_t a[CH];
    for (int u = 0; u < CH; ++u) a[u] = threadIdx.x + u;
    BODY("v_mad_u64_u32 %0, s[0:1], %1, %1, %0", "+v"(a[u]) : "v"(y) : "s0", "s1")
    uint64_t s = 0; for (int u = 0; u < CH; ++u) s ^= a[u];
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t) s;
}
__global__ void k_fma64(uint32_t *out, int iters, uint32_t y)
{
    double a[CH];
    const double b = 1.0000001 + y * 1e-30;
    for (int u = 0; u < CH; ++u) a[u] = threadIdx.x + u;
    BODY("v_fma_f64 %0, %0, %1, %1", "+v"(a[u]) : "v"(b))
    double s = 0; for (int u = 0; u < CH; ++u) s += a[u];
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t) s;
}
__global__ void k_fma32(uint32_t *out, int iters, uint32_t y)
{
    float a[CH];
    const float b = 1.0001f + y * 1e-30f;
    for (int u = 0; u < CH; ++u) a[u] = threadIdx.x + u;
    BODY("v_fma_f32 %0, %0, %1, %1", "+v"(a[u]) : "v"(b))
    float s = 0; for (int u = 0; u < CH; ++u) s += a[u];
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t) s;
}
__global__ void k_pkfma32(uint32_t *out, int iters, uint32_t y)
{
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 a[CH];
    const float bb = 1.0001f + y * 1e-30f;
    const f2 b = {bb, bb};
    for (int u = 0; u < CH; ++u) a[u] = (f2){(float) threadIdx.x + u, (float) u};
    BODY("v_pk_fma_f32 %0, %0, %1, %1", "+v"(a[u]) : "v"(b))
    float s = 0; for (int u = 0; u < CH; ++u) s += a[u].x + a[u].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t) s;
}
__global__ void k_lshladd64(uint32_t *out, int iters, uint32_t y)
{
    uint64_t a[CH];
    uint64_t b = y;
    for (int u = 0; u < CH; ++u) a[u] = threadIdx.x + u;
    BODY("v_lshl_add_u64 %0, %0, 1, %1", "+v"(a[u]) : "v"(b))
    uint64_t s = 0; for (int u = 0; u < CH; ++u) s ^= a[u];
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t) s;
}
__global__ void k_pkadd16(uint32_t *out, int iters, uint32_t y)
{
    uint32_t a[CH];
    for (int u = 0; u < CH; ++u) a[u] = threadIdx.x + u;
    BODY("v_pk_add_u16 %0, %0, %1", "+v"(a[u]) : "v"(y))
    uint32_t s = 0; for (int u = 0; u < CH; ++u) s ^= a[u];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_dot4(uint32_t *out, int iters, uint32_t y)
{
    uint32_t a[CH];
    for (int u = 0; u < CH; ++u) a[u] = threadIdx.x + u;
    BODY("v_dot4_u32_u8 %0, %1, %1, %0", "+v"(a[u]) : "v"(y))
    uint32_t s = 0; for (int u = 0; u < CH; ++u) s ^= a[u];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

typedef void (*KF)(uint32_t *, int, uint32_t);

int main()
{
    uint32_t *buf;
    const int threads = 256;
    CHECK(hipMalloc(&buf, sizeof(uint32_t) * 256 * 8 * 4 * threads));
    struct { const char *name; KF k; } ks[] = {
        {"v_add_u32", k_add},       {"v_xor_b32", k_xor},        {"v_alignbit_b32", k_alignbit},
        {"v_add3_u32", k_add3},     {"v_mul_lo_u32", k_mullo},   {"v_mul_hi_u32", k_mulhi},
        {"v_mul_u32_u24", k_mul24}, {"v_mad_u32_u24", k_mad24},  {"v_mul_hi_u32_u24", k_mulhi24},
        {"v_mad_u64_u32", k_mad64}, {"v_fma_f64", k_fma64},      {"v_fma_f32", k_fma32},
        {"v_pk_fma_f32", k_pkfma32}, {"v_lshl_add_u64", k_lshladd64}, {"v_pk_add_u16", k_pkadd16},
        {"v_dot4_u32_u8", k_dot4},
    };
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    for (int wps : {1, 2, 8}) {
        const int blocks = 256 * wps; // 256-thread blocks = 4 waves = 1 per SIMD per block
        for (auto &k : ks) {
            const int iters = 2000;
            hipLaunchKernelGGL(k.k, dim3(blocks), dim3(threads), 0, 0, buf, 10, 3u);
            CHECK(hipDeviceSynchronize());
            float best = 1e9;
            for (int r = 0; r < 3; ++r) {
                CHECK(hipEventRecord(a, 0));
                hipLaunchKernelGGL(k.k, dim3(blocks), dim3(threads), 0, 0, buf, iters, 3u);
                CHECK(hipEventRecord(b, 0));
                CHECK(hipEventSynchronize(b));
                float ms;
                CHECK(hipEventElapsedTime(&ms, a, b));
                best = ms < best ? ms : best;
            }
            const double winstr_per_simd = (double) wps * iters * CH; // wave-instructions each SIMD issues
            const double ns_per = best * 1e6 / winstr_per_simd;
            printf("%d w/SIMD %-18s %.3f ms  %.2f ns/wave-instr/SIMD (= %.1f cyc @2.4GHz)  %.1f T lane-ops/s\n", wps,
                   k.name, best, ns_per, ns_per * 2.4, (double) blocks * threads * iters * CH / best / 1e9);
        }
    }
    return 0;
}
