// VALU issue rates on gfx950 (MI355X): cycles per wave64 instruction per
// SIMD, for the instructions the CURVE frame kernel is made of, at 1, 2, 4
// and 8 waves per SIMD.  Reconciles the 16-lanes-per-cycle figure used for
// roofline.valu.peak with MI355X_MICROARCH.md's 2-cycle v_fma_f32.
//
// Method: every kernel runs 256 x k workgroups of 256 threads (one wave per
// SIMD per workgroup, k waves per SIMD), each lane a loop of 16 independent
// dependency chains of the instruction under test (or one chain: latency),
// long enough (>= 2 ms) for steady clocks.  Cycles = kernel wall time (HIP
// events) x in-kernel clock (s_memtime / s_memrealtime of workgroup 0, 100
// MHz reference); per SIMD instruction count = k x iters x instructions per
// iteration.  Output: one JSON object per line (tools/valu_rates.py makes
// the table under profiles/).
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/bin/valu_rates tools/valu_rates.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include "../libzmq_amd/csrc/curve_device.hpp"
using namespace zmqg;

__device__ unsigned long long g_clk[2];

#define OPS16(STMT)                       \
    _Pragma("unroll") for (int u = 0; u < 16; ++u) { STMT; }

template <int OP>
__global__ __launch_bounds__(256) void k_op(uint32_t *out, int iters, uint32_t y)
{
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    uint32_t a[16];
    float f[16];
    for (int u = 0; u < 16; ++u) {
        a[u] = threadIdx.x * 16 + u + y;
        f[u] = (float) a[u];
    }
    for (int it = 0; it < iters; ++it) {
        if (OP == 0) OPS16(asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[u]) : "v"(y)))
        else if (OP == 1) OPS16(asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[u]) : "v"(y)))
        else if (OP == 2) OPS16(asm volatile("v_alignbit_b32 %0, %0, %0, 25" : "+v"(a[u])))
        else if (OP == 3) OPS16(asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(a[u]) : "v"(y)))
        else if (OP == 4) OPS16(asm volatile("v_xad_u32 %0, %0, %1, %1" : "+v"(a[u]) : "v"(y)))
        else if (OP == 5) OPS16(asm volatile("v_bitop3_b32 %0, %0, %1, %1 bitop3:0x96" : "+v"(a[u]) : "v"(y)))
        else if (OP == 6) OPS16(asm volatile("v_lshl_or_b32 %0, %0, 7, %1" : "+v"(a[u]) : "v"(y)))
        else if (OP == 7) {
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                uint64_t t = ((uint64_t) a[2 * u + 1] << 32) | a[2 * u];
                asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %1, %0" : "+v"(t) : "v"(y) : "s0", "s1");
                a[2 * u] = (uint32_t) t;
                a[2 * u + 1] = (uint32_t) (t >> 32);
            }
        } else if (OP == 8) OPS16(asm volatile("v_mad_u32_u24 %0, %0, %1, %1" : "+v"(a[u]) : "v"(y)))
        else if (OP == 9) OPS16(asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[u]) : "v"(y)))
        else if (OP == 10) OPS16(asm volatile("v_fma_f32 %0, %0, %0, %0" : "+v"(f[u])))
        else if (OP == 11) OPS16(asm volatile("v_add_f32 %0, %0, %0" : "+v"(f[u])))
        else if (OP == 12) {
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                typedef float f2 __attribute__((ext_vector_type(2)));
                f2 t = {f[2 * u], f[2 * u + 1]};
                asm volatile("v_pk_fma_f32 %0, %0, %0, %0" : "+v"(t));
                f[2 * u] = t.x;
                f[2 * u + 1] = t.y;
            }
        } else if (OP == 13) OPS16(asm volatile("v_mov_b32 %0, %1" : "=v"(a[u]) : "v"(a[(u + 1) & 15])))
        else if (OP == 14) OPS16(asm volatile("v_alignbyte_b32 %0, %0, %1, 1" : "+v"(a[u]) : "v"(y)))
        else if (OP == 15) OPS16(asm volatile("v_and_b32 %0, %0, %1" : "+v"(a[u]) : "v"(y)))
        else if (OP == 16) OPS16(asm volatile("v_lshrrev_b32 %0, 3, %0" : "+v"(a[u])))
        else if (OP == 17) OPS16(asm volatile("v_perm_b32 %0, %0, %1, %1" : "+v"(a[u]) : "v"(y)))
        else if (OP == 18) { // one dependent chain of v_add_u32 (latency)
#pragma unroll
            for (int u = 0; u < 16; ++u)
                asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[0]) : "v"(y));
        } else if (OP == 19) { // one dependent chain of v_alignbit_b32
#pragma unroll
            for (int u = 0; u < 16; ++u)
                asm volatile("v_alignbit_b32 %0, %0, %0, 25" : "+v"(a[0]));
        } else if (OP == 20) { // 4 chains (one Salsa20 round's parallelism)
#pragma unroll
            for (int u = 0; u < 16; ++u)
                asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[u & 3]) : "v"(y));
        } else if (OP == 21) { // 2 chains
#pragma unroll
            for (int u = 0; u < 16; ++u)
                asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[u & 1]) : "v"(y));
        } else if (OP == 22) OPS16(asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(a[u]) : "v"(y) : "vcc"))
        else if (OP == 23) { // v_mad_u64_u32 with 4 independent accumulators per group of 4 (mad chain shape)
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                uint64_t t = ((uint64_t) a[2 * u + 1] << 32) | a[2 * u];
                t = (uint64_t) a[(2 * u + 3) & 15] * y + t;
                a[2 * u] = (uint32_t) t;
                a[2 * u + 1] = (uint32_t) (t >> 32);
            }
        }
    }
    uint32_t s = 0;
    for (int u = 0; u < 16; ++u)
        s ^= a[u] ^ __float_as_uint(f[u]);
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        g_clk[0] = __builtin_amdgcn_s_memtime() - t0;
        g_clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
}

// NB Salsa20 blocks per lane per iteration (NB independent blocks interleave)
template <int NB>
__global__ __launch_bounds__(256) void k_salsa(uint32_t *out, int iters, uint32_t y)
{
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    uint32_t k8[8];
    for (int u = 0; u < 8; ++u)
        k8[u] = threadIdx.x * 8 + u + y;
    uint32_t acc = y;
    for (int it = 0; it < iters; ++it) {
        uint32_t ks[NB][16];
#pragma unroll
        for (int b = 0; b < NB; ++b)
            salsa20_block(ks[b], k8, acc, y, it * NB + b, 0);
#pragma unroll
        for (int b = 0; b < NB; ++b)
#pragma unroll
            for (int u = 0; u < 16; ++u)
                acc ^= ks[b][u];
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        g_clk[0] = __builtin_amdgcn_s_memtime() - t0;
        g_clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
}

typedef void (*KF)(uint32_t *, int, uint32_t);
int main()
{
    uint32_t *buf;
    if (hipMalloc(&buf, sizeof(uint32_t) * 256 * 8 * 256) != hipSuccess)
        return 1;
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    struct {
        const char *name;
        KF k;
        double ipi; // instructions (or Salsa20 blocks) per iteration per lane
        int iters1; // iterations at 1 wave per SIMD
    } ks[] = {
        {"v_add_u32", k_op<0>, 16, 60000},         {"v_xor_b32", k_op<1>, 16, 60000},
        {"v_alignbit_b32", k_op<2>, 16, 60000},    {"v_add3_u32", k_op<3>, 16, 60000},
        {"v_xad_u32", k_op<4>, 16, 60000},         {"v_bitop3_b32", k_op<5>, 16, 60000},
        {"v_lshl_or_b32", k_op<6>, 16, 60000},     {"v_mad_u64_u32", k_op<7>, 8, 60000},
        {"v_mad_u32_u24", k_op<8>, 16, 60000},     {"v_mul_lo_u32", k_op<9>, 16, 30000},
        {"v_fma_f32", k_op<10>, 16, 60000},        {"v_add_f32", k_op<11>, 16, 60000},
        {"v_pk_fma_f32", k_op<12>, 8, 60000},      {"v_mov_b32", k_op<13>, 16, 60000},
        {"v_alignbyte_b32", k_op<14>, 16, 60000},  {"v_and_b32", k_op<15>, 16, 60000},
        {"v_lshrrev_b32", k_op<16>, 16, 60000},    {"v_perm_b32", k_op<17>, 16, 60000},
        {"v_add_u32 1 chain", k_op<18>, 16, 20000}, {"v_alignbit 1 chain", k_op<19>, 16, 20000},
        {"v_add_u32 4 chains", k_op<20>, 16, 40000}, {"v_add_u32 2 chains", k_op<21>, 16, 30000},
        {"v_add_co_u32", k_op<22>, 16, 60000},     {"mad64 compiler", k_op<23>, 8, 60000},
        {"salsa20 block x1", k_salsa<1>, 1, 800},  {"salsa20 block x2", k_salsa<2>, 2, 400},
    };
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (auto &k : ks) {
        for (int wps : {1, 2, 3, 4, 8}) {
            const int blocks = cus * wps;
            const int iters = k.iters1 * 2 / (wps + 1); // similar wall time per row
            hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, buf, iters / 4 + 1, 3u);
            if (hipDeviceSynchronize() != hipSuccess)
                return 2;
            hipEventRecord(a, 0);
            hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, buf, iters, 3u);
            hipEventRecord(b, 0);
            if (hipEventSynchronize(b) != hipSuccess)
                return 3;
            float ms;
            hipEventElapsedTime(&ms, a, b);
            unsigned long long clk[2];
            hipMemcpyFromSymbol(clk, HIP_SYMBOL(g_clk), sizeof clk);
            const double ghz = (double) clk[0] / (double) clk[1] * 0.1;
            const double units = (double) wps * iters * k.ipi; // per SIMD
            printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"clock_ghz\": %.3f, "
                   "\"cycles_per_unit_per_simd\": %.3f}\n",
                   k.name, wps, ms, ghz, ms * 1e6 * ghz / units);
            fflush(stdout);
        }
    }
    return 0;
}
