// Dependent VOP2/VOP3 chains on gfx950 (why a Salsa20 block costs more than
// the sum of its instructions' independent issue costs): C chains of
// add -> alignbit -> xor steps (each step's add reads the previous xor).
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/bin/dep_mix tools/dep_mix.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
__device__ unsigned long long g_clk[2];

// MODE 0: add, alignbit, xor   1: add, xor, xor (all VOP2)   2: alignbit x3   3: add,add,add
//      4: add, alignbit, xor with the alignbit of a chain two steps behind (software pipelined)
template <int C, int MODE>
__global__ __launch_bounds__(256) void k_dep(uint32_t *o, int iters, uint32_t y)
{
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    uint32_t s[C], u[C], t[C];
    for (int c = 0; c < C; ++c) { s[c] = threadIdx.x + c * 77 + y; u[c] = s[c] * 3; t[c] = 0; }
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int rep = 0; rep < 16 / C * 4; ++rep) {
#pragma unroll
            for (int c = 0; c < C; ++c) {
                if (MODE == 0 || MODE == 4) asm volatile("v_add_u32 %0, %1, %2" : "=v"(t[c]) : "v"(s[c]), "v"(u[c]));
                else if (MODE == 1 || MODE == 3) asm volatile("v_add_u32 %0, %1, %2" : "=v"(t[c]) : "v"(s[c]), "v"(u[c]));
                else asm volatile("v_alignbit_b32 %0, %1, %1, 25" : "=v"(t[c]) : "v"(s[c]));
            }
#pragma unroll
            for (int c = 0; c < C; ++c) {
                if (MODE == 0 || MODE == 2 || MODE == 4) asm volatile("v_alignbit_b32 %0, %0, %0, 25" : "+v"(t[c]));
                else if (MODE == 1) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(t[c]) : "v"(u[c]));
                else asm volatile("v_add_u32 %0, %0, %1" : "+v"(t[c]) : "v"(u[c]));
            }
#pragma unroll
            for (int c = 0; c < C; ++c) {
                if (MODE == 2) asm volatile("v_alignbit_b32 %0, %1, %1, 7" : "=v"(s[c]) : "v"(t[c]));
                else if (MODE == 3) asm volatile("v_add_u32 %0, %0, %1" : "+v"(s[c]) : "v"(t[c]));
                else asm volatile("v_xor_b32 %0, %0, %1" : "+v"(s[c]) : "v"(t[c]));
            }
        }
    }
    uint32_t a = 0;
    for (int c = 0; c < C; ++c) a ^= s[c];
    o[blockIdx.x * blockDim.x + threadIdx.x] = a;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        g_clk[0] = __builtin_amdgcn_s_memtime() - t0;
        g_clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
}
typedef void (*KF)(uint32_t *, int, uint32_t);
int main()
{
    uint32_t *buf;
    if (hipMalloc(&buf, 4 << 22) != hipSuccess) return 1;
    int cus = 0;
    (void) hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    hipEvent_t a, b;
    (void) hipEventCreate(&a);
    (void) hipEventCreate(&b);
    struct { const char *n; KF k; } ks[] = {
        {"add>align>xor C4", k_dep<4, 0>}, {"add>align>xor C8", k_dep<8, 0>}, {"add>align>xor C16", k_dep<16, 0>},
        {"add>xor>xor C4", k_dep<4, 1>},   {"add>xor>xor C16", k_dep<16, 1>},
        {"align x3 C4", k_dep<4, 2>},      {"align x3 C16", k_dep<16, 2>},
        {"add x3 C4", k_dep<4, 3>},        {"add x3 C16", k_dep<16, 3>},
    };
    for (auto &k : ks)
        for (int wps : {2, 4, 8}) {
            const int iters = 20000 * 2 / (wps + 1);
            hipLaunchKernelGGL(k.k, dim3(cus * wps), dim3(256), 0, 0, buf, iters / 4 + 1, 3u);
            if (hipDeviceSynchronize() != hipSuccess) return 2;
            (void) hipEventRecord(a, 0);
            hipLaunchKernelGGL(k.k, dim3(cus * wps), dim3(256), 0, 0, buf, iters, 3u);
            (void) hipEventRecord(b, 0);
            if (hipEventSynchronize(b) != hipSuccess) return 3;
            float ms = 0;
            (void) hipEventElapsedTime(&ms, a, b);
            unsigned long long clk[2];
            (void) hipMemcpyFromSymbol(clk, HIP_SYMBOL(g_clk), sizeof clk);
            const double ghz = (double) clk[0] / (double) clk[1] * 0.1;
            printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"clock_ghz\": %.3f, \"cycles_per_unit_per_simd\": %.3f}\n",
                   k.n, wps, ghz, ms * 1e6 * ghz / ((double) wps * iters * 16 * 4 * 3));
            fflush(stdout);
        }
    return 0;
}
