// Issue cost of global dwordx4 loads/stores on gfx950 by access shape: one
// wave per SIMD, each instruction's 64 lanes spread over 64, 32, 16 or 4
// distinct 64-byte pieces (LPP = lanes per piece: 1, 2, 4, 16), pieces
// strided 1,057 bytes apart (the config-2 frame stride), 4-byte aligned
// (misaligned to 16) or 16-byte aligned.  Cycles per instruction per wave
// from s_memtime around bursts of 8 instructions (no wait inside the burst).
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/bin/vmem_issue tools/vmem_issue.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 u32x4_a4 __attribute__((aligned(4)));
__device__ unsigned long long g_cyc[2];

template <int LPP, int STORE, int ALIGN16>
__global__ __launch_bounds__(256) void k_vm(uint8_t *buf, int iters, unsigned long long *out)
{
    const uint32_t lane = threadIdx.x & 63, wave = blockIdx.x * 4 + (threadIdx.x >> 6);
    // piece p of this wave: 64 / LPP pieces per instruction
    const uint32_t piece = lane / LPP, sub = lane % LPP;
    const uint32_t npieces = 64 / LPP;
    uint64_t base = (uint64_t) (uintptr_t) buf + (uint64_t) wave * 64 * 1057;
    uint64_t addr = base + (uint64_t) piece * 1057 + (ALIGN16 ? 0 : 4);
    if (ALIGN16)
        addr &= ~15ull;
    addr += 16ull * (sub % 4) + 64ull * (sub / 4); // LPP=16: 256 contiguous bytes
    u32x4 acc = {lane, 0, 0, 0};
    unsigned long long tot = 0;
    for (int it = 0; it < iters; ++it) {
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint64_t a = addr + (uint64_t) k * npieces * 1057 * 0 + 64ull * 4 * k * (LPP < 16);
            if (STORE)
                *(u32x4_a4 *) (uintptr_t) a = acc;
            else {
                const u32x4 v = *(const u32x4_a4 *) (uintptr_t) a;
                acc ^= v;
            }
        }
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        tot += t1 - t0;
        acc.y += it;
    }
    if (lane == 0)
        out[wave] = tot;
    if (acc.x == 0xdeadbeef)
        buf[0] = 1;
}

typedef void (*KF)(uint8_t *, int, unsigned long long *);
int main()
{
    int cus = 0;
    (void) hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const size_t nw = (size_t) cus * 4;
    uint8_t *buf;
    unsigned long long *out;
    if (hipMalloc(&buf, nw * 64 * 1057 + 8192) != hipSuccess || hipMalloc(&out, nw * 8) != hipSuccess)
        return 1;
    (void) hipMemset(buf, 0, nw * 64 * 1057 + 8192);
    struct { const char *n; KF k; } ks[] = {
        {"load  1 lane/piece a4", k_vm<1, 0, 0>},  {"load  2 lanes/piece a4", k_vm<2, 0, 0>},
        {"load  4 lanes/piece a4", k_vm<4, 0, 0>}, {"load 16 lanes/piece a4", k_vm<16, 0, 0>},
        {"load  1 lane/piece a16", k_vm<1, 0, 1>}, {"load  4 lanes/piece a16", k_vm<4, 0, 1>},
        {"store 1 lane/piece a4", k_vm<1, 1, 0>},  {"store 2 lanes/piece a4", k_vm<2, 1, 0>},
        {"store 4 lanes/piece a4", k_vm<4, 1, 0>}, {"store 16 lanes/piece a4", k_vm<16, 1, 0>},
        {"store 1 lane/piece a16", k_vm<1, 1, 1>}, {"store 4 lanes/piece a16", k_vm<4, 1, 1>},
    };
    for (auto &k : ks) {
        const int iters = 64;
        hipLaunchKernelGGL(k.k, dim3(cus), dim3(256), 0, 0, buf, iters, out);
        if (hipDeviceSynchronize() != hipSuccess)
            return 2;
        unsigned long long h[4096];
        (void) hipMemcpy(h, out, nw * 8, hipMemcpyDeviceToHost);
        double s = 0;
        for (size_t w = 0; w < nw; ++w)
            s += (double) h[w];
        printf("%-26s %.1f cycles per instruction (mean over waves)\n", k.n, s / nw / iters / 8);
    }
    return 0;
}
