// Cost model of the frame kernel's loop, built up part by part (timing
// experiments only; outputs are not checked): config-2 geometry, 65,536
// frames of 1,057 wire bytes, G = 2 lanes per frame, 256-thread workgroups,
// 9 steps per lane.  F = feature bits: 1 input loads (a step ahead) + XOR,
// 2 input byte shift, 4 output stores (aligned, no shift), 8 output shift,
// 16 Poly1305 (parallel form, as curve_frames.hpp), 32 s_setprio schedule.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/bin/frames_proto tools/frames_proto.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include "../libzmq_amd/csrc/curve_frames.hpp"
using namespace zmqg;


// Poly1305 in radix 2^32 (h0..h3 words + h4 small), h = (h + m) * r with the
// clamped r (s_k = r_k + r_k/4): 19 v_mad_u64_u32 + 1 v_mul_lo_u32 per block
struct P32 { uint32_t h0, h1, h2, h3, h4; };
__device__ __forceinline__ void p32_block(P32 &h, uint32_t m0, uint32_t m1, uint32_t m2, uint32_t m3, uint32_t hib,
                                          uint32_t r0, uint32_t r1, uint32_t r2, uint32_t r3, uint32_t s1, uint32_t s2,
                                          uint32_t s3)
{
    uint64_t t = (uint64_t) h.h0 + m0;
    const uint32_t a0 = (uint32_t) t;
    t = (uint64_t) h.h1 + m1 + (t >> 32);
    const uint32_t a1 = (uint32_t) t;
    t = (uint64_t) h.h2 + m2 + (t >> 32);
    const uint32_t a2 = (uint32_t) t;
    t = (uint64_t) h.h3 + m3 + (t >> 32);
    const uint32_t a3 = (uint32_t) t;
    const uint32_t a4 = h.h4 + hib + (uint32_t) (t >> 32);
    uint64_t d0 = mad64(a3, s1, mad64(a2, s2, mad64(a1, s3, (uint64_t) a0 * r0)));
    uint64_t d1 = mad64(a4, s1, mad64(a3, s2, mad64(a2, s3, mad64(a1, r0, (uint64_t) a0 * r1))));
    uint64_t d2 = mad64(a4, s2, mad64(a3, s3, mad64(a2, r0, mad64(a1, r1, (uint64_t) a0 * r2))));
    uint64_t d3 = mad64(a4, s3, mad64(a3, r0, mad64(a2, r1, mad64(a1, r2, (uint64_t) a0 * r3))));
    uint32_t h4 = a4 * r0;
    h.h0 = (uint32_t) d0;
    d1 += d0 >> 32;
    h.h1 = (uint32_t) d1;
    d2 += d1 >> 32;
    h.h2 = (uint32_t) d2;
    d3 += d2 >> 32;
    h.h3 = (uint32_t) d3;
    h4 += (uint32_t) (d3 >> 32);
    const uint32_t c = (h4 >> 2) + (h4 & ~3u);
    h4 &= 3u;
    t = (uint64_t) h.h0 + c;
    h.h0 = (uint32_t) t;
    t = (uint64_t) h.h1 + (t >> 32);
    h.h1 = (uint32_t) t;
    t = (uint64_t) h.h2 + (t >> 32);
    h.h2 = (uint32_t) t;
    t = (uint64_t) h.h3 + (t >> 32);
    h.h3 = (uint32_t) t;
    h.h4 = h4 + (uint32_t) (t >> 32);
}

template <int F>
__global__ __launch_bounds__(256) void k_proto(uint32_t n, const uint8_t *__restrict__ in, uint8_t *__restrict__ out,
                                               const uint32_t *__restrict__ key_in, uint32_t *__restrict__ sink)
{
    constexpr int G = 2;
    const uint32_t gl = blockIdx.x * 256 + threadIdx.x, lane = threadIdx.x & 63;
    const uint32_t i = gl / G, q = gl % G;
    if (i >= n)
        return;
    uint32_t key[8];
#pragma unroll
    for (int t = 0; t < 8; ++t)
        key[t] = key_in[t];
    const uint32_t S = 1057, nw = 17;
    const uint64_t A = (uint64_t) (uintptr_t) in + (uint64_t) i * S;
    const uint64_t B = (uint64_t) (uintptr_t) out + (uint64_t) i * S;
    const uint32_t n0 = i, n1 = 0x01000000u;
    const uint32_t steps = (nw + G - 1) / G;
    uint32_t acc = 0;
    uint32_t dn[17];
    if (F & 1)
        frame_load_raw(A, q, S, dn);
    fe5 P1, P2, P3, P4, PG;
    uint64_t H[5] = {0, 0, 0, 0, 0};
    bool hasH = false;
    P32 h32 = {0, 0, 0, 0, 0};
    const uint32_t R0 = key_in[8] & 0x0fffffff, R1 = key_in[9] & 0x0ffffffc, R2 = key_in[10] & 0x0ffffffc,
                   R3 = key_in[11] & 0x0ffffffc, S1 = R1 + (R1 >> 2), S2 = R2 + (R2 >> 2), S3 = R3 + (R3 >> 2);
#pragma unroll 1
    for (uint32_t t = 0; t < steps; ++t) {
        if (F & 32) {
            if (4 * t < steps)
                __builtin_amdgcn_s_setprio(3);
            else if (2 * t < steps)
                __builtin_amdgcn_s_setprio(2);
            else if (4 * t < 3 * steps)
                __builtin_amdgcn_s_setprio(1);
            else
                __builtin_amdgcn_s_setprio(0);
        }
        const uint32_t w = t * G + q;
        const bool act = w < nw;
        uint32_t ks[16];
        salsa20_block(ks, key, n0, n1, w, 0);
        uint32_t x[16];
        if (F & 1) {
            uint32_t dc[17];
#pragma unroll
            for (int k = 0; k < 17; ++k)
                dc[k] = dn[k];
            if (w + G < nw)
                frame_load_raw(A, w + G, S, dn);
            if (F & 2) {
#pragma unroll
                for (int k = 0; k < 16; ++k)
                    x[k] = __builtin_amdgcn_alignbyte(dc[k + 1], dc[k], 1);
            } else {
#pragma unroll
                for (int k = 0; k < 16; ++k)
                    x[k] = dc[k];
            }
        } else {
#pragma unroll
            for (int k = 0; k < 16; ++k)
                x[k] = k;
        }
        if (t == 0) {
            const fe r0 = poly_r_from_key(ks[0], ks[1], ks[2], ks[3]);
            fe r;
#pragma unroll
            for (int k = 0; k < 5; ++k)
                r.l[k] = (uint32_t) __shfl((int) r0.l[k], (int) (lane - q));
            P1 = fe5_of(r);
            fe t2 = r;
            fe_mul(t2, r);
            P2 = fe5_of(t2);
            fe t3 = t2;
            fe_mul(t3, r);
            P3 = fe5_of(t3);
            fe t4 = t2;
            fe_mul(t4, t2);
            P4 = fe5_of(t4);
            fe tg = t4;
            fe_mul(tg, tg);
            PG = fe5_of(tg);
        }
        uint32_t y[16];
#pragma unroll
        for (int k = 0; k < 16; ++k)
            y[k] = x[k] ^ ks[k];
        if ((F & 16) && act && w < nw - 1) {
            uint64_t a[5] = {0, 0, 0, 0, 0};
            if (hasH) {
                uint32_t hh[5];
                const fe hf = fe_from_wide(H);
#pragma unroll
                for (int k = 0; k < 5; ++k)
                    hh[k] = hf.l[k];
                acc_mul(a, hh, PG);
            }
            uint32_t m[5];
            block_limbs(x, 16, m);
            acc_mul(a, m, P4);
            block_limbs(x + 4, 16, m);
            acc_mul(a, m, P3);
            block_limbs(x + 8, 16, m);
            acc_mul(a, m, P2);
            block_limbs(x + 12, 16, m);
            acc_mul(a, m, P1);
#pragma unroll
            for (int k = 0; k < 5; ++k)
                H[k] = a[k];
            hasH = true;
        }
        if ((F & 512) && act && w < nw - 1) {
#pragma unroll
            for (int j = 0; j < 4; ++j)
                p32_block(h32, x[4 * j], x[4 * j + 1], x[4 * j + 2], x[4 * j + 3], 1u, R0, R1, R2, R3, S1, S2, S3);
        }
        if ((F & 4) && act && w > 0) {
            if (F & 128) {
                GU4 *p = (GU4 *) (uintptr_t) ((uint64_t) (uintptr_t) out + 64ull * (lane & 7));
                __builtin_nontemporal_store((u32x4){y[0], y[1], y[2], y[3]}, (u32x4 *) p);
            } else if (F & 64) {
                GU4 *p = (GU4 *) (uintptr_t) ((B & ~15ull) + 64ull * w);
                p[0] = (u32x4){y[0] ^ y[4] ^ y[8] ^ y[12], y[1] ^ y[5] ^ y[9] ^ y[13], y[2] ^ y[6] ^ y[10] ^ y[14], y[3] ^ y[7] ^ y[11] ^ y[15]};
            } else if (F & 256) {
                u32x4 *p = (u32x4 *) (uintptr_t) ((B & ~15ull) + 64ull * w);
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    __builtin_nontemporal_store((u32x4){y[4 * k], y[4 * k + 1], y[4 * k + 2], y[4 * k + 3]}, p + k);
            } else if (F & 8) {
                const uint32_t y15 = y[15];
                const uint32_t yprev = (uint32_t) __shfl((int) y15, (int) (lane > 0 ? lane - 1 : 0));
                frame_store(B, w, S, y, yprev, false);
            } else {
                GU4 *p = (GU4 *) (uintptr_t) ((B & ~15ull) + 64ull * w);
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    p[k] = (u32x4){y[4 * k], y[4 * k + 1], y[4 * k + 2], y[4 * k + 3]};
            }
        } else {
#pragma unroll
            for (int k = 0; k < 16; ++k)
                acc ^= y[k];
        }
    }
    if (F & 512)
        acc ^= h32.h0 ^ h32.h4;
    if (F & 16) {
        const fe hf = fe_from_wide(H);
        acc ^= hf.l[0] ^ hf.l[4];
    }
    sink[gl] = acc;
}


// Segment mapping (lane q of a frame's G lanes takes a contiguous run of
// windows), sequential radix-2^32 Poly1305 per lane, loads for the next
// window and stores of this one issued together at the end of the step (so
// that the compiler's vmcnt wait at the next use comes after a whole Salsa20
// block).  SP = software-pipelined poly (window t-1's ciphertext in step t).
template <int G, int SP, int ALIGN>
__global__ __launch_bounds__(256) void k_seg(uint32_t n, const uint8_t *__restrict__ in, uint8_t *__restrict__ out,
                                             const uint32_t *__restrict__ key_in, uint32_t *__restrict__ sink)
{
    const uint32_t gl = blockIdx.x * 256 + threadIdx.x;
    const uint32_t i = gl / G, q = gl % G;
    if (i >= n)
        return;
    uint32_t key[8];
#pragma unroll
    for (int t = 0; t < 8; ++t)
        key[t] = key_in[t];
    const uint32_t S = 1057, nw = 17;
    const uint32_t a0 = q * nw / G, a1 = (q + 1) * nw / G;
    const uint64_t A = (uint64_t) (uintptr_t) in + (uint64_t) i * S;
    const uint64_t B = (uint64_t) (uintptr_t) out + 64 + (uint64_t) i * S;
    const uint32_t n0 = i, n1 = 0x01000000u;
    const uint32_t steps = (nw + G - 1) / G;
    const uint32_t R0 = key_in[8] & 0x0fffffff, R1 = key_in[9] & 0x0ffffffc, R2 = key_in[10] & 0x0ffffffc,
                   R3 = key_in[11] & 0x0ffffffc, S1 = R1 + (R1 >> 2), S2 = R2 + (R2 >> 2), S3 = R3 + (R3 >> 2);
    P32 h = {0, 0, 0, 0, 0};
    const uint32_t v = ALIGN ? 0u : (uint32_t) A & 3u;
    const uint64_t A4 = A & ~3ull;
    // raw words of the lane's current window: d[0..16] = aligned words 16w .. 16w+16
    uint32_t d[17];
    {
        const GCU4a4 *p = (const GCU4a4 *) (uintptr_t) (A4 + 64ull * a0);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const u32x4 t = p[k];
            d[4 * k] = t.x; d[4 * k + 1] = t.y; d[4 * k + 2] = t.z; d[4 * k + 3] = t.w;
        }
        d[16] = *(GCU32 *) (uintptr_t) (A4 + 64ull * a0 + 64);
    }
    uint32_t cprev[16];
    uint32_t ycarry = 0;
    uint32_t acc = 0;
#pragma unroll 1
    for (uint32_t t = 0; t < steps; ++t) {
        const uint32_t w = a0 + t;
        const bool act = w < a1;
        uint32_t ks[16];
        salsa20_block(ks, key, n0, n1, w, 0);
        uint32_t x[16];
#pragma unroll
        for (int k = 0; k < 16; ++k)
            x[k] = ALIGN ? d[k] : __builtin_amdgcn_alignbyte(d[k + 1], d[k], v);
        if (SP) {
            if (t > 0 && act)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    p32_block(h, cprev[4 * j], cprev[4 * j + 1], cprev[4 * j + 2], cprev[4 * j + 3], 1u, R0, R1, R2,
                              R3, S1, S2, S3);
#pragma unroll
            for (int k = 0; k < 16; ++k)
                cprev[k] = x[k];
        } else if (act) {
#pragma unroll
            for (int j = 0; j < 4; ++j)
                p32_block(h, x[4 * j], x[4 * j + 1], x[4 * j + 2], x[4 * j + 3], 1u, R0, R1, R2, R3, S1, S2, S3);
        }
        uint32_t y[16];
#pragma unroll
        for (int k = 0; k < 16; ++k)
            y[k] = x[k] ^ ks[k];
        // next window's words: d[0] = this window's d[16]; 16 more
        const uint32_t d16 = d[16];
        if (w + 1 < a1) {
            const GCU4a4 *p = (const GCU4a4 *) (uintptr_t) (A4 + 64ull * (w + 1) + 4);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const u32x4 tt = p[k];
                d[4 * k + 1] = tt.x; d[4 * k + 2] = tt.y; d[4 * k + 3] = tt.z; d[4 * k + 4] = tt.w;
            }
            d[0] = d16;
        }
        if (act) {
            if (ALIGN) {
                GU4 *p = (GU4 *) (uintptr_t) ((B & ~15ull) + 64ull * w);
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    p[k] = (u32x4){y[4 * k], y[4 * k + 1], y[4 * k + 2], y[4 * k + 3]};
            } else {
                const uint32_t u = (uint32_t) B & 3u, up = u ? u : 4u, sh = 4u - up;
                GU4a4 *p = (GU4a4 *) (uintptr_t) (B - up + 64ull * w);
                uint32_t o[16];
                o[0] = __builtin_amdgcn_alignbyte(y[0], ycarry, sh);
#pragma unroll
                for (int k = 1; k < 16; ++k)
                    o[k] = __builtin_amdgcn_alignbyte(y[k], y[k - 1], sh);
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    p[k] = (u32x4){o[4 * k], o[4 * k + 1], o[4 * k + 2], o[4 * k + 3]};
                ycarry = y[15];
            }
        }
    }
    if (SP)
#pragma unroll
        for (int j = 0; j < 4; ++j)
            p32_block(h, cprev[4 * j], cprev[4 * j + 1], cprev[4 * j + 2], cprev[4 * j + 3], 1u, R0, R1, R2, R3, S1, S2,
                      S3);
    acc ^= h.h0 ^ h.h1 ^ h.h4;
    sink[gl] = acc;
}


typedef __attribute__((address_space(3))) void LdsVoid;
typedef __attribute__((address_space(1))) void GVoid;
// One lane per frame with the wave's window I/O transposed through LDS: each
// global instruction moves 16 frames x 64 bytes (4 lanes per frame, 16 bytes
// each) instead of 64 frames x 16 bytes.  Loads by LDS-DMA (no VGPRs, issued
// a step ahead), stores through an LDS image written by the owner lanes.
// TIO: 1 transposed loads, 2 transposed stores.
template <int TIO>
__global__ __launch_bounds__(256) void k_seq_lds(uint32_t n, const uint8_t *__restrict__ in, uint8_t *__restrict__ out,
                                                 const uint32_t *__restrict__ key_in, uint32_t *__restrict__ sink)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[4 * 8192];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint8_t *const ibuf = lds + wv * 8192, *const obuf = ibuf + 4096;
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    uint32_t key[8];
#pragma unroll
    for (int t = 0; t < 8; ++t)
        key[t] = key_in[t];
    const uint32_t S = 1057, nw = 17;
    const uint64_t A = (uint64_t) (uintptr_t) in + (uint64_t) i * S;
    const uint64_t B = (uint64_t) (uintptr_t) out + 64 + (uint64_t) i * S;
    const uint32_t v = (uint32_t) A & 3u;
    const uint64_t A4 = A & ~3ull;
    const uint32_t u = (uint32_t) B & 3u, up = u ? u : 4u, sh = 4u - up;
    const uint32_t n0 = i, n1 = 0x01000000u;
    const PolyKey32 pk = poly32_key(key_in[8], key_in[9], key_in[10], key_in[11]);
    // transposed bases: for instruction k, this lane serves frame 16k + lane/4, chunk lane%4
    uint64_t gin[4], gout[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int src = 16 * k + (int) (lane >> 2);
        const uint32_t alo = (uint32_t) __shfl((int) (uint32_t) A4, src), ahi = (uint32_t) __shfl((int) (uint32_t) (A4 >> 32), src);
        const uint64_t bb = B - up;
        const uint32_t blo = (uint32_t) __shfl((int) (uint32_t) bb, src), bhi = (uint32_t) __shfl((int) (uint32_t) (bb >> 32), src);
        gin[k] = (((uint64_t) ahi << 32) | alo) + 4 + 16 * (lane & 3);
        gout[k] = (((uint64_t) bhi << 32) | blo) + 16 * (lane & 3);
    }
    uint32_t dd[16], d0 = *(const uint32_t *) (uintptr_t) (A4 + 64);
    u32x4 tq[4]; // TIO & 4: transposed granules in flight
    // window 1's words
    if (TIO & 4) {
#pragma unroll
        for (int k = 0; k < 4; ++k)
            tq[k] = *(const GCU4a4 *) (uintptr_t) (gin[k] + 64);
    } else if (TIO & 1) {
#pragma unroll
        for (int k = 0; k < 4; ++k)
            __builtin_amdgcn_global_load_lds((GVoid *) (uintptr_t) (gin[k] + 64), (LdsVoid *) (ibuf + 1024 * k), 16, 0, 0);
    } else {
        const GCU4a4 *p = (const GCU4a4 *) (uintptr_t) (A4 + 64 + 4);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const u32x4 tt = p[k];
            dd[4 * k] = tt.x; dd[4 * k + 1] = tt.y; dd[4 * k + 2] = tt.z; dd[4 * k + 3] = tt.w;
        }
    }
    Poly32 h = {0, 0, 0, 0, 0};
    uint32_t cp[16];
#pragma unroll
    for (int k = 0; k < 16; ++k)
        cp[k] = 0;
    uint32_t ycarry = 0, acc = 0;
#pragma unroll 1
    for (uint32_t t = 1; t < nw - 1; ++t) {
        uint32_t ks[16];
        salsa20_block(ks, key, n0, n1, t, 0);
        if (t > 1)
            poly32_window_full(h, pk, cp);
#pragma unroll
        for (int k = 0; k < 16; ++k)
            asm volatile("" : "+v"(ks[k]));
        if (TIO & 4) {
#pragma unroll
            for (int k = 0; k < 4; ++k)
                *(u32x4 *) (ibuf + 1024 * k + 16 * lane) = tq[k];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const u32x4 tt = *(const u32x4 *) (ibuf + 64 * lane + 16 * k);
                dd[4 * k] = tt.x; dd[4 * k + 1] = tt.y; dd[4 * k + 2] = tt.z; dd[4 * k + 3] = tt.w;
            }
        } else if (TIO & 1) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const u32x4 tt = *(const u32x4 *) (ibuf + 64 * lane + 16 * k);
                dd[4 * k] = tt.x; dd[4 * k + 1] = tt.y; dd[4 * k + 2] = tt.z; dd[4 * k + 3] = tt.w;
            }
        }
        uint32_t x[16];
        x[0] = __builtin_amdgcn_alignbyte(dd[0], d0, v);
#pragma unroll
        for (int k = 1; k < 16; ++k)
            x[k] = __builtin_amdgcn_alignbyte(dd[k], dd[k - 1], v);
        d0 = dd[15];
        uint32_t y[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            y[k] = x[k] ^ ks[k];
            cp[k] = x[k];
        }
        // next window's words
        if (TIO & 4) {
#pragma unroll
            for (int k = 0; k < 4; ++k)
                tq[k] = *(const GCU4a4 *) (uintptr_t) (gin[k] + 64ull * (t + 1));
        } else if (TIO & 1) {
            __builtin_amdgcn_s_waitcnt(0xc07f); // lgkmcnt(0): this window's LDS reads are done
#pragma unroll
            for (int k = 0; k < 4; ++k)
                __builtin_amdgcn_global_load_lds((GVoid *) (uintptr_t) (gin[k] + 64ull * (t + 1)),
                                                 (LdsVoid *) (ibuf + 1024 * k), 16, 0, 0);
        } else {
            const GCU4a4 *p = (const GCU4a4 *) (uintptr_t) (A4 + 64ull * (t + 1) + 4);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const u32x4 tt = p[k];
                dd[4 * k] = tt.x; dd[4 * k + 1] = tt.y; dd[4 * k + 2] = tt.z; dd[4 * k + 3] = tt.w;
            }
        }
        // this window's output words (aligned to B - up + 64t)
        uint32_t o[16];
        o[0] = __builtin_amdgcn_alignbyte(y[0], ycarry, sh);
#pragma unroll
        for (int k = 1; k < 16; ++k)
            o[k] = __builtin_amdgcn_alignbyte(y[k], y[k - 1], sh);
        ycarry = y[15];
        if (TIO & 2) {
#pragma unroll
            for (int k = 0; k < 4; ++k)
                *(u32x4 *) (obuf + 64 * lane + 16 * k) = (u32x4){o[4 * k], o[4 * k + 1], o[4 * k + 2], o[4 * k + 3]};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const u32x4 tt = *(const u32x4 *) (obuf + 1024 * k + 16 * lane);
                *(GU4a4 *) (uintptr_t) (gout[k] + 64ull * t) = tt;
            }
        } else {
            GU4a4 *p = (GU4a4 *) (uintptr_t) (B - up + 64ull * t);
#pragma unroll
            for (int k = 0; k < 4; ++k)
                p[k] = (u32x4){o[4 * k], o[4 * k + 1], o[4 * k + 2], o[4 * k + 3]};
        }
    }
    poly32_window_full(h, pk, cp);
    acc ^= h.h0 ^ h.h4;
    sink[i] = acc;
}


// The same with both directions transposed and software-pipelined: step t
// reads its own input words from LDS (written at the end of step t-1) and
// the transposed image of window t-1's output (stores them), runs the
// keystream, writes window t's output image, then moves the transposed
// granules of window t+1 (loaded a step earlier) into LDS and loads those
// of window t+2.
__global__ __launch_bounds__(256) void k_seq_pipe(uint32_t n, const uint8_t *__restrict__ in, uint8_t *__restrict__ out,
                                                  const uint32_t *__restrict__ key_in, uint32_t *__restrict__ sink)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[4 * 8192];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint8_t *const ibuf = lds + wv * 8192, *const obuf = ibuf + 4096;
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    uint32_t key[8];
#pragma unroll
    for (int t = 0; t < 8; ++t)
        key[t] = key_in[t];
    const uint32_t S = 1057, nw = 17;
    const uint64_t A = (uint64_t) (uintptr_t) in + (uint64_t) i * S;
    const uint64_t B = (uint64_t) (uintptr_t) out + 64 + (uint64_t) i * S;
    const uint32_t v = (uint32_t) A & 3u;
    const uint64_t A4 = A & ~3ull;
    const uint32_t u = (uint32_t) B & 3u, up = u ? u : 4u, sh = 4u - up;
    const uint32_t n0 = i, n1 = 0x01000000u;
    const PolyKey32 pk = poly32_key(key_in[8], key_in[9], key_in[10], key_in[11]);
    uint64_t gin[4], gout[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int src = 16 * k + (int) (lane >> 2);
        const uint32_t alo = (uint32_t) __shfl((int) (uint32_t) A4, src), ahi = (uint32_t) __shfl((int) (uint32_t) (A4 >> 32), src);
        const uint64_t bb = B - up;
        const uint32_t blo = (uint32_t) __shfl((int) (uint32_t) bb, src), bhi = (uint32_t) __shfl((int) (uint32_t) (bb >> 32), src);
        gin[k] = (((uint64_t) ahi << 32) | alo) + 4 + 16 * (lane & 3);
        gout[k] = (((uint64_t) bhi << 32) | blo) + 16 * (lane & 3);
    }
    uint32_t d0 = *(const uint32_t *) (uintptr_t) (A4 + 64);
    u32x4 tq[4];
    // window 1 into LDS now, window 2 in flight
#pragma unroll
    for (int k = 0; k < 4; ++k)
        tq[k] = *(const GCU4a4 *) (uintptr_t) (gin[k] + 64);
#pragma unroll
    for (int k = 0; k < 4; ++k)
        *(u32x4 *) (ibuf + 1024 * k + 16 * lane) = tq[k];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        tq[k] = *(const GCU4a4 *) (uintptr_t) (gin[k] + 128);
    Poly32 h = {0, 0, 0, 0, 0};
    uint32_t cp[16];
#pragma unroll
    for (int k = 0; k < 16; ++k)
        cp[k] = 0;
    uint32_t ycarry = 0, acc = 0;
#pragma unroll 1
    for (uint32_t t = 1; t < nw - 1; ++t) {
        // own input words of window t
        uint32_t dd[16];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const u32x4 tt = *(const u32x4 *) (ibuf + 64 * lane + 16 * k);
            dd[4 * k] = tt.x; dd[4 * k + 1] = tt.y; dd[4 * k + 2] = tt.z; dd[4 * k + 3] = tt.w;
        }
        // window t-1's output, transposed
        if (t > 1) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const u32x4 tt = *(const u32x4 *) (obuf + 1024 * k + 16 * lane);
                *(GU4a4 *) (uintptr_t) (gout[k] + 64ull * (t - 1)) = tt;
            }
        }
        uint32_t ks[16];
        salsa20_block(ks, key, n0, n1, t, 0);
        if (t > 1)
            poly32_window_full(h, pk, cp);
#pragma unroll
        for (int k = 0; k < 16; ++k)
            asm volatile("" : "+v"(ks[k]));
        uint32_t x[16];
        x[0] = __builtin_amdgcn_alignbyte(dd[0], d0, v);
#pragma unroll
        for (int k = 1; k < 16; ++k)
            x[k] = __builtin_amdgcn_alignbyte(dd[k], dd[k - 1], v);
        d0 = dd[15];
        uint32_t y[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            y[k] = x[k] ^ ks[k];
            cp[k] = x[k];
        }
        uint32_t o[16];
        o[0] = __builtin_amdgcn_alignbyte(y[0], ycarry, sh);
#pragma unroll
        for (int k = 1; k < 16; ++k)
            o[k] = __builtin_amdgcn_alignbyte(y[k], y[k - 1], sh);
        ycarry = y[15];
#pragma unroll
        for (int k = 0; k < 4; ++k)
            *(u32x4 *) (obuf + 64 * lane + 16 * k) = (u32x4){o[4 * k], o[4 * k + 1], o[4 * k + 2], o[4 * k + 3]};
        // window t+1's granules into LDS, window t+2's loaded
#pragma unroll
        for (int k = 0; k < 4; ++k)
            *(u32x4 *) (ibuf + 1024 * k + 16 * lane) = tq[k];
        if (t + 2 < nw)
#pragma unroll
            for (int k = 0; k < 4; ++k)
                tq[k] = *(const GCU4a4 *) (uintptr_t) (gin[k] + 64ull * (t + 2));
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const u32x4 tt = *(const u32x4 *) (obuf + 1024 * k + 16 * lane);
        *(GU4a4 *) (uintptr_t) (gout[k] + 64ull * (nw - 2)) = tt;
    }
    poly32_window_full(h, pk, cp);
    acc ^= h.h0 ^ h.h4;
    sink[i] = acc;
}


// One lane per frame, VMEM spread through the keystream: step t issues the
// stores of window t-1 and the loads of window t+1 (double-buffered words)
// inside its Salsa20 block, interleaved by sched_group_barrier (IL = VALU
// instructions between two VMEM instructions; 0 = no interleave hint).
template <int IL>
__global__ __launch_bounds__(256) void k_seq_il(uint32_t n, const uint8_t *__restrict__ in, uint8_t *__restrict__ out,
                                                const uint32_t *__restrict__ key_in, uint32_t *__restrict__ sink)
{
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    uint32_t key[8];
#pragma unroll
    for (int t = 0; t < 8; ++t)
        key[t] = key_in[t];
    const uint32_t S = 1057, nw = 17;
    const uint64_t A = (uint64_t) (uintptr_t) in + (uint64_t) i * S;
    const uint64_t B = (uint64_t) (uintptr_t) out + 64 + (uint64_t) i * S;
    const uint32_t v = (uint32_t) A & 3u;
    const uint64_t A4 = A & ~3ull;
    const uint32_t u = (uint32_t) B & 3u, up = u ? u : 4u, sh = 4u - up;
    const uint32_t n0 = i, n1 = 0x01000000u;
    const PolyKey32 pk = poly32_key(key_in[8], key_in[9], key_in[10], key_in[11]);
    uint32_t d0 = *(const uint32_t *) (uintptr_t) (A4 + 64);
    uint32_t ddA[16], ddB[16];
    auto ld = [&](uint32_t w, uint32_t (&dd)[16]) {
        const GCU4a4 *p = (const GCU4a4 *) (uintptr_t) (A4 + 64ull * w + 4);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const u32x4 tt = p[k];
            dd[4 * k] = tt.x; dd[4 * k + 1] = tt.y; dd[4 * k + 2] = tt.z; dd[4 * k + 3] = tt.w;
        }
    };
    ld(1, ddA);
    Poly32 h = {0, 0, 0, 0, 0};
    uint32_t cp[16], o[16];
#pragma unroll
    for (int k = 0; k < 16; ++k)
        cp[k] = o[k] = 0;
    uint32_t ycarry = 0, acc = 0;
    auto step = [&](uint32_t t, uint32_t (&cur)[16], uint32_t (&nxt)[16]) {
        // window t+1's loads and window t-1's stores, then the keystream
        if (t + 1 < nw - 1)
            ld(t + 1, nxt);
        if (t > 1) {
            GU4a4 *p = (GU4a4 *) (uintptr_t) (B - up + 64ull * (t - 1));
#pragma unroll
            for (int k = 0; k < 4; ++k)
                p[k] = (u32x4){o[4 * k], o[4 * k + 1], o[4 * k + 2], o[4 * k + 3]};
        }
        uint32_t ks[16];
        salsa20_block(ks, key, n0, n1, t, 0);
        if (t > 1)
            poly32_window_full(h, pk, cp);
        if (IL) {
#pragma unroll
            for (int g = 0; g < 8; ++g) {
                __builtin_amdgcn_sched_group_barrier(0x020 | 0x040, 1, 0); // one VMEM read or write
                __builtin_amdgcn_sched_group_barrier(0x002, IL, 0);        // IL VALU
            }
        }
#pragma unroll
        for (int k = 0; k < 16; ++k)
            asm volatile("" : "+v"(ks[k]));
        uint32_t x[16];
        x[0] = __builtin_amdgcn_alignbyte(cur[0], d0, v);
#pragma unroll
        for (int k = 1; k < 16; ++k)
            x[k] = __builtin_amdgcn_alignbyte(cur[k], cur[k - 1], v);
        d0 = cur[15];
        uint32_t y[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            y[k] = x[k] ^ ks[k];
            cp[k] = x[k];
        }
        o[0] = __builtin_amdgcn_alignbyte(y[0], ycarry, sh);
#pragma unroll
        for (int k = 1; k < 16; ++k)
            o[k] = __builtin_amdgcn_alignbyte(y[k], y[k - 1], sh);
        ycarry = y[15];
    };
#pragma unroll 1
    for (uint32_t t = 1; t + 1 < nw - 1; t += 2) {
        step(t, ddA, ddB);
        step(t + 1, ddB, ddA);
    }
    {
        GU4a4 *p = (GU4a4 *) (uintptr_t) (B - up + 64ull * (nw - 2));
#pragma unroll
        for (int k = 0; k < 4; ++k)
            p[k] = (u32x4){o[4 * k], o[4 * k + 1], o[4 * k + 2], o[4 * k + 3]};
    }
    poly32_window_full(h, pk, cp);
    acc ^= h.h0 ^ h.h4;
    sink[i] = acc;
}

typedef void (*KF)(uint32_t, const uint8_t *, uint8_t *, const uint32_t *, uint32_t *);
int main(int argc, char **argv)
{
    const uint32_t n = 65536;
    uint8_t *in, *out;
    uint32_t *key, *sink;
    if (hipMalloc(&in, (size_t) n * 1057 + 256) || hipMalloc(&out, (size_t) n * 1057 + 512) ||
        hipMalloc(&key, 64) || hipMalloc(&sink, 4 * 2 * n))
        return 1;
    (void) hipMemset(in, 0x5a, (size_t) n * 1057 + 256);
    (void) hipMemset(key, 0x33, 64);
    struct { const char *name; KF k; int gmul; } ks[] = {
        {"salsa only", k_proto<0>, 2},         {"+loads", k_proto<1>, 2},          {"+loads+shift", k_proto<3>, 2},
        {"+loads+shift+store", k_proto<7>, 2}, {"+... +store shift", k_proto<15>, 2}, {"+... +poly", k_proto<31>, 2},
        {"+... poly32 (no poly26)", k_proto<15 + 512>, 2}, {"salsa+poly26", k_proto<16>, 2}, {"salsa+poly32", k_proto<512>, 2},
        {"loads+store x1", k_proto<1 + 4 + 64>, 2}, {"loads+store same addr", k_proto<1 + 4 + 128>, 2},
        {"loads+store nt", k_proto<1 + 4 + 256>, 2}, {"loads+store", k_proto<1 + 4>, 2},
        {"seg G2", k_seg<2, 0, 0>, 2}, {"seg G2 SP", k_seg<2, 1, 0>, 2}, {"seg G2 aligned", k_seg<2, 0, 1>, 2},
        {"seg G1", k_seg<1, 0, 0>, 2}, {"seg G1 SP", k_seg<1, 1, 0>, 2}, {"seg G4", k_seg<4, 0, 0>, 2},
        {"seg G1 SP grid1", k_seg<1, 1, 0>, 1}, {"seg G1 grid1", k_seg<1, 0, 0>, 1},
        {"seqlds direct", k_seq_lds<0>, 1}, {"seqlds T-loads", k_seq_lds<1>, 1}, {"seqlds T-stores", k_seq_lds<2>, 1},
        {"seqlds T-both", k_seq_lds<3>, 1}, {"seqlds T-vloads", k_seq_lds<4>, 1},
        {"seqlds T-vloads+T-stores", k_seq_lds<6>, 1}, {"seq pipe", k_seq_pipe, 1},
        {"seq il0", k_seq_il<0>, 1}, {"seq il60", k_seq_il<60>, 1}, {"seq il110", k_seq_il<110>, 1},
    };
    hipEvent_t a, b;
    (void) hipEventCreate(&a);
    (void) hipEventCreate(&b);
    const int reps = 20;
    for (auto &k : ks) {
        const dim3 grid((n * k.gmul + 255) / 256);
        hipLaunchKernelGGL(k.k, grid, dim3(256), 0, 0, n, in, out, key, sink);
        if (hipDeviceSynchronize() != hipSuccess) {
            printf("%s: launch failed: %s\n", k.name, hipGetErrorString(hipGetLastError()));
            return 2;
        }
        (void) hipEventRecord(a, 0);
        for (int r = 0; r < reps; ++r)
            hipLaunchKernelGGL(k.k, grid, dim3(256), 0, 0, n, in, out, key, sink);
        (void) hipEventRecord(b, 0);
        if (hipEventSynchronize(b) != hipSuccess)
            return 3;
        float ms = 0;
        (void) hipEventElapsedTime(&ms, a, b);
        printf("%-24s %.1f us\n", k.name, ms * 1000 / reps);
        fflush(stdout);
    }
    return 0;
}
