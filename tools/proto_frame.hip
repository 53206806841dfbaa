// Prototype: one lane per frame, the whole frame (keystream block 0, every
// window, Poly1305 serially, tag) in one kernel, with unaligned 16-byte
// global loads/stores.  Checks against libzmqg_curve.so and times both.
// Build: hipcc -O3 --offload-arch=gfx950 -o build/proto_frame tools/proto_frame.hip -Llibzmq_amd -lzmqg_curve
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

#include "../include/zmqg_curve.h"
#include "../libzmq_amd/csrc/curve_device.hpp"

using namespace zmqg;

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

typedef u32x4 u32x4_u __attribute__((aligned(1)));
typedef __attribute__((address_space(1))) const u32x4_u GCU4u;
typedef __attribute__((address_space(1))) u32x4_u GU4u;

__device__ __forceinline__ void ld64(const uint8_t *p, uint32_t w[16])
{
    const GCU4u *q = (const GCU4u *) (uintptr_t) p;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const u32x4 v = q[k];
        w[4 * k] = v.x;
        w[4 * k + 1] = v.y;
        w[4 * k + 2] = v.z;
        w[4 * k + 3] = v.w;
    }
}

__device__ __forceinline__ void st64(uint8_t *p, const uint32_t w[16])
{
    GU4u *q = (GU4u *) (uintptr_t) p;
#pragma unroll
    for (int k = 0; k < 4; ++k)
        q[k] = (u32x4){w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]};
}

__device__ __forceinline__ uint32_t pt_header(uint32_t msg_flags, uint32_t hw[3])
{
    hw[0] = msg_flags & 3;
    hw[1] = hw[2] = 0;
    return 1;
}

template <int HL>
__device__ __forceinline__ void shift_in(const uint32_t p[16], uint32_t out[8])
{
    constexpr int A = HL >> 2, B = HL & 3;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint32_t hi = (i - A >= 0) ? p[i - A] : 0u;
        const uint32_t lo = (i - A - 1 >= 0) ? p[i - A - 1] : 0u;
        out[i] = B == 0 ? hi : __builtin_amdgcn_alignbyte(hi, lo, 4 - B);
    }
}

// encode, normal messages only (hl = 1) for the prototype
template <int MODE>
__global__ __launch_bounds__(256) void k_enc_frame(uint32_t n, const uint32_t *__restrict__ keys,
                                                   const uint64_t *__restrict__ nonce,
                                                   const uint8_t *__restrict__ flags,
                                                   const uint64_t *__restrict__ in_off,
                                                   const uint32_t *__restrict__ len, const uint8_t *__restrict__ in,
                                                   const uint64_t *__restrict__ out_off, uint8_t *__restrict__ out)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    uint32_t key[8];
#pragma unroll
    for (int t = 0; t < 8; ++t)
        key[t] = keys[t];
    const uint64_t nc = nonce[i];
    const uint32_t n0 = bswap32((uint32_t) (nc >> 32)), n1 = bswap32((uint32_t) nc);
    const uint32_t P = len[i];
    const uint32_t hl = 1, mlen = P + 1, S = mlen + 32;
    const uint8_t *src = in + in_off[i];
    uint8_t *o = out + out_off[i];

    uint32_t ks[16];
    salsa20_block(ks, key, n0, n1, 0, 0);
    const fe r = poly_r_from_key(ks[0], ks[1], ks[2], ks[3]);
    const uint32_t s1 = r.l[1] * 5, s2 = r.l[2] * 5, s3 = r.l[3] * 5, s4 = r.l[4] * 5;
    uint32_t pw16[16];
    load_window(src, P < 32 ? (int) P : 32, pw16);
    uint32_t pt[8];
    shift_in<1>(pw16, pt);
    pt[0] |= flags[i] & 3;
    const int nv0 = mlen < 32 ? (int) mlen : 32;
    uint32_t ct[16];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        ct[t] = pt[t] ^ ks[8 + t];
        ct[8 + t] = 0;
    }
    mask_tail(ct, nv0);
    store_window(o + 32, nv0, ct);
    fe h = fe_zero();
    poly_absorb64(h, r, s1, s2, s3, s4, ct, nv0);
    const uint32_t spad[4] = {ks[4], ks[5], ks[6], ks[7]};

    const uint32_t nw = (S + 63) >> 6;
    uint32_t d[16];
    if (nw > 1) {
        if (S >= 128)
            ld64(src + 64 - 32 - hl, d);
        else
            load_window(src + 64 - 32 - hl, (int) (S - 64), d);
    }
#pragma unroll 1
    for (uint32_t w = 1; w < nw; ++w) {
        const uint32_t nv = S - 64 * w >= 64 ? 64 : S - 64 * w;
        uint32_t x[16];
#pragma unroll
        for (int q = 0; q < 16; ++q)
            x[q] = d[q];
        if (w + 1 < nw) { // prefetch the next window
            const uint32_t nv2 = S - 64 * (w + 1);
            if (nv2 >= 64)
                ld64(src + 64 * (w + 1) - 32 - hl, d);
            else
                load_window(src + 64 * (w + 1) - 32 - hl, (int) nv2, d);
        }
        if (MODE & 2) {
#pragma unroll
            for (int q = 0; q < 16; ++q)
                ks[q] = w * 977 + q;
        } else
            salsa20_block(ks, key, n0, n1, w, 0);
#pragma unroll
        for (int q = 0; q < 16; ++q)
            x[q] ^= ks[q];
        if (nv == 64) {
            st64(o + 64 * w, x);
            if (MODE & 1)
                h.l[0] ^= x[0] ^ x[5] ^ x[10] ^ x[15];
            else
                poly_absorb64(h, r, s1, s2, s3, s4, x, 64);
        } else {
            mask_tail(x, (int) nv);
            store_window(o + 64 * w, (int) nv, x);
            poly_absorb64(h, r, s1, s2, s3, s4, x, (int) nv);
        }
    }
    uint32_t tag[4];
    poly_finish(h, spad, tag);
    uint32_t hdr[16] = {0x53454d07u, 0x45474153u, n0, n1, tag[0], tag[1], tag[2], tag[3]};
    store_window(o, 32, hdr);
}

__global__ __launch_bounds__(256) void k_dec_frame(uint32_t n, const uint32_t *__restrict__ keys,
                                                   const uint64_t *__restrict__ in_off,
                                                   const uint32_t *__restrict__ wire_len,
                                                   const uint8_t *__restrict__ in,
                                                   const uint64_t *__restrict__ out_off, uint8_t *__restrict__ out,
                                                   uint8_t *__restrict__ flags_out, int32_t *__restrict__ status_out)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    uint32_t key[8];
#pragma unroll
    for (int t = 0; t < 8; ++t)
        key[t] = keys[t];
    const uint32_t S = wire_len[i];
    const uint8_t *src = in + in_off[i];
    uint8_t *dst = out + out_off[i];
    uint32_t w0[16];
    load_window(src, S < 64 ? (int) S : 64, w0);
    int32_t status = 0;
    if (S < 33 || w0[0] != 0x53454d07u || w0[1] != 0x45474153u)
        status = ZMQG_ERR_UNEXPECTED_COMMAND;
    const uint32_t n0 = w0[2], n1 = w0[3];
    uint32_t ks[16];
    salsa20_block(ks, key, n0, n1, 0, 0);
    const fe r = poly_r_from_key(ks[0], ks[1], ks[2], ks[3]);
    const uint32_t s1 = r.l[1] * 5, s2 = r.l[2] * 5, s3 = r.l[3] * 5, s4 = r.l[4] * 5;
    const uint32_t mlen = S - 32;
    const int nv0 = mlen < 32 ? (int) mlen : 32;
    uint32_t ct[16];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        ct[t] = w0[8 + t];
        ct[8 + t] = 0;
    }
    fe h = fe_zero();
    poly_absorb64(h, r, s1, s2, s3, s4, ct, nv0);
    uint32_t pt[16];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        pt[t] = ct[t] ^ ks[8 + t];
        pt[8 + t] = 0;
    }
    mask_tail(pt, nv0);
    uint32_t pay[16];
#pragma unroll
    for (int t = 0; t < 15; ++t)
        pay[t] = __builtin_amdgcn_alignbyte(pt[t + 1], pt[t], 1);
    pay[15] = 0;
    store_window(dst, nv0 - 1, pay);
    const uint32_t fl = pt[0] & 3;
    const uint32_t spad[4] = {ks[4], ks[5], ks[6], ks[7]};
    const uint32_t wtag[4] = {w0[4], w0[5], w0[6], w0[7]};

    const uint32_t nw = (S + 63) >> 6;
    uint32_t d[16];
    if (nw > 1) {
        if (S >= 128)
            ld64(src + 64, d);
        else
            load_window(src + 64, (int) (S - 64), d);
    }
#pragma unroll 1
    for (uint32_t w = 1; w < nw; ++w) {
        const uint32_t nv = S - 64 * w >= 64 ? 64 : S - 64 * w;
        uint32_t x[16];
#pragma unroll
        for (int q = 0; q < 16; ++q)
            x[q] = d[q];
        if (w + 1 < nw) {
            const uint32_t nv2 = S - 64 * (w + 1);
            if (nv2 >= 64)
                ld64(src + 64 * (w + 1), d);
            else
                load_window(src + 64 * (w + 1), (int) nv2, d);
        }
        salsa20_block(ks, key, n0, n1, w, 0);
        poly_absorb64(h, r, s1, s2, s3, s4, x, (int) nv);
#pragma unroll
        for (int q = 0; q < 16; ++q)
            x[q] ^= ks[q];
        if (nv == 64) {
            st64(dst + 64 * w - 33, x);
        } else {
            mask_tail(x, (int) nv);
            store_window(dst + 64 * w - 33, (int) nv, x);
        }
    }
    uint32_t tag[4];
    poly_finish(h, spad, tag);
    if (status == 0 && ((tag[0] ^ wtag[0]) | (tag[1] ^ wtag[1]) | (tag[2] ^ wtag[2]) | (tag[3] ^ wtag[3])))
        status = ZMQG_ERR_CRYPTOGRAPHIC;
    status_out[i] = status;
    flags_out[i] = status == 0 ? fl : 0;
}

// ---------------------------------------------------------------- v2: LDS-transposed windows
constexpr int kSlotB = 80; // LDS bytes per frame slot (64 + 16 pad: conflict-free per-lane b128 reads)

__device__ __forceinline__ uint32_t wave_max(uint32_t v)
{
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const uint32_t o = __shfl_xor(v, d);
        v = o > v ? o : v;
    }
    return __builtin_amdgcn_readfirstlane(v);
}

__device__ __forceinline__ void lds_fence()
{
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}

// bytes [0, cnt) of an (unaligned) 16-byte granule, zero beyond; cnt in 0..16
__device__ __forceinline__ u32x4 load_gran(const uint8_t *p, uint32_t cnt)
{
    if (cnt >= 16)
        return *(const GCU4u *) (uintptr_t) p;
    uint32_t w[4] = {0, 0, 0, 0};
    for (uint32_t b = 0; b < cnt; ++b)
        w[b >> 2] |= (uint32_t) p[b] << (8 * (b & 3));
    return (u32x4){w[0], w[1], w[2], w[3]};
}

__device__ __forceinline__ void store_gran(uint8_t *p, uint32_t cnt, u32x4 v)
{
    if (cnt >= 16) {
        *(GU4u *) (uintptr_t) p = v;
        return;
    }
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    for (uint32_t b = 0; b < cnt; ++b)
        p[b] = (uint8_t) (w[b >> 2] >> (8 * (b & 3)));
}

__device__ __forceinline__ uint32_t gran_cnt(uint32_t S, uint32_t off)
{
    return S > off ? (S - off >= 16 ? 16u : S - off) : 0u;
}

template <bool DEC>
__global__ __launch_bounds__(256) void k_frame2(uint32_t n, const uint32_t *__restrict__ keys,
                                                const uint64_t *__restrict__ nonce, const uint8_t *__restrict__ flags,
                                                const uint64_t *__restrict__ in_off,
                                                const uint32_t *__restrict__ len, const uint8_t *__restrict__ in,
                                                const uint64_t *__restrict__ out_off, uint8_t *__restrict__ out,
                                                uint8_t *__restrict__ flags_out, int32_t *__restrict__ status_out)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[4 * 64 * kSlotB];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint8_t *const wl = lds + wv * 64 * kSlotB;
    uint8_t *const myslot = wl + lane * kSlotB;
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    const bool valid = i < n;
    const uint32_t ii = valid ? i : n - 1;
    uint32_t key[8];
#pragma unroll
    for (int t = 0; t < 8; ++t)
        key[t] = keys[t];
    const uint8_t *src = in + in_off[ii];
    uint8_t *dst = out + out_off[ii];
    uint32_t S, n0, n1, nv0;
    uint32_t ct[16];
    fe h = fe_zero(), r;
    uint32_t spad[4], wtag[4] = {0, 0, 0, 0}, fl = 0;
    int32_t status = 0;
    uint32_t ks[16];
    const uint8_t *cin_base; // stream byte 0 of the input
    uint8_t *cout_base;      // stream byte 0 of the output
    if (!DEC) {
        const uint64_t nc = nonce[ii];
        n0 = bswap32((uint32_t) (nc >> 32));
        n1 = bswap32((uint32_t) nc);
        const uint32_t P = len[ii];
        const uint32_t mlen = P + 1;
        S = valid ? mlen + 32 : 0;
        salsa20_block(ks, key, n0, n1, 0, 0);
        r = poly_r_from_key(ks[0], ks[1], ks[2], ks[3]);
        uint32_t pw16[16];
        load_window(src, P < 32 ? (int) P : 32, pw16);
        uint32_t pt[8];
        shift_in<1>(pw16, pt);
        pt[0] |= flags[ii] & 3;
        nv0 = mlen < 32 ? mlen : 32;
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            ct[t] = pt[t] ^ ks[8 + t];
            ct[8 + t] = 0;
        }
        mask_tail(ct, (int) nv0);
        if (valid)
            store_window(dst + 32, (int) nv0, ct);
        cin_base = src - 33;
        cout_base = dst;
    } else {
        const uint32_t wlen = len[ii];
        S = valid ? wlen : 0;
        uint32_t w0[16];
        load_window(src, wlen < 64 ? (int) wlen : 64, w0);
        if (wlen < 33 || w0[0] != 0x53454d07u || w0[1] != 0x45474153u)
            status = ZMQG_ERR_UNEXPECTED_COMMAND;
        n0 = w0[2];
        n1 = w0[3];
        salsa20_block(ks, key, n0, n1, 0, 0);
        r = poly_r_from_key(ks[0], ks[1], ks[2], ks[3]);
        const uint32_t mlen = wlen - 32;
        nv0 = mlen < 32 ? mlen : 32;
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            ct[t] = w0[8 + t];
            ct[8 + t] = 0;
            wtag[t & 3] = w0[4 + (t & 3)];
        }
        uint32_t pt[16];
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            pt[t] = ct[t] ^ ks[8 + t];
            pt[8 + t] = 0;
        }
        mask_tail(pt, (int) nv0);
        uint32_t pay[16];
#pragma unroll
        for (int t = 0; t < 15; ++t)
            pay[t] = __builtin_amdgcn_alignbyte(pt[t + 1], pt[t], 1);
        pay[15] = 0;
        if (valid)
            store_window(dst, (int) nv0 - 1, pay);
        fl = pt[0] & 3;
        cin_base = src;
        cout_base = dst - 33;
    }
    const uint32_t s1 = r.l[1] * 5, s2 = r.l[2] * 5, s3 = r.l[3] * 5, s4 = r.l[4] * 5;
    poly_absorb64(h, r, s1, s2, s3, s4, ct, (int) nv0);
#pragma unroll
    for (int t = 0; t < 4; ++t)
        spad[t] = ks[4 + t];

    const uint32_t nw = (S + 63) >> 6;
    const uint32_t nwmax = wave_max(nw);
    // cooperative granules: round k moves granule g of the frame in lane fr
    const uint32_t g = lane & 3;
    const uint64_t ib = (uint64_t) (uintptr_t) cin_base, ob = (uint64_t) (uintptr_t) cout_base;
    uint64_t cin[4], cout[4];
    uint32_t cS[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int fr = 16 * k + (int) (lane >> 2);
        cin[k] = ((uint64_t) (uint32_t) __shfl((uint32_t) (ib >> 32), fr) << 32) | (uint32_t) __shfl((uint32_t) ib, fr);
        cout[k] = ((uint64_t) (uint32_t) __shfl((uint32_t) (ob >> 32), fr) << 32) | (uint32_t) __shfl((uint32_t) ob, fr);
        cS[k] = (uint32_t) __shfl(S, fr);
        cin[k] += 16 * g;
        cout[k] += 16 * g;
    }
    u32x4 pre[4];
    if (nwmax > 1) {
#pragma unroll
        for (int k = 0; k < 4; ++k)
            pre[k] = load_gran((const uint8_t *) (uintptr_t) (cin[k] + 64), gran_cnt(cS[k], 64 + 16 * g));
    }
#pragma unroll 1
    for (uint32_t w = 1; w < nwmax; ++w) {
#pragma unroll
        for (int k = 0; k < 4; ++k)
            *(u32x4 *) (wl + (16 * k + (lane >> 2)) * kSlotB + 16 * g) = pre[k];
        if (w + 1 < nwmax) {
#pragma unroll
            for (int k = 0; k < 4; ++k)
                pre[k] = load_gran((const uint8_t *) (uintptr_t) (cin[k] + 64 * (w + 1)),
                                   gran_cnt(cS[k], 64 * (w + 1) + 16 * g));
        }
        lds_fence();
        if (w < nw) {
            const uint32_t nv = S - 64 * w >= 64 ? 64 : S - 64 * w;
            uint32_t x[16];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const u32x4 v = *(const u32x4 *) (myslot + 16 * q);
                x[4 * q] = v.x;
                x[4 * q + 1] = v.y;
                x[4 * q + 2] = v.z;
                x[4 * q + 3] = v.w;
            }
            salsa20_block(ks, key, n0, n1, w, 0);
            if (DEC)
                poly_absorb64(h, r, s1, s2, s3, s4, x, (int) nv);
#pragma unroll
            for (int q = 0; q < 16; ++q)
                x[q] ^= ks[q];
            if (nv < 64)
                mask_tail(x, (int) nv);
            if (!DEC)
                poly_absorb64(h, r, s1, s2, s3, s4, x, (int) nv);
#pragma unroll
            for (int q = 0; q < 4; ++q)
                *(u32x4 *) (myslot + 16 * q) = (u32x4){x[4 * q], x[4 * q + 1], x[4 * q + 2], x[4 * q + 3]};
        }
        lds_fence();
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t cnt = gran_cnt(cS[k], 64 * w + 16 * g);
            if (cnt) {
                const u32x4 v = *(const u32x4 *) (wl + (16 * k + (lane >> 2)) * kSlotB + 16 * g);
                store_gran((uint8_t *) (uintptr_t) (cout[k] + 64 * w), cnt, v);
            }
        }
        lds_fence();
    }
    if (!valid)
        return;
    uint32_t tag[4];
    poly_finish(h, spad, tag);
    if (!DEC) {
        uint32_t hdr[16] = {0x53454d07u, 0x45474153u, n0, n1, tag[0], tag[1], tag[2], tag[3]};
        store_window(dst, 32, hdr);
    } else {
        if (status == 0 && ((tag[0] ^ wtag[0]) | (tag[1] ^ wtag[1]) | (tag[2] ^ wtag[2]) | (tag[3] ^ wtag[3])))
            status = ZMQG_ERR_CRYPTOGRAPHIC;
        status_out[i] = status;
        flags_out[i] = status == 0 ? fl : 0;
    }
}

// ---------------------------------------------------------------- v3: aligned coop granules through LDS
// Stream image: stream byte j of a frame is at address A + j on input and
// B + j on output.  A window is 64 stream bytes.  Each wave = 64 frames,
// lane = frame for the compute; granule moves are cooperative: round k,
// lane l moves granule g = (64k+l)%5 of frame (64k+l)/5 (5 aligned granules
// cover any 64-byte window).
constexpr int kSl = 80;

__device__ __forceinline__ void st_partial(uint8_t *p, uint32_t lo, uint32_t hi, u32x4 v)
{
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t a = lo > 4u * q ? lo : 4u * q, b = hi < 4u * q + 4 ? hi : 4u * q + 4;
        if (a == 4u * q && b == 4u * q + 4) {
            *(uint32_t *) (p + 4 * q) = w[q];
        } else {
            for (uint32_t t = a; t < b; ++t)
                p[t] = (uint8_t) (w[q] >> (8 * (t - 4 * q)));
        }
    }
}

template <bool DEC>
__global__ __launch_bounds__(256) void k_frame3(uint32_t n, const uint32_t *__restrict__ keys,
                                                const uint64_t *__restrict__ nonce, const uint8_t *__restrict__ flags,
                                                const uint64_t *__restrict__ in_off,
                                                const uint32_t *__restrict__ len, const uint8_t *__restrict__ in,
                                                const uint64_t *__restrict__ out_off, uint8_t *__restrict__ out,
                                                uint8_t *__restrict__ flags_out, int32_t *__restrict__ status_out)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[4 * 2 * 64 * kSl];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint8_t *const ibuf = lds + wv * 2 * 64 * kSl;
    uint8_t *const obuf = ibuf + 64 * kSl;
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    const bool valid = i < n;
    const uint32_t ii = valid ? i : n - 1;
    uint32_t key[8];
#pragma unroll
    for (int t = 0; t < 8; ++t)
        key[t] = keys[t];
    const uint8_t *src = in + in_off[ii];
    uint8_t *dst = out + out_off[ii];
    const uint32_t L = len[ii];
    // this lane's frame: stream length S, input/output stream bases, valid ranges
    uint32_t S, ilo, olo, hl = 1;
    uint64_t A, B;
    uint32_t n0 = 0, n1 = 0, msgfl = 0;
    if (!DEC) {
        const uint64_t nc = nonce[ii];
        n0 = bswap32((uint32_t) (nc >> 32));
        n1 = bswap32((uint32_t) nc);
        msgfl = flags[ii] & 3;
        S = valid ? L + hl + 32 : 0;
        A = (uint64_t) (uintptr_t) src - 32 - hl;
        B = (uint64_t) (uintptr_t) dst;
        ilo = 32 + hl;
        olo = 0;
    } else {
        S = valid ? L : 0;
        A = (uint64_t) (uintptr_t) src;
        B = (uint64_t) (uintptr_t) dst - 33;
        ilo = 0;
        olo = 33;
    }
    const uint32_t nw = (S + 63) >> 6;
    const uint32_t nwmax = wave_max(nw);
    const uint32_t s_in = (uint32_t) (A & 15), s_out = (uint32_t) (B & 15);
    // cooperative granule descriptors
    uint64_t ga[5], gb[5];
    uint32_t gS[5], gsi[5], gso[5], gilo[5], golo[5], gnw[5];
    uint8_t *gslot_i[5], *gslot_o[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        const uint32_t idx = 64 * k + lane, fr = idx / 5, g = idx - 5 * fr;
        const uint64_t a = ((uint64_t) (uint32_t) __shfl((uint32_t) (A >> 32), (int) fr) << 32) |
                           (uint32_t) __shfl((uint32_t) A, (int) fr);
        const uint64_t b = ((uint64_t) (uint32_t) __shfl((uint32_t) (B >> 32), (int) fr) << 32) |
                           (uint32_t) __shfl((uint32_t) B, (int) fr);
        gsi[k] = (uint32_t) (a & 15);
        gso[k] = (uint32_t) (b & 15);
        ga[k] = (a & ~15ull) + 16 * g;
        gb[k] = (b & ~15ull) + 16 * g;
        gS[k] = (uint32_t) __shfl(S, (int) fr);
        gilo[k] = (uint32_t) __shfl(ilo, (int) fr);
        golo[k] = (uint32_t) __shfl(olo, (int) fr);
        gnw[k] = (uint32_t) __shfl(nw, (int) fr);
        gslot_i[k] = ibuf + idx * 16;
        gslot_o[k] = obuf + idx * 16;
    }
    uint8_t *const myin = ibuf + lane * kSl + s_in;
    uint8_t *const myout = obuf + lane * kSl + s_out;

    auto gload = [&](int k, uint32_t w) -> u32x4 {
        const uint32_t g = (64 * k + lane) % 5;
        const int gs = (int) (64 * w + 16 * g) - (int) gsi[k];
        const int lo = (int) gilo[k] > (int) (64 * w) ? (int) gilo[k] : (int) (64 * w);
        const int hi = (int) gS[k] < (int) (64 * w + 64) ? (int) gS[k] : (int) (64 * w + 64);
        if (gs + 16 > lo && gs < hi)
            return *(const GCU4 *) (uintptr_t) (ga[k] + 64 * w);
        return (u32x4){0, 0, 0, 0};
    };
    auto gstore = [&](int k, uint32_t w) {
        const uint32_t g = (64 * k + lane) % 5;
        if (g == 4 && w + 1 != gnw[k])
            return;
        const int gs = (int) (64 * w + 16 * g) - (int) gso[k];
        int lo = gs > (int) golo[k] ? gs : (int) golo[k];
        int hi = gs + 16 < (int) gS[k] ? gs + 16 : (int) gS[k];
        if (!DEC && w == 0) { // the tag [16, 32) is stored at the end
            if (lo >= 16 && hi <= 32)
                return;
            if (lo < 16 && hi > 16)
                hi = 16;
            if (lo < 32 && hi > 32)
                lo = 32;
        }
        if (lo >= hi)
            return;
        const u32x4 v = *(const u32x4 *) gslot_o[k];
        uint8_t *p = (uint8_t *) (uintptr_t) (gb[k] + 64 * w);
        if (lo == gs && hi == gs + 16)
            *(GU4 *) (uintptr_t) p = v;
        else
            st_partial(p, (uint32_t) (lo - gs), (uint32_t) (hi - gs), v);
    };

    u32x4 pa[5], pb[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        pa[k] = gload(k, 0);
        pb[k] = nwmax > 1 ? gload(k, 1) : (u32x4){0, 0, 0, 0};
    }
    fe h = fe_zero(), r = fe_zero();
    uint32_t s1 = 0, s2 = 0, s3 = 0, s4 = 0, spad[4] = {0, 0, 0, 0}, wtag[4] = {0, 0, 0, 0}, fl = 0;
    int32_t status = 0;

    auto step = [&](uint32_t w, u32x4 *pr) {
#pragma unroll
        for (int k = 0; k < 5; ++k)
            *(u32x4 *) gslot_i[k] = pr[k];
        if (w + 2 < nwmax) {
#pragma unroll
            for (int k = 0; k < 5; ++k)
                pr[k] = gload(k, w + 2);
        }
        lds_fence();
        if (w < nw) {
            const uint32_t nv = S - 64 * w >= 64 ? 64 : S - 64 * w;
            uint32_t x[16];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const u32x4 v = *(const u32x4 *) (myin + 16 * q);
                x[4 * q] = v.x;
                x[4 * q + 1] = v.y;
                x[4 * q + 2] = v.z;
                x[4 * q + 3] = v.w;
            }
            if (nv < 64)
                mask_tail(x, (int) nv);
            uint32_t ks[16];
            if (w == 0) {
                if (DEC) {
                    if (L < 33 || x[0] != 0x53454d07u || x[1] != 0x45474153u)
                        status = ZMQG_ERR_UNEXPECTED_COMMAND;
                    n0 = x[2];
                    n1 = x[3];
                }
                salsa20_block(ks, key, n0, n1, 0, 0);
                r = poly_r_from_key(ks[0], ks[1], ks[2], ks[3]);
                s1 = r.l[1] * 5;
                s2 = r.l[2] * 5;
                s3 = r.l[3] * 5;
                s4 = r.l[4] * 5;
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    spad[t] = ks[4 + t];
                    wtag[t] = x[4 + t];
                }
                uint32_t c[16];
                if (!DEC)
                    x[8] = (x[8] & ~0xffu) | msgfl; // plaintext byte 0 = flags (hl = 1)
#pragma unroll
                for (int t = 0; t < 16; ++t)
                    c[t] = t < 8 ? 0u : (DEC ? x[t] : x[t] ^ ks[t]);
                mask_tail(c, (int) nv);
                uint32_t c8[16];
#pragma unroll
                for (int t = 0; t < 16; ++t)
                    c8[t] = t < 8 ? c[8 + t] : 0u;
                poly_absorb64(h, r, s1, s2, s3, s4, c8, (int) nv - 32);
                if (DEC) {
                    fl = (x[8] ^ ks[8]) & 3;
#pragma unroll
                    for (int t = 8; t < 16; ++t)
                        x[t] ^= ks[t];
                } else {
                    x[0] = 0x53454d07u;
                    x[1] = 0x45474153u;
                    x[2] = n0;
                    x[3] = n1;
#pragma unroll
                    for (int t = 8; t < 16; ++t)
                        x[t] = c[t];
                }
            } else {
                salsa20_block(ks, key, n0, n1, w, 0);
                if (DEC)
                    poly_absorb64(h, r, s1, s2, s3, s4, x, (int) nv);
#pragma unroll
                for (int q = 0; q < 16; ++q)
                    x[q] ^= ks[q];
                if (nv < 64)
                    mask_tail(x, (int) nv);
                if (!DEC)
                    poly_absorb64(h, r, s1, s2, s3, s4, x, (int) nv);
            }
#pragma unroll
            for (int q = 0; q < 4; ++q)
                *(u32x4 *) (myout + 16 * q) = (u32x4){x[4 * q], x[4 * q + 1], x[4 * q + 2], x[4 * q + 3]};
        }
        lds_fence();
#pragma unroll
        for (int k = 0; k < 5; ++k)
            gstore(k, w);
        lds_fence();
        // carry the window's tail granule to the front of the slot
        const u32x4 t4 = *(const u32x4 *) (obuf + lane * kSl + 64);
        lds_fence();
        *(u32x4 *) (obuf + lane * kSl) = t4;
    };
#pragma unroll 1
    for (uint32_t w = 0; w < nwmax; w += 2) {
        step(w, pa);
        if (w + 1 < nwmax)
            step(w + 1, pb);
    }
    if (!valid)
        return;
    uint32_t tag[4];
    poly_finish(h, spad, tag);
    if (!DEC) {
        uint32_t tw[16] = {tag[0], tag[1], tag[2], tag[3]};
        store_window(dst + 16, 16, tw);
    } else {
        if (status == 0 && ((tag[0] ^ wtag[0]) | (tag[1] ^ wtag[1]) | (tag[2] ^ wtag[2]) | (tag[3] ^ wtag[3])))
            status = ZMQG_ERR_CRYPTOGRAPHIC;
        status_out[i] = status;
        flags_out[i] = status == 0 ? fl : 0;
    }
}

// encode key (client prefix) at out[0..8), decode key (client prefix too: the
// decoder mirrors the encoder's session) at out[8..16)
__global__ void k_keys(const uint32_t *in, uint32_t *out)
{
    uint32_t k[8];
    for (int i = 0; i < 8; ++i)
        k[i] = in[i];
    hsalsa20(out, k, in + 8);
    hsalsa20(out + 8, k, in + 8);
}

static uint64_t sm(uint64_t &s)
{
    uint64_t z = (s += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

int main(int argc, char **argv)
{
    const uint32_t n = argc > 1 ? atoi(argv[1]) : 65536, P = argc > 2 ? atoi(argv[2]) : 1024;
    const uint32_t W = P + 33;
    uint64_t seed = 1;
    std::vector<uint8_t> pay((size_t) n * P + 64), flags(n);
    for (auto &b : pay)
        b = (uint8_t) sm(seed);
    std::vector<uint32_t> sid(n, 0), len(n, P), wl(n, W);
    std::vector<uint64_t> nonce(n), ioff(n), ooff(n), poff(n);
    for (uint32_t i = 0; i < n; ++i) {
        nonce[i] = 3 + i;
        flags[i] = (i % 16 == 0) ? 1 : 0;
        ioff[i] = (uint64_t) i * P;
        ooff[i] = (uint64_t) i * W;
    }
    uint8_t precom[32];
    for (int i = 0; i < 32; ++i)
        precom[i] = (uint8_t) sm(seed);
    const char *cp = "CurveZMQMESSAGEC", *sp = "CurveZMQMESSAGES";

    auto dev = [](const void *h, size_t b) {
        void *d;
        CHECK(hipMalloc(&d, b + 64));
        CHECK(hipMemcpy(d, h, b, hipMemcpyHostToDevice));
        return d;
    };
    uint32_t *d_sid = (uint32_t *) dev(sid.data(), 4 * n), *d_len = (uint32_t *) dev(len.data(), 4 * n),
             *d_wl = (uint32_t *) dev(wl.data(), 4 * n);
    uint64_t *d_nonce = (uint64_t *) dev(nonce.data(), 8 * n), *d_ioff = (uint64_t *) dev(ioff.data(), 8 * n),
             *d_ooff = (uint64_t *) dev(ooff.data(), 8 * n);
    uint8_t *d_flags = (uint8_t *) dev(flags.data(), n), *d_pay = (uint8_t *) dev(pay.data(), pay.size());
    uint8_t *d_wire_ref, *d_wire, *d_back, *d_fl;
    int32_t *d_st;
    const size_t wb = (size_t) n * W + 64;
    CHECK(hipMalloc(&d_wire_ref, wb));
    CHECK(hipMalloc(&d_wire, wb));
    CHECK(hipMalloc(&d_back, pay.size()));
    CHECK(hipMalloc(&d_fl, n));
    CHECK(hipMalloc(&d_st, 4 * n));
    CHECK(hipMemset(d_wire, 0, wb));
    CHECK(hipMemset(d_wire_ref, 0, wb));

    zmqg_ctx *ctx;
    if (zmqg_ctx_create(0, 1, &ctx) || zmqg_session_set(ctx, 0, precom, (const uint8_t *) cp, (const uint8_t *) sp, 0, 0))
        return printf("ctx failed\n"), 1;
    uint32_t *d_key;
    CHECK(hipMalloc(&d_key, 32 * 2));
    {
        uint32_t in[16];
        memcpy(in, precom, 32);
        memcpy(in + 8, cp, 16);
        memcpy(in + 12, sp, 16);
        uint32_t *d_in = (uint32_t *) dev(in, 64);
        hipLaunchKernelGGL(k_keys, dim3(1), dim3(1), 0, 0, d_in, d_key);
    }
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    auto timeit = [&](auto fn, int reps) {
        fn();
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(a, 0));
        for (int r = 0; r < reps; ++r)
            fn();
        CHECK(hipEventRecord(b, 0));
        CHECK(hipEventSynchronize(b));
        float ms;
        CHECK(hipEventElapsedTime(&ms, a, b));
        return ms * 1000.0 / reps;
    };
    const int reps = 20;
    double t_ref = timeit([&] {
        zmqg_encode_batch(ctx, n, d_sid, d_nonce, d_flags, d_ioff, d_len, d_pay, d_ooff, d_wire_ref, 0);
    }, reps);
    const uint32_t blocks = (n + 255) / 256;
    double t_ab[4];
    t_ab[3] = timeit([&] { hipLaunchKernelGGL(k_enc_frame<3>, dim3(blocks), dim3(256), 0, 0, n, d_key, d_nonce, d_flags, d_ioff, d_len, d_pay, d_ooff, d_wire); }, reps);
    t_ab[2] = timeit([&] { hipLaunchKernelGGL(k_enc_frame<2>, dim3(blocks), dim3(256), 0, 0, n, d_key, d_nonce, d_flags, d_ioff, d_len, d_pay, d_ooff, d_wire); }, reps);
    t_ab[1] = timeit([&] { hipLaunchKernelGGL(k_enc_frame<1>, dim3(blocks), dim3(256), 0, 0, n, d_key, d_nonce, d_flags, d_ioff, d_len, d_pay, d_ooff, d_wire); }, reps);
    printf("ablation (encode): no poly %.1f us, no salsa %.1f us, neither %.1f us\n", t_ab[1], t_ab[2], t_ab[3]);
    double t_new = timeit([&] {
        hipLaunchKernelGGL(k_enc_frame<0>, dim3(blocks), dim3(256), 0, 0, n, d_key, d_nonce, d_flags, d_ioff, d_len,
                           d_pay, d_ooff, d_wire);
    }, reps);
    std::vector<uint8_t> h_ref(wb), h_new(wb);
    CHECK(hipMemcpy(h_ref.data(), d_wire_ref, wb, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(h_new.data(), d_wire, wb, hipMemcpyDeviceToHost));
    size_t bad = 0;
    for (size_t k = 0; k < (size_t) n * W; ++k)
        bad += h_ref[k] != h_new[k];
    printf("encode n=%u P=%u: library %.1f us, frame-kernel %.1f us (%.1f GB/s payload), mismatched bytes %zu\n", n,
           P, t_ref, t_new, (double) n * P / t_new / 1e3, bad);
    double t_dec = timeit([&] {
        hipLaunchKernelGGL(k_dec_frame, dim3(blocks), dim3(256), 0, 0, n, d_key + 8, d_ooff, d_wl, d_wire, d_ioff,
                           d_back, d_fl, d_st);
    }, reps);
    // v2
    CHECK(hipMemset(d_wire, 0, wb));
    double t_new2 = timeit([&] {
        hipLaunchKernelGGL(k_frame2<false>, dim3(blocks), dim3(256), 0, 0, n, d_key, d_nonce, d_flags, d_ioff, d_len,
                           d_pay, d_ooff, d_wire, nullptr, nullptr);
    }, reps);
    CHECK(hipMemcpy(h_new.data(), d_wire, wb, hipMemcpyDeviceToHost));
    size_t bad3 = 0;
    for (size_t k = 0; k < (size_t) n * W; ++k)
        bad3 += h_ref[k] != h_new[k];
    printf("v2 encode %.1f us (%.1f GB/s payload), mismatched bytes %zu\n", t_new2, (double) n * P / t_new2 / 1e3, bad3);
    CHECK(hipMemset(d_back, 0, pay.size()));
    double t_dec2 = timeit([&] {
        hipLaunchKernelGGL(k_frame2<true>, dim3(blocks), dim3(256), 0, 0, n, d_key + 8, nullptr, nullptr, d_ooff, d_wl,
                           d_wire, d_ioff, d_back, d_fl, d_st);
    }, reps);
    {
        std::vector<uint8_t> hb(pay.size());
        CHECK(hipMemcpy(hb.data(), d_back, pay.size(), hipMemcpyDeviceToHost));
        size_t b4 = 0;
        for (size_t k = 0; k < (size_t) n * P; ++k)
            b4 += hb[k] != pay[k];
        printf("v2 decode %.1f us (%.1f GB/s payload), payload mismatches %zu\n", t_dec2, (double) n * P / t_dec2 / 1e3, b4);
        bad3 += b4;
    }
    // v3
    CHECK(hipMemset(d_wire, 0, wb));
    double t_new3 = timeit([&] {
        hipLaunchKernelGGL(k_frame3<false>, dim3(blocks), dim3(256), 0, 0, n, d_key, d_nonce, d_flags, d_ioff, d_len,
                           d_pay, d_ooff, d_wire, nullptr, nullptr);
    }, reps);
    CHECK(hipMemcpy(h_new.data(), d_wire, wb, hipMemcpyDeviceToHost));
    {
        size_t b5 = 0, first = (size_t) -1;
        for (size_t k = 0; k < (size_t) n * W; ++k)
            if (h_ref[k] != h_new[k]) { b5++; if (first == (size_t) -1) first = k; }
        printf("v3 encode %.1f us (%.1f GB/s payload), mismatched bytes %zu (first %zd)\n", t_new3, (double) n * P / t_new3 / 1e3, b5, (ssize_t) first);
        bad3 += b5;
    }
    CHECK(hipMemset(d_back, 0, pay.size()));
    CHECK(hipMemset(d_st, 0xff, 4 * n));
    double t_dec3 = timeit([&] {
        hipLaunchKernelGGL(k_frame3<true>, dim3(blocks), dim3(256), 0, 0, n, d_key + 8, nullptr, nullptr, d_ooff, d_wl,
                           d_wire_ref, d_ioff, d_back, d_fl, d_st);
    }, reps);
    {
        std::vector<uint8_t> hb(pay.size());
        std::vector<int32_t> st3(n);
        std::vector<uint8_t> fl3(n);
        CHECK(hipMemcpy(hb.data(), d_back, pay.size(), hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(st3.data(), d_st, 4 * n, hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(fl3.data(), d_fl, n, hipMemcpyDeviceToHost));
        size_t b4 = 0, bs = 0;
        for (size_t k = 0; k < (size_t) n * P; ++k)
            b4 += hb[k] != pay[k];
        for (uint32_t k = 0; k < n; ++k)
            bs += st3[k] != 0 || fl3[k] != flags[k];
        printf("v3 decode %.1f us (%.1f GB/s payload), payload mismatches %zu, status/flags %zu\n", t_dec3, (double) n * P / t_dec3 / 1e3, b4, bs);
        bad3 += b4 + bs;
    }
    std::vector<uint8_t> h_back(pay.size());
    std::vector<int32_t> st(n);
    std::vector<uint8_t> fl(n);
    CHECK(hipMemcpy(h_back.data(), d_back, pay.size(), hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(st.data(), d_st, 4 * n, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(fl.data(), d_fl, n, hipMemcpyDeviceToHost));
    size_t bad2 = 0, badst = 0;
    for (size_t k = 0; k < (size_t) n * P; ++k)
        bad2 += h_back[k] != pay[k];
    for (uint32_t i = 0; i < n; ++i)
        badst += st[i] != 0 || fl[i] != flags[i];
    printf("decode frame-kernel %.1f us (%.1f GB/s payload), payload mismatches %zu, status/flag mismatches %zu\n",
           t_dec, (double) n * P / t_dec / 1e3, bad2, badst);
    return (bad || bad2 || badst || bad3) ? 2 : 0;
}

