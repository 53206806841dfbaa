// curve_device.hpp -- device-side building blocks of the CURVE MESSAGE path
// for gfx950: Salsa20/HSalsa20 keystream, radix-2^26 Poly1305 field
// arithmetic, and byte-exact loads/stores of arbitrarily aligned 64-byte
// windows.
//
// Algorithms: XSalsa20 and Poly1305 as composed by NaCl/libsodium 1.0.18
// crypto_box_easy_afternm (the call at reference
// src/curve_mechanism_base.cpp:172-174): keystream block 0 bytes 0..31 are
// the Poly1305 key, plaintext byte i is XORed with keystream byte 32+i.
// Everything here is 32-bit integer VALU work: v_add/v_xor/v_alignbit for
// Salsa20, v_mad_u64_u32 for the Poly1305 limb products.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace zmqg {

// ---------------------------------------------------------------- Salsa20
__device__ __forceinline__ uint32_t rotl32(uint32_t x, uint32_t n)
{
    return __builtin_rotateleft32(x, n); // one v_alignbit_b32
}

#define ZMQG_QR(a, b, c, d)        \
    b ^= rotl32(a + d, 7);         \
    c ^= rotl32(b + a, 9);         \
    d ^= rotl32(c + b, 13);        \
    a ^= rotl32(d + c, 18);

// 20 rounds (10 column + row double rounds) over 16 registers.
#define ZMQG_SALSA20_ROUNDS(x)                                   \
    _Pragma("unroll") for (int rr_ = 0; rr_ < 10; ++rr_)         \
    {                                                            \
        ZMQG_QR(x[0], x[4], x[8], x[12]);                        \
        ZMQG_QR(x[5], x[9], x[13], x[1]);                        \
        ZMQG_QR(x[10], x[14], x[2], x[6]);                       \
        ZMQG_QR(x[15], x[3], x[7], x[11]);                       \
        ZMQG_QR(x[0], x[1], x[2], x[3]);                         \
        ZMQG_QR(x[5], x[6], x[7], x[4]);                         \
        ZMQG_QR(x[10], x[11], x[8], x[9]);                       \
        ZMQG_QR(x[15], x[12], x[13], x[14]);                     \
    }

constexpr uint32_t SIGMA0 = 0x61707865, SIGMA1 = 0x3320646e, SIGMA2 = 0x79622d32, SIGMA3 = 0x6b206574;

// Keystream block `ctr` of Salsa20/20 under subkey k[8] and 8-byte nonce
// (n0, n1 = the nonce bytes as little-endian words).
__device__ __forceinline__ void salsa20_block(uint32_t out[16], const uint32_t k[8], uint32_t n0, uint32_t n1,
                                              uint32_t ctr_lo, uint32_t ctr_hi)
{
    uint32_t x[16] = {SIGMA0, k[0], k[1], k[2], k[3], SIGMA1, n0, n1,
                      ctr_lo, ctr_hi, SIGMA2, k[4], k[5], k[6], k[7], SIGMA3};
    ZMQG_SALSA20_ROUNDS(x);
    out[0] = x[0] + SIGMA0;
    out[1] = x[1] + k[0];
    out[2] = x[2] + k[1];
    out[3] = x[3] + k[2];
    out[4] = x[4] + k[3];
    out[5] = x[5] + SIGMA1;
    out[6] = x[6] + n0;
    out[7] = x[7] + n1;
    out[8] = x[8] + ctr_lo;
    out[9] = x[9] + ctr_hi;
    out[10] = x[10] + SIGMA2;
    out[11] = x[11] + k[4];
    out[12] = x[12] + k[5];
    out[13] = x[13] + k[6];
    out[14] = x[14] + k[7];
    out[15] = x[15] + SIGMA3;
}

// HSalsa20(k, in[4 words]) -> 8-word subkey (no feed-forward).
__device__ __forceinline__ void hsalsa20(uint32_t out[8], const uint32_t k[8], const uint32_t in[4])
{
    uint32_t x[16] = {SIGMA0, k[0], k[1], k[2], k[3], SIGMA1, in[0], in[1],
                      in[2], in[3], SIGMA2, k[4], k[5], k[6], k[7], SIGMA3};
    ZMQG_SALSA20_ROUNDS(x);
    out[0] = x[0];
    out[1] = x[5];
    out[2] = x[10];
    out[3] = x[15];
    out[4] = x[6];
    out[5] = x[7];
    out[6] = x[8];
    out[7] = x[9];
}

// ---------------------------------------------------------------- Poly1305
// Field elements mod 2^130-5 in five 26-bit limbs.  "Partially reduced":
// every limb < 2^26 except limb 1, which may exceed it by a few bits.
constexpr uint32_t M26 = 0x3ffffff;

struct fe {
    uint32_t l[5];
};

__device__ __forceinline__ fe fe_zero()
{
    fe z;
    z.l[0] = z.l[1] = z.l[2] = z.l[3] = z.l[4] = 0;
    return z;
}

__device__ __forceinline__ fe fe_one()
{
    fe o = fe_zero();
    o.l[0] = 1;
    return o;
}

// r from the first 16 keystream bytes, clamped
// (r &= 0x0ffffffc0ffffffc0ffffffc0fffffff), split into 26-bit limbs.
__device__ __forceinline__ fe poly_r_from_key(uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3)
{
    fe r;
    r.l[0] = k0 & 0x3ffffff;
    r.l[1] = __builtin_amdgcn_alignbit(k1, k0, 26) & 0x3ffff03;
    r.l[2] = __builtin_amdgcn_alignbit(k2, k1, 20) & 0x3ffc0ff;
    r.l[3] = __builtin_amdgcn_alignbit(k3, k2, 14) & 0x3f03fff;
    r.l[4] = (k3 >> 8) & 0x00fffff;
    return r;
}

// h += 16-byte block (m0..m3 little-endian words) + hibit*2^128.
__device__ __forceinline__ void fe_add_block(fe &h, uint32_t m0, uint32_t m1, uint32_t m2, uint32_t m3,
                                             uint32_t hibit)
{
    h.l[0] += m0 & M26;
    h.l[1] += __builtin_amdgcn_alignbit(m1, m0, 26) & M26;
    h.l[2] += __builtin_amdgcn_alignbit(m2, m1, 20) & M26;
    h.l[3] += __builtin_amdgcn_alignbit(m3, m2, 14) & M26;
    h.l[4] += (m3 >> 8) | hibit;
}

__device__ __forceinline__ void fe_add(fe &h, const fe &x)
{
#pragma unroll
    for (int i = 0; i < 5; ++i)
        h.l[i] += x.l[i];
}

__device__ __forceinline__ uint64_t mad64(uint32_t a, uint32_t b, uint64_t c)
{
    return (uint64_t) a * b + c; // v_mad_u64_u32
}

// h = h * r mod 2^130-5, partially reduced.  s = 5*r[1..4] precomputed.
// Inputs: h limbs < 2^27, r limbs < 2^26 + 2^8.
__device__ __forceinline__ void fe_mul_s(fe &h, const fe &r, const uint32_t s1, const uint32_t s2, const uint32_t s3,
                                         const uint32_t s4)
{
    const uint32_t h0 = h.l[0], h1 = h.l[1], h2 = h.l[2], h3 = h.l[3], h4 = h.l[4];
    uint64_t d0 = mad64(h4, s1, mad64(h3, s2, mad64(h2, s3, mad64(h1, s4, (uint64_t) h0 * r.l[0]))));
    uint64_t d1 = mad64(h4, s2, mad64(h3, s3, mad64(h2, s4, mad64(h1, r.l[0], (uint64_t) h0 * r.l[1]))));
    uint64_t d2 = mad64(h4, s3, mad64(h3, s4, mad64(h2, r.l[0], mad64(h1, r.l[1], (uint64_t) h0 * r.l[2]))));
    uint64_t d3 = mad64(h4, s4, mad64(h3, r.l[0], mad64(h2, r.l[1], mad64(h1, r.l[2], (uint64_t) h0 * r.l[3]))));
    uint64_t d4 = mad64(h4, r.l[0], mad64(h3, r.l[1], mad64(h2, r.l[2], mad64(h1, r.l[3], (uint64_t) h0 * r.l[4]))));
    uint32_t c;
    c = (uint32_t) (d0 >> 26);
    h.l[0] = (uint32_t) d0 & M26;
    d1 += c;
    c = (uint32_t) (d1 >> 26);
    h.l[1] = (uint32_t) d1 & M26;
    d2 += c;
    c = (uint32_t) (d2 >> 26);
    h.l[2] = (uint32_t) d2 & M26;
    d3 += c;
    c = (uint32_t) (d3 >> 26);
    h.l[3] = (uint32_t) d3 & M26;
    d4 += c;
    c = (uint32_t) (d4 >> 26);
    h.l[4] = (uint32_t) d4 & M26;
    h.l[0] += c * 5;
    c = h.l[0] >> 26;
    h.l[0] &= M26;
    h.l[1] += c;
}

__device__ __forceinline__ void fe_mul(fe &h, const fe &r)
{
    fe_mul_s(h, r, r.l[1] * 5, r.l[2] * 5, r.l[3] * 5, r.l[4] * 5);
}

// Fold 64-bit limb sums (from lane reductions / atomics) back to a
// partially reduced element.
__device__ __forceinline__ fe fe_from_wide(const uint64_t w[5])
{
    uint64_t a0 = w[0], a1 = w[1], a2 = w[2], a3 = w[3], a4 = w[4];
    a1 += a0 >> 26;
    a0 &= M26;
    a2 += a1 >> 26;
    a1 &= M26;
    a3 += a2 >> 26;
    a2 &= M26;
    a4 += a3 >> 26;
    a3 &= M26;
    a0 += (a4 >> 26) * 5;
    a4 &= M26;
    a1 += a0 >> 26;
    a0 &= M26;
    fe h;
    h.l[0] = (uint32_t) a0;
    h.l[1] = (uint32_t) a1;
    h.l[2] = (uint32_t) a2;
    h.l[3] = (uint32_t) a3;
    h.l[4] = (uint32_t) a4;
    return h;
}

// Freeze h mod 2^130-5 and add the pad s (mod 2^128): the tag, as 4 words.
__device__ __forceinline__ void poly_finish(fe h, const uint32_t s[4], uint32_t tag[4])
{
    uint32_t h0 = h.l[0], h1 = h.l[1], h2 = h.l[2], h3 = h.l[3], h4 = h.l[4], c;
    c = h1 >> 26;
    h1 &= M26;
    h2 += c;
    c = h2 >> 26;
    h2 &= M26;
    h3 += c;
    c = h3 >> 26;
    h3 &= M26;
    h4 += c;
    c = h4 >> 26;
    h4 &= M26;
    h0 += c * 5;
    c = h0 >> 26;
    h0 &= M26;
    h1 += c;
    uint32_t g0 = h0 + 5;
    c = g0 >> 26;
    g0 &= M26;
    uint32_t g1 = h1 + c;
    c = g1 >> 26;
    g1 &= M26;
    uint32_t g2 = h2 + c;
    c = g2 >> 26;
    g2 &= M26;
    uint32_t g3 = h3 + c;
    c = g3 >> 26;
    g3 &= M26;
    uint32_t g4 = h4 + c - (1u << 26);
    const uint32_t mask = (g4 >> 31) - 1u;
    h0 = (h0 & ~mask) | (g0 & mask);
    h1 = (h1 & ~mask) | (g1 & mask);
    h2 = (h2 & ~mask) | (g2 & mask);
    h3 = (h3 & ~mask) | (g3 & mask);
    h4 = (h4 & ~mask) | (g4 & mask);
    uint64_t f0 = (uint64_t) (h0 | (h1 << 26)) + s[0];
    uint64_t f1 = (uint64_t) ((h1 >> 6) | (h2 << 20)) + s[1] + (f0 >> 32);
    uint64_t f2 = (uint64_t) ((h2 >> 12) | (h3 << 14)) + s[2] + (f1 >> 32);
    uint64_t f3 = (uint64_t) ((h3 >> 18) | (h4 << 8)) + s[3] + (f2 >> 32);
    tag[0] = (uint32_t) f0;
    tag[1] = (uint32_t) f1;
    tag[2] = (uint32_t) f2;
    tag[3] = (uint32_t) f3;
}

// Poly1305-absorb 16 words (64 bytes) of which `nv` bytes are valid,
// as up to four 16-byte blocks; a partial final block is padded 0x01 0...
// Bytes beyond nv in w[] must already be zero.
__device__ __forceinline__ void poly_absorb64(fe &h, const fe &r, const uint32_t s1, const uint32_t s2,
                                              const uint32_t s3, const uint32_t s4, uint32_t w[16], int nv)
{
    if (nv >= 64) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            fe_add_block(h, w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3], 1u << 24);
            fe_mul_s(h, r, s1, s2, s3, s4);
        }
        return;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int bl = nv - 16 * q;
        if (bl <= 0)
            break;
        uint32_t m[4] = {w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]};
        uint32_t hibit = 1u << 24;
        if (bl < 16) {
            hibit = 0;
            const int wi = bl >> 2, bi = bl & 3;
#pragma unroll
            for (int t = 0; t < 4; ++t)
                if (t == wi)
                    m[t] |= 1u << (8 * bi);
        }
        fe_add_block(h, m[0], m[1], m[2], m[3], hibit);
        fe_mul_s(h, r, s1, s2, s3, s4);
    }
}

// ---------------------------------------------------------------- Poly1305, radix 2^32
// The sequential form h = (h + m) * r with h in four 32-bit words plus a
// small fifth (h4 <= 6 between blocks) and r clamped: the clamp (r_k < 2^28,
// r_1..r_3 multiples of 4) keeps every sum of four word products below 2^64
// and lets 2^130 = 5/4 fold into s_k = r_k + r_k/4.  19 v_mad_u64_u32 and one
// v_mul_lo_u32 per 16-byte block, against 25 v_mad_u64_u32 plus the limb
// split of the radix-2^26 form (measured 0.72x the Poly1305 time of that
// form in the frame loop, tools/frames_proto.hip).
struct Poly32 {
    uint32_t h0, h1, h2, h3, h4;
};

struct PolyKey32 {
    uint32_t r0, r1, r2, r3, s1, s2, s3;
};

__device__ __forceinline__ PolyKey32 poly32_key(uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3)
{
    PolyKey32 k;
    k.r0 = k0 & 0x0fffffffu;
    k.r1 = k1 & 0x0ffffffcu;
    k.r2 = k2 & 0x0ffffffcu;
    k.r3 = k3 & 0x0ffffffcu;
    k.s1 = k.r1 + (k.r1 >> 2);
    k.s2 = k.r2 + (k.r2 >> 2);
    k.s3 = k.r3 + (k.r3 >> 2);
    return k;
}

// h = (h + m + hib * 2^128) * r, partially reduced (h4 <= 4 on return).
// Carries are 32-bit add-with-carry chains (v_add_co / v_addc_co); written
// as 64-bit sums the compiler materialises zero high halves and 64-bit adds
// (245 instructions per window against 165 this way).
__device__ __forceinline__ void poly32_block(Poly32 &h, uint32_t m0, uint32_t m1, uint32_t m2, uint32_t m3,
                                             uint32_t hib, const PolyKey32 &k)
{
    unsigned c;
    const uint32_t a0 = __builtin_addc(h.h0, m0, 0u, &c);
    const uint32_t a1 = __builtin_addc(h.h1, m1, c, &c);
    const uint32_t a2 = __builtin_addc(h.h2, m2, c, &c);
    const uint32_t a3 = __builtin_addc(h.h3, m3, c, &c);
    const uint32_t a4 = h.h4 + hib + c;
    const uint64_t d0 = mad64(a3, k.s1, mad64(a2, k.s2, mad64(a1, k.s3, (uint64_t) a0 * k.r0)));
    const uint64_t d1 = mad64(a4, k.s1, mad64(a3, k.s2, mad64(a2, k.s3, mad64(a1, k.r0, (uint64_t) a0 * k.r1))));
    const uint64_t d2 = mad64(a4, k.s2, mad64(a3, k.s3, mad64(a2, k.r0, mad64(a1, k.r1, (uint64_t) a0 * k.r2))));
    const uint64_t d3 = mad64(a4, k.s3, mad64(a3, k.r0, mad64(a2, k.r1, mad64(a1, k.r2, (uint64_t) a0 * k.r3))));
    // h = d0 + d1 2^32 + d2 2^64 + d3 2^96 + (a4 r0) 2^128
    const uint32_t h0 = (uint32_t) d0;
    const uint32_t h1 = __builtin_addc((uint32_t) d1, (uint32_t) (d0 >> 32), 0u, &c);
    const uint32_t c1 = (uint32_t) (d1 >> 32) + c;
    const uint32_t h2 = __builtin_addc((uint32_t) d2, c1, 0u, &c);
    const uint32_t c2 = (uint32_t) (d2 >> 32) + c;
    const uint32_t h3 = __builtin_addc((uint32_t) d3, c2, 0u, &c);
    const uint32_t h4 = a4 * k.r0 + (uint32_t) (d3 >> 32) + c;
    const uint32_t f = (h4 >> 2) + (h4 & ~3u); // 5 * (h >> 130)
    h.h0 = __builtin_addc(h0, f, 0u, &c);
    h.h1 = __builtin_addc(h1, 0u, c, &c);
    h.h2 = __builtin_addc(h2, 0u, c, &c);
    h.h3 = __builtin_addc(h3, 0u, c, &c);
    h.h4 = (h4 & 3u) + c;
}

// Absorb the ciphertext blocks of one 64-byte keystream window: the window's
// 16 words c (zero beyond the ciphertext), its first block slot j0 (2 for
// window 0, whose first 32 stream bytes are the Poly1305 key, else 0) and the
// ciphertext bytes it holds (len, 1..64).  A final partial block gets the
// 0x01 pad byte and no 2^128 bit.
__device__ __forceinline__ void poly32_window(Poly32 &h, const PolyKey32 &k, const uint32_t c[16], uint32_t j0,
                                              uint32_t len)
{
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int off = 16 * (j - (int) j0);
        if (j >= (int) j0 && off < (int) len) {
            const int nb = (int) len - off;
            uint32_t m0 = c[4 * j], m1 = c[4 * j + 1], m2 = c[4 * j + 2], m3 = c[4 * j + 3], hib = 1u;
            if (nb < 16) {
                hib = 0u;
                const uint32_t pad = 1u << (8 * (nb & 3));
                const int wi = nb >> 2;
                m0 |= wi == 0 ? pad : 0u;
                m1 |= wi == 1 ? pad : 0u;
                m2 |= wi == 2 ? pad : 0u;
                m3 |= wi == 3 ? pad : 0u;
            }
            poly32_block(h, m0, m1, m2, m3, hib, k);
        }
    }
}

// The four full blocks of an interior window.
__device__ __forceinline__ void poly32_window_full(Poly32 &h, const PolyKey32 &k, const uint32_t c[16])
{
#pragma unroll
    for (int j = 0; j < 4; ++j)
        poly32_block(h, c[4 * j], c[4 * j + 1], c[4 * j + 2], c[4 * j + 3], 1u, k);
}

// Conversions between the two forms (the chunked path's Horner runs in radix
// 2^32, its cross-lane sums in 26-bit limbs).  r: a clamped key's limbs.
__device__ __forceinline__ PolyKey32 poly32_key_from_fe(const uint32_t r[5])
{
    return poly32_key(r[0] | (r[1] << 26), (r[1] >> 6) | (r[2] << 20), (r[2] >> 12) | (r[3] << 14),
                      (r[3] >> 18) | (r[4] << 8));
}

// A partially reduced element (limbs a little above 2^26 allowed) as h0..h4
// (h4 small: the value is below 2^131).
__device__ __forceinline__ Poly32 fe_to_poly32(fe x)
{
    uint32_t c;
    c = x.l[0] >> 26;
    x.l[0] &= M26;
    x.l[1] += c;
    c = x.l[1] >> 26;
    x.l[1] &= M26;
    x.l[2] += c;
    c = x.l[2] >> 26;
    x.l[2] &= M26;
    x.l[3] += c;
    c = x.l[3] >> 26;
    x.l[3] &= M26;
    x.l[4] += c; // < 2^26 + 2: h4 <= 4
    Poly32 h;
    h.h0 = x.l[0] | (x.l[1] << 26);
    h.h1 = (x.l[1] >> 6) | (x.l[2] << 20);
    h.h2 = (x.l[2] >> 12) | (x.l[3] << 14);
    h.h3 = (x.l[3] >> 18) | (x.l[4] << 8);
    h.h4 = x.l[4] >> 24;
    return h;
}

// h (h4 <= 6) as 26-bit limbs, the top one below 2^27 (fe_mul's input bound).
__device__ __forceinline__ fe poly32_to_fe(const Poly32 &h)
{
    fe x;
    x.l[0] = h.h0 & M26;
    x.l[1] = ((h.h0 >> 26) | (h.h1 << 6)) & M26;
    x.l[2] = ((h.h1 >> 20) | (h.h2 << 12)) & M26;
    x.l[3] = ((h.h2 >> 14) | (h.h3 << 18)) & M26;
    x.l[4] = (h.h3 >> 8) | (h.h4 << 24);
    return x;
}

// Tag = (h mod 2^130-5) + s mod 2^128 (h4 <= 4, so one conditional
// subtraction of p reduces it).
__device__ __forceinline__ void poly32_finish(const Poly32 &h, const uint32_t s[4], uint32_t tag[4])
{
    unsigned c;
    const uint32_t g0 = __builtin_addc(h.h0, 5u, 0u, &c);
    const uint32_t g1 = __builtin_addc(h.h1, 0u, c, &c);
    const uint32_t g2 = __builtin_addc(h.h2, 0u, c, &c);
    const uint32_t g3 = __builtin_addc(h.h3, 0u, c, &c);
    const uint32_t g4 = h.h4 + c;
    const uint32_t m = 0u - (g4 >> 2); // all ones when h + 5 >= 2^130: take h - p
    const uint32_t f0 = (g0 & m) | (h.h0 & ~m), f1 = (g1 & m) | (h.h1 & ~m), f2 = (g2 & m) | (h.h2 & ~m),
                   f3 = (g3 & m) | (h.h3 & ~m);
    tag[0] = __builtin_addc(f0, s[0], 0u, &c);
    tag[1] = __builtin_addc(f1, s[1], c, &c);
    tag[2] = __builtin_addc(f2, s[2], c, &c);
    tag[3] = __builtin_addc(f3, s[3], c, &c);
}

// ---------------------------------------------------------------- bytes
// Little-endian word of 4 bytes from a byte pointer (any alignment).
__device__ __forceinline__ uint32_t bswap32(uint32_t x)
{
    return __builtin_bswap32(x);
}

// Zero bytes >= nv of a 16-word window.
__device__ __forceinline__ void mask_tail(uint32_t w[16], int nv)
{
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int b = nv - 4 * i;
        const uint32_t m = b >= 4 ? 0xffffffffu : (b <= 0 ? 0u : ((1u << (8 * b)) - 1u));
        w[i] &= m;
    }
}

// Load bytes p[0 .. nv) (0 <= nv <= 64, any alignment) as 16 little-endian
// words, zero beyond nv.  Only 4-byte words that hold a valid byte are read,
// so the access never leaves the 4-byte granules of the valid range.
__device__ __forceinline__ void load_window(const uint8_t *p, int nv, uint32_t w[16])
{
    const uint32_t sh = (uint32_t) ((uintptr_t) p & 3);
    const uint32_t *q = (const uint32_t *) (p - sh); // keep the global address space (no inttoptr)
    uint32_t d[17];
    if (nv >= 64) {
#pragma unroll
        for (int i = 0; i < 16; ++i)
            d[i] = q[i];
        d[16] = sh ? q[16] : 0u;
    } else {
        const int nd = (int) ((sh + (uint32_t) nv + 3) >> 2);
#pragma unroll
        for (int i = 0; i < 17; ++i)
            d[i] = i < nd ? q[i] : 0u;
    }
#pragma unroll
    for (int i = 0; i < 16; ++i)
        w[i] = __builtin_amdgcn_alignbyte(d[i + 1], d[i], sh);
    if (nv < 64)
        mask_tail(w, nv);
}

// Store bytes w[0 .. nv) (as a little-endian byte stream) at p (any
// alignment).  Only bytes [p, p+nv) are written: up to 3 leading and 3
// trailing bytes by byte stores, the rest as aligned dword stores.
__device__ __forceinline__ void store_window(uint8_t *p, int nv, const uint32_t w[16])
{
    const uintptr_t a = (uintptr_t) p;
    const uint32_t sh = (uint32_t) (a & 3);
    if (sh == 0 && nv >= 64) {
        typedef unsigned int u32x4_ __attribute__((ext_vector_type(4)));
        typedef __attribute__((address_space(1))) u32x4_ __attribute__((aligned(4))) GU4a4_;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            *(GU4a4_ *) (a + 16u * i) = (u32x4_){w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]};
        return;
    }
    const uint32_t s = (4u - sh) & 3u; // bytes before the first aligned dword
    (void) a;
    uint32_t e[16];
#pragma unroll
    for (int k = 0; k < 15; ++k)
        e[k] = __builtin_amdgcn_alignbyte(w[k + 1], w[k], s);
    e[15] = __builtin_amdgcn_alignbyte(0u, w[15], s);
    const int lead = (int) s < nv ? (int) s : nv;
#pragma unroll
    for (int b = 0; b < 3; ++b)
        if (b < lead)
            p[b] = (uint8_t) (w[0] >> (8 * b));
    if (nv <= (int) s)
        return;
    const int rem = nv - (int) s;
    const int nd = rem >> 2;
    uint32_t *q = (uint32_t *) (p + s);
#pragma unroll
    for (int k = 0; k < 16; ++k)
        if (k < nd)
            q[k] = e[k];
    const int tb = rem & 3;
    if (tb) {
        uint32_t t = 0;
#pragma unroll
        for (int k = 0; k < 16; ++k)
            if (k == nd)
                t = e[k];
        uint8_t *pt = (uint8_t *) (q + nd);
#pragma unroll
        for (int b = 0; b < 3; ++b)
            if (b < tb)
                pt[b] = (uint8_t) (t >> (8 * b));
    }
}

// Store bytes w[0 .. NV) (NV a multiple of 4, 8 <= NV <= 64) at p, any
// alignment, as one fixed sequence: the leading bytes up to the first 4-byte
// boundary (a byte and a short store, each when needed), the aligned dwords
// (dwordx4 where whole), the trailing bytes (a short and a byte store).  A
// lane's stores each touch other lines than its neighbours' (frames sit at
// arbitrary strides), so every store instruction costs the address unit all
// 64 lanes; store_window's runtime length issues one instruction per dword
// and per edge byte (about 22 for 16 bytes), this about 7 for 16 and 10 for
// 64.
template <int NV>
__device__ __forceinline__ void store_bytes_c(uint8_t *p, const uint32_t w[16])
{
    static_assert(NV % 4 == 0 && NV >= 8 && NV <= 64, "whole dwords, at most one window");
    typedef __attribute__((address_space(1))) uint8_t GU8_;
    typedef __attribute__((address_space(1))) uint16_t GU16_;
    typedef __attribute__((address_space(1))) uint32_t GU32_;
    typedef unsigned int u32x2_ __attribute__((ext_vector_type(2)));
    typedef unsigned int u32x3_ __attribute__((ext_vector_type(3)));
    typedef __attribute__((address_space(1))) u32x2_ __attribute__((aligned(4))) GU2a4_;
    typedef __attribute__((address_space(1))) u32x3_ __attribute__((aligned(4))) GU3a4_;
    typedef unsigned int u32x4_ __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(1))) u32x4_ __attribute__((aligned(4))) GU4a4_;
    const uint64_t a = (uint64_t) (uintptr_t) p;
    const uint32_t sh = (uint32_t) a & 3u, s = (4u - sh) & 3u; // s leading bytes before the first aligned dword
    constexpr int ND = NV / 4;
    uint32_t e[ND]; // e[k] = bytes [s + 4k, s + 4k + 4) of the stream w
#pragma unroll
    for (int k = 0; k < ND; ++k)
        e[k] = __builtin_amdgcn_alignbyte(k + 1 < 16 ? w[k + 1] : 0u, w[k], s);
    // leading bytes: s = 1 -> [0]; 2 -> [0,1]; 3 -> [0] and [1,2]
    if (s & 1u)
        *(GU8_ *) (uintptr_t) a = (uint8_t) w[0];
    if (s & 2u)
        *(GU16_ *) (uintptr_t) (a + (s & 1u)) = (uint16_t) (w[0] >> (8u * (s & 1u)));
    // ND - 1 dwords for every alignment, the last one only when s == 0
    const uint64_t q = a + s;
    constexpr int NU = ND - 1;
#pragma unroll
    for (int g = 0; g + 4 <= NU; g += 4)
        *(GU4a4_ *) (uintptr_t) (q + 4u * g) = (u32x4_){e[g], e[g + 1], e[g + 2], e[g + 3]};
    constexpr int G4 = NU / 4 * 4;
    if (NU - G4 == 3)
        *(GU3a4_ *) (uintptr_t) (q + 4u * G4) = (u32x3_){e[G4], e[G4 + 1], e[G4 + 2]};
    else if (NU - G4 == 2)
        *(GU2a4_ *) (uintptr_t) (q + 4u * G4) = (u32x2_){e[G4], e[G4 + 1]};
    else if (NU - G4 == 1)
        *(GU32_ *) (uintptr_t) (q + 4u * G4) = e[G4];
    if (s == 0u)
        *(GU32_ *) (uintptr_t) (q + 4u * NU) = e[NU];
    // trailing bytes (sh of them, the first bytes of e[NU]): 1 -> [0]; 2 -> [0,1]; 3 -> [0,1] and [2]
    const uint64_t t = q + 4u * NU;
    if (sh & 2u)
        *(GU16_ *) (uintptr_t) t = (uint16_t) e[NU];
    if (sh & 1u)
        *(GU8_ *) (uintptr_t) (t + (sh & 2u)) = (uint8_t) (e[NU] >> (8u * (sh & 2u)));
}

// Load bytes p[0 .. NV) (NV a multiple of 16, at most 48; any alignment) as
// NV/4 little-endian words: the aligned words covering them, NV/16 dwordx4
// and one dword when p is not 4-byte aligned (a word holding a byte of the
// range never crosses into a page the range does not touch) -- a fixed
// sequence where load_window's runtime length issues one load per word.
template <int NV>
__device__ __forceinline__ void load_bytes_c(const uint8_t *p, uint32_t w[NV / 4])
{
    static_assert(NV % 16 == 0 && NV >= 16 && NV <= 48, "whole granules");
    typedef __attribute__((address_space(1))) const uint32_t GCU32_;
    typedef unsigned int u32x4_ __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(1))) const u32x4_ __attribute__((aligned(4))) GCU4a4_;
    const uint64_t a = (uint64_t) (uintptr_t) p;
    const uint32_t sh = (uint32_t) a & 3u;
    const uint64_t q = a - sh;
    constexpr int ND = NV / 4;
    uint32_t d[ND + 1];
#pragma unroll
    for (int g = 0; g < ND / 4; ++g) {
        const u32x4_ t = *(GCU4a4_ *) (uintptr_t) (q + 16u * g);
        d[4 * g] = t.x;
        d[4 * g + 1] = t.y;
        d[4 * g + 2] = t.z;
        d[4 * g + 3] = t.w;
    }
    d[ND] = sh ? *(GCU32_ *) (uintptr_t) (q + 4u * ND) : 0u;
#pragma unroll
    for (int k = 0; k < ND; ++k)
        w[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh);
}

// Store bytes [0, nb) of the word stream o (0 <= nb <= 68) at the 4-byte
// aligned address a, as a fixed sequence of lane-predicated stores: four
// dwordx4 (each while whole), three dwords, a short and a byte -- at most 9
// instructions, where a per-word loop issues one per word (frame tails).
__device__ __forceinline__ void store_tail(uint64_t a, uint32_t nb, const uint32_t o[17])
{
    typedef __attribute__((address_space(1))) uint8_t GU8_;
    typedef __attribute__((address_space(1))) uint16_t GU16_;
    typedef __attribute__((address_space(1))) uint32_t GU32_;
    typedef unsigned int u32x4_ __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(1))) u32x4_ __attribute__((aligned(4))) GU4a4_;
    const uint32_t nw = nb >> 2, ng = nw >> 2; // whole words, whole 4-word groups
#pragma unroll
    for (uint32_t g = 0; g < 4; ++g)
        if (g < ng)
            *(GU4a4_ *) (uintptr_t) (a + 16u * g) = (u32x4_){o[4 * g], o[4 * g + 1], o[4 * g + 2], o[4 * g + 3]};
    // words 4ng .. nw-1 (at most 3; with ng = 4 only word 16), then the partial word nw
    uint32_t r[4];
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
        uint32_t v = 0;
#pragma unroll
        for (uint32_t g = 0; g < 5; ++g)
            if (g == ng && 4 * g + k < 17)
                v = o[4 * g + k];
        r[k] = v;
    }
    const uint64_t b = a + 16u * ng;
    const uint32_t nr = nw - 4u * ng; // 0..3
#pragma unroll
    for (uint32_t k = 0; k < 3; ++k)
        if (k < nr)
            *(GU32_ *) (uintptr_t) (b + 4u * k) = r[k];
    uint32_t last = r[0];
#pragma unroll
    for (uint32_t k = 1; k < 4; ++k)
        if (k == nr)
            last = r[k];
    const uint32_t tb = nb & 3u;
    const uint64_t c = b + 4u * nr;
    if (tb & 2u)
        *(GU16_ *) (uintptr_t) c = (uint16_t) last;
    if (tb & 1u)
        *(GU8_ *) (uintptr_t) (c + (tb & 2u)) = (uint8_t) (last >> (8u * (tb & 2u)));
}

// Zero bytes [p, p + len) by one lane: byte stores up to the first 16-byte
// boundary and after the last, dwordx4 stores between.  (Only for regions a
// lane may afford to clear alone: a frame the frame kernel holds, at most a
// few KiB; larger regions go to the cooperative fill kernel.)
__device__ __forceinline__ void zero_bytes(uint8_t *p, uint32_t len)
{
    const uint32_t head = (uint32_t) ((16u - ((uintptr_t) p & 15u)) & 15u);
    const uint32_t h = head < len ? head : len;
    for (uint32_t b = 0; b < h; ++b)
        p[b] = 0;
    uint32_t k = h;
    typedef unsigned int z4 __attribute__((ext_vector_type(4)));
    for (; k + 16u <= len; k += 16u)
        *(z4 *) (p + k) = (z4){0u, 0u, 0u, 0u};
    for (; k < len; ++k)
        p[k] = 0;
}

// ---------------------------------------------------------------- streams
// Global-address-space views (keep global_load/store, not flat, for
// addresses rebuilt from integers).
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) uint8_t GU8;
typedef __attribute__((address_space(1))) const u32x4 GCU4;
typedef __attribute__((address_space(1))) u32x4 GU4;
typedef __attribute__((address_space(1))) uint32_t GU32;

// out[i] = v[i + ws] for a runtime ws in 0..3, branch-free (two cndmask
// stages), so lanes of differently aligned frames never diverge.
template <int N>
__device__ __forceinline__ void select_shift(const uint32_t *v, uint32_t ws, uint32_t *out)
{
    // bit-select (v_bfi_b32) rather than ?: so the optimizer cannot turn the
    // selects back into a dynamically indexed (scratch) array
    const uint32_t m1 = 0u - (ws & 1u), m2 = 0u - ((ws >> 1) & 1u);
    uint32_t a[N + 2];
#pragma unroll
    for (int i = 0; i < N + 2; ++i)
        a[i] = (v[i + 1] & m1) | (v[i] & ~m1);
#pragma unroll
    for (int i = 0; i < N; ++i)
        out[i] = (a[i + 2] & m2) | (a[i] & ~m2);
}

// Sequential reader of 64-byte windows of a byte stream of L bytes at an
// arbitrary address.  Loads whole aligned 16-byte granules (dwordx4), each
// once (one carried between windows), and never a granule with no valid byte.
struct StreamReader {
    const GCU4 *g;  // aligned-down base
    uint32_t off;   // base misalignment (0..15)
    uint32_t end;   // off + L
    u32x4 carry;    // granule 4t, loaded with the previous window
};

__device__ __forceinline__ void reader_init(StreamReader &r, uint64_t p, uint32_t L)
{
    r.off = (uint32_t) (p & 15);
    r.g = (const GCU4 *) (uintptr_t) (p - r.off);
    r.end = r.off + L;
    r.carry = (L > 0) ? r.g[0] : (u32x4){0, 0, 0, 0};
}

__device__ __forceinline__ u32x4 granule_or_zero(const StreamReader &r, uint32_t k)
{
    return (16 * k < r.end) ? r.g[k] : (u32x4){0, 0, 0, 0};
}

// Window t: stream bytes [64t, 64t+64) (valid up to nv), zero beyond nv.
__device__ __forceinline__ void reader_window(StreamReader &r, uint32_t t, int nv, uint32_t w[16])
{
    const u32x4 a = r.carry;
    const u32x4 b = granule_or_zero(r, 4 * t + 1), c = granule_or_zero(r, 4 * t + 2),
                d = granule_or_zero(r, 4 * t + 3), e = granule_or_zero(r, 4 * t + 4);
    r.carry = e;
    const uint32_t v[20] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y,
                            c.z, c.w, d.x, d.y, d.z, d.w, e.x, e.y, e.z, e.w};
    uint32_t u[17];
    select_shift<17>(v, r.off >> 2, u);
    const uint32_t bs = r.off & 3;
#pragma unroll
    for (int i = 0; i < 16; ++i)
        w[i] = __builtin_amdgcn_alignbyte(u[i + 1], u[i], bs);
    if (nv < 64)
        mask_tail(w, nv);
}

// Store `len` (< 16) bytes of the 4 words at an aligned address.
__device__ __forceinline__ void store_partial_granule(GU8 *p, int len, const uint32_t o[4])
{
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int rem = len - 4 * k;
        if (rem >= 4) {
            *(GU32 *) (p + 4 * k) = o[k];
        } else if (rem > 0) {
#pragma unroll
            for (int b = 0; b < 3; ++b)
                if (b < rem)
                    p[4 * k + b] = (uint8_t) (o[k] >> (8 * b));
        }
    }
}

// Writer of a lane's output stream S (L bytes) to an arbitrarily aligned
// address a.  The s0 bytes before the first 16-byte aligned address are
// stored individually; the rest goes out as whole aligned granules (dwordx4)
// once complete, plus at most one partial granule at the end.  Granule G
// holds stream bytes [s0 + 16G, s0 + 16G + 16).  Windows in order.
struct GranuleWriter {
    uint64_t a;  // stream byte 0
    uint32_t s0; // 0..15
    int L;
    uint32_t p12, p13, p14, p15; // previous window's last words
};

__device__ __forceinline__ void gw_init(GranuleWriter &gw, uint64_t a, int L)
{
    gw.a = a;
    gw.s0 = (16u - (uint32_t) (a & 15)) & 15u;
    gw.L = L;
    gw.p12 = gw.p13 = gw.p14 = gw.p15 = 0;
}

__device__ __forceinline__ void gw_window(GranuleWriter &gw, int t, const uint32_t w[16])
{
    GU8 *base = (GU8 *) (uintptr_t) gw.a;
    GU8 *gq = base + gw.s0; // first aligned granule
    if (t == 0) { // the s0 leading bytes (inside words 0..3)
        const int lead = (int) gw.s0 < gw.L ? (int) gw.s0 : gw.L;
#pragma unroll
        for (int b = 0; b < 15; ++b)
            if (b < lead)
                base[b] = (uint8_t) (w[b >> 2] >> (8 * (b & 3)));
    }
    // v = stream words 16t-4 .. 16t+19 (previous tail, this window, zeros)
    const uint32_t v[24] = {gw.p12, gw.p13, gw.p14, gw.p15, w[0], w[1], w[2],  w[3],  w[4],  w[5],  w[6], w[7],
                            w[8],   w[9],   w[10],  w[11],  w[12], w[13], w[14], w[15], 0u,    0u,    0u,   0u};
    uint32_t u[21];
    select_shift<21>(v, gw.s0 >> 2, u);
    const uint32_t bs = gw.s0 & 3;
    const bool last = gw.L <= 64 * t + 64;
    // candidate granules G = 4t-1+q; a granule is emitted in the window
    // that completes it, or in the last window if the stream ends inside it
#pragma unroll
    for (int q = 0; q < 5; ++q) {
        const int G = 4 * t - 1 + q;
        const int start = (int) gw.s0 + 16 * G;
        const int endg = start + 16;
        const bool due = (endg > 64 * t && endg <= 64 * t + 64) || (last && endg > 64 * t + 64);
        const int len = gw.L - start;
        if (!due || G < 0 || len <= 0)
            continue;
        const uint32_t o[4] = {__builtin_amdgcn_alignbyte(u[4 * q + 1], u[4 * q], bs),
                               __builtin_amdgcn_alignbyte(u[4 * q + 2], u[4 * q + 1], bs),
                               __builtin_amdgcn_alignbyte(u[4 * q + 3], u[4 * q + 2], bs),
                               __builtin_amdgcn_alignbyte(u[4 * q + 4], u[4 * q + 3], bs)};
        if (len >= 16)
            *(GU4 *) (gq + 16 * G) = (u32x4){o[0], o[1], o[2], o[3]};
        else
            store_partial_granule(gq + 16 * G, len, o);
    }
    gw.p12 = w[12];
    gw.p13 = w[13];
    gw.p14 = w[14];
    gw.p15 = w[15];
}

// ---------------------------------------------------------------- wave search
// Frame lookup for a tile of 64 consecutive chunks [g0, g0+64): the frame of
// chunk g is the first i with chunk_end[i] > g.  wave_find_lo locates the
// tile's first frame from scratch; a wave walking consecutive tiles gets the
// next tile's first frame from next_tile_lo instead.
__device__ __forceinline__ uint32_t wave_find_lo(const uint32_t *__restrict__ chunk_end, uint32_t n, uint32_t g0)
{
    // first frame i with chunk_end[i] > g0 (the frame holding chunk g0):
    // 64-ary search with one coalesced probe per level
    const uint32_t lane = threadIdx.x & 63;
    uint32_t lo = 0, hi = n; // answer in [lo, hi]
    while (hi - lo > 64) {
        const uint32_t step = (hi - lo + 63) / 64;
        const uint32_t probe = lo + lane * step;
        const bool p = probe < hi && chunk_end[probe] > g0;
        const unsigned long long m = __ballot(p);
        if (m == 0) { // every probe below hi failed: answer is above the last one
            const uint32_t k = (hi - 1 - lo) / step;
            lo = lo + (k < 63 ? k : 63) * step + 1;
        } else {
            const uint32_t f = __builtin_ctzll(m);
            const uint32_t nhi = lo + f * step;
            lo = f ? lo + (f - 1) * step + 1 : lo;
            hi = nhi;
        }
    }
    const uint32_t probe = lo + lane;
    const bool p = probe < hi && chunk_end[probe] > g0;
    const unsigned long long m = __ballot(p);
    return m ? lo + (uint32_t) __builtin_ctzll(m) : hi;
}

// The 64 frames lo .. lo+63 cover the 64 chunks of a tile that starts in
// frame lo (each frame has >= 1 chunk).  window_load fetches their chunk
// ends (one coalesced load); window_find gives lane's frame for chunk g and
// that frame's chunk end.
__device__ __forceinline__ uint32_t window_load(const uint32_t *__restrict__ chunk_end, uint32_t n, uint32_t lo)
{
    // unconditional load (clamped index); window_find masks the lanes past
    // n when it uses the value, so nothing waits for the load here
    const uint32_t mine = lo + (threadIdx.x & 63);
    return chunk_end[mine < n ? mine : n - 1];
}

struct FrameLook {
    uint32_t i;  // frame holding the lane's chunk
    uint32_t ce; // chunk_end[i]
};

__device__ __forceinline__ FrameLook window_find(uint32_t ce_raw, uint32_t lo, uint32_t n, uint32_t g)
{
    const uint32_t ce = lo + (threadIdx.x & 63) < n ? ce_raw : 0xffffffffu;
    uint32_t a = 0; // first lane index j with ce_j > g
#pragma unroll
    for (int b = 32; b >= 1; b >>= 1) {
        const uint32_t v = __shfl(ce, (int) (a + b - 1));
        if (v <= g)
            a += b;
    }
    return FrameLook{lo + a, (uint32_t) __shfl(ce, (int) a)};
}

// First frame of the tile after the one described by `lk` (tile start t0):
// the frame of the tile's last chunk, or the one after it if that frame ends
// exactly at the next tile's start.
__device__ __forceinline__ uint32_t next_tile_lo(const FrameLook &lk, uint32_t next_t0)
{
    const uint32_t i63 = __shfl(lk.i, 63), ce63 = __shfl(lk.ce, 63);
    return ce63 > next_t0 ? i63 : i63 + 1;
}

} // namespace zmqg
