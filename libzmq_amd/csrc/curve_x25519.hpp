// curve_x25519.hpp -- batched X25519 and crypto_box_beforenm for mass CURVE
// session setup.
//
// The handshake derives each connection's precomputed key with
// crypto_box_beforenm(precom, peer_public, own_secret)
// (reference src/curve_client_tools.hpp:105, src/curve_server.cpp:382-383)
// = HSalsa20(X25519(secret, public), 0^16) (libsodium 1.0.18,
// crypto_box_curve25519xsalsa20poly1305_beforenm), and zmq_curve_public
// (src/zmq_utils.cpp:222-245) derives a public key with
// crypto_scalarmult_base.  A server accepting thousands of connections does
// one of each per connection; here one thread does one key, 64 per wave.
//
// Arithmetic: GF(2^255 - 19) in ten signed limbs of 26, 25, 26, ... bits
// (limb i at bit ceil(25.5 i)); a product is 100 32x32->64 multiplies
// (v_mad_i64_i32) with the wrap-around terms pre-multiplied by 19 and the
// odd x odd terms doubled, then one carry chain.  The Montgomery ladder of
// RFC 7748 section 5 with a branch-free conditional swap; the inverse is
// z^(p-2).  Failure rule of libsodium's crypto_scalarmult_curve25519: an
// all-zero shared point (a small-order public key) returns -1, and
// crypto_box_beforenm then returns -1 without writing the key.
#pragma once

#include <stdint.h>

namespace zmqg {

struct fe10 {
    int32_t v[10];
};

__device__ __forceinline__ void fe_carry(int64_t h[10], fe10 &out)
{
    int64_t c;
    c = (h[0] + (1ll << 25)) >> 26; h[1] += c; h[0] -= c << 26;
    c = (h[4] + (1ll << 25)) >> 26; h[5] += c; h[4] -= c << 26;
    c = (h[1] + (1ll << 24)) >> 25; h[2] += c; h[1] -= c << 25;
    c = (h[5] + (1ll << 24)) >> 25; h[6] += c; h[5] -= c << 25;
    c = (h[2] + (1ll << 25)) >> 26; h[3] += c; h[2] -= c << 26;
    c = (h[6] + (1ll << 25)) >> 26; h[7] += c; h[6] -= c << 26;
    c = (h[3] + (1ll << 24)) >> 25; h[4] += c; h[3] -= c << 25;
    c = (h[7] + (1ll << 24)) >> 25; h[8] += c; h[7] -= c << 25;
    c = (h[4] + (1ll << 25)) >> 26; h[5] += c; h[4] -= c << 26;
    c = (h[8] + (1ll << 25)) >> 26; h[9] += c; h[8] -= c << 26;
    c = (h[9] + (1ll << 24)) >> 25; h[0] += c * 19; h[9] -= c << 25;
    c = (h[0] + (1ll << 25)) >> 26; h[1] += c; h[0] -= c << 26;
#pragma unroll
    for (int i = 0; i < 10; ++i)
        out.v[i] = (int32_t) h[i];
}

// h = f * g
__device__ __forceinline__ void fe10_mul(fe10 &h, const fe10 &f, const fe10 &g)
{
    int32_t g19[10], f2[10];
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        g19[i] = 19 * g.v[i];
        f2[i] = (i & 1) ? 2 * f.v[i] : f.v[i];
    }
    int64_t a[10];
#pragma unroll
    for (int k = 0; k < 10; ++k) {
        int64_t s = 0;
#pragma unroll
        for (int i = 0; i < 10; ++i) {
            const int j = k - i;
            // limb i * limb j lands on limb i + j (doubled when both are odd,
            // 19x when i + j >= 10: 2^255 = 19 mod p)
            if (j >= 0)
                s += (int64_t) ((j & 1) ? f2[i] : f.v[i]) * g.v[j];
            else
                s += (int64_t) ((j & 1) ? f2[i] : f.v[i]) * g19[j + 10];
        }
        a[k] = s;
    }
    fe_carry(a, h);
}

__device__ __forceinline__ void fe10_sq(fe10 &h, const fe10 &f)
{
    fe10_mul(h, f, f);
}

__device__ __forceinline__ void fe10_add(fe10 &h, const fe10 &f, const fe10 &g)
{
#pragma unroll
    for (int i = 0; i < 10; ++i)
        h.v[i] = f.v[i] + g.v[i];
}

__device__ __forceinline__ void fe10_sub(fe10 &h, const fe10 &f, const fe10 &g)
{
#pragma unroll
    for (int i = 0; i < 10; ++i)
        h.v[i] = f.v[i] - g.v[i];
}

// h = f * 121665 (a24 of RFC 7748)
__device__ __forceinline__ void fe10_mul_a24(fe10 &h, const fe10 &f)
{
    int64_t a[10];
#pragma unroll
    for (int i = 0; i < 10; ++i)
        a[i] = (int64_t) f.v[i] * 121665;
    fe_carry(a, h);
}

__device__ __forceinline__ void fe10_cswap(fe10 &f, fe10 &g, uint32_t b)
{
    const int32_t m = -(int32_t) b;
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        const int32_t x = (f.v[i] ^ g.v[i]) & m;
        f.v[i] ^= x;
        g.v[i] ^= x;
    }
}

// bit offset of limb i: 0, 26, 51, 77, 102, 128, 153, 179, 204, 230
__device__ constexpr int fe_bit(int i)
{
    return (51 * i + 1) / 2;
}

// 32 little-endian bytes -> limbs (bit 255 ignored, RFC 7748 section 5)
__device__ __forceinline__ void fe10_frombytes(fe10 &h, const uint8_t *s)
{
    uint64_t w[5];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        uint64_t x = 0;
#pragma unroll
        for (int b = 0; b < 8; ++b)
            x |= (uint64_t) s[8 * k + b] << (8 * b);
        w[k] = x;
    }
    w[4] = 0;
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        const int bit = fe_bit(i), wi = bit >> 6, sh = bit & 63, width = (i & 1) ? 25 : 26;
        uint64_t x = w[wi] >> sh;
        if (sh + width > 64)
            x |= w[wi + 1] << (64 - sh);
        h.v[i] = (int32_t) (x & ((1ull << width) - 1));
    }
}

// canonical little-endian encoding (the value mod p)
__device__ __forceinline__ void fe10_tobytes(uint8_t *s, const fe10 &f)
{
    int64_t h[10];
#pragma unroll
    for (int i = 0; i < 10; ++i)
        h[i] = f.v[i];
    // q = floor(h / p) for the carried (bounded) limbs: 0 or 1
    int64_t q = (19 * h[9] + (1ll << 24)) >> 25;
#pragma unroll
    for (int i = 0; i < 10; ++i)
        q = (h[i] + q) >> ((i & 1) ? 25 : 26);
    h[0] += 19 * q;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        const int w = (i & 1) ? 25 : 26;
        const int64_t c = h[i] >> w;
        h[i + 1] += c;
        h[i] -= c << w;
    }
    h[9] &= (1ll << 25) - 1; // drops q * 2^255
    uint64_t w[4] = {0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        const int bit = fe_bit(i), wi = bit >> 6, sh = bit & 63;
        const uint64_t x = (uint64_t) h[i];
        w[wi] |= x << sh;
        if (sh + ((i & 1) ? 25 : 26) > 64)
            w[wi + 1] |= x >> (64 - sh);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int b = 0; b < 8; ++b)
            s[8 * k + b] = (uint8_t) (w[k] >> (8 * b));
}

__device__ __forceinline__ void fe10_sqn(fe10 &h, const fe10 &f, int n)
{
    fe10_sq(h, f);
    for (int i = 1; i < n; ++i)
        fe10_sq(h, h);
}

// z^(p-2) = z^(2^255 - 21)
__device__ __forceinline__ void fe10_invert(fe10 &out, const fe10 &z)
{
    fe10 t0, t1, t2, t3;
    fe10_sq(t0, z);          // 2
    fe10_sqn(t1, t0, 2);     // 8
    fe10_mul(t1, z, t1);     // 9
    fe10_mul(t0, t0, t1);    // 11
    fe10_sq(t2, t0);         // 22
    fe10_mul(t1, t1, t2);    // 2^5 - 1
    fe10_sqn(t2, t1, 5);
    fe10_mul(t1, t2, t1);    // 2^10 - 1
    fe10_sqn(t2, t1, 10);
    fe10_mul(t2, t2, t1);    // 2^20 - 1
    fe10_sqn(t3, t2, 20);
    fe10_mul(t2, t3, t2);    // 2^40 - 1
    fe10_sqn(t2, t2, 10);
    fe10_mul(t1, t2, t1);    // 2^50 - 1
    fe10_sqn(t2, t1, 50);
    fe10_mul(t2, t2, t1);    // 2^100 - 1
    fe10_sqn(t3, t2, 100);
    fe10_mul(t2, t3, t2);    // 2^200 - 1
    fe10_sqn(t2, t2, 50);
    fe10_mul(t1, t2, t1);    // 2^250 - 1
    fe10_sqn(t1, t1, 5);     // 2^255 - 32
    fe10_mul(out, t1, t0);   // 2^255 - 21
}

// X25519(scalar, u): RFC 7748 section 5.  Returns 0, or -1 when the result
// is all zero (libsodium's check in crypto_scalarmult_curve25519).
__device__ __forceinline__ int x25519(uint8_t out[32], const uint8_t scalar[32], const uint8_t u[32])
{
    uint64_t k[4]; // the clamped scalar (RFC 7748 decodeScalar25519)
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        uint64_t x = 0;
#pragma unroll
        for (int b = 0; b < 8; ++b)
            x |= (uint64_t) scalar[8 * w + b] << (8 * b);
        k[w] = x;
    }
    k[0] &= ~7ull;
    k[3] &= ~(1ull << 63);
    k[3] |= 1ull << 62;
    fe10 x1, x2, z2, x3, z3;
    fe10_frombytes(x1, u);
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        x2.v[i] = i == 0;
        z2.v[i] = 0;
        x3.v[i] = x1.v[i];
        z3.v[i] = i == 0;
    }
    uint32_t swap = 0;
    for (int t = 254; t >= 0; --t) {
        const uint64_t kw = t >= 192 ? k[3] : t >= 128 ? k[2] : t >= 64 ? k[1] : k[0]; // t is wave-uniform
        const uint32_t kt = (uint32_t) (kw >> (t & 63)) & 1u;
        swap ^= kt;
        fe10_cswap(x2, x3, swap);
        fe10_cswap(z2, z3, swap);
        swap = kt;
        fe10 A, B, C, D, AA, BB, E, DA, CB, t0;
        fe10_add(A, x2, z2);
        fe10_sq(AA, A);
        fe10_sub(B, x2, z2);
        fe10_sq(BB, B);
        fe10_sub(E, AA, BB);
        fe10_add(C, x3, z3);
        fe10_sub(D, x3, z3);
        fe10_mul(DA, D, A);
        fe10_mul(CB, C, B);
        fe10_add(t0, DA, CB);
        fe10_sq(x3, t0);
        fe10_sub(t0, DA, CB);
        fe10_sq(t0, t0);
        fe10_mul(z3, x1, t0);
        fe10_mul(x2, AA, BB);
        fe10_mul_a24(t0, E);
        fe10_add(t0, AA, t0);
        fe10_mul(z2, E, t0);
    }
    fe10_cswap(x2, x3, swap);
    fe10_cswap(z2, z3, swap);
    fe10 zi, r;
    fe10_invert(zi, z2);
    fe10_mul(r, x2, zi);
    fe10_tobytes(out, r);
    uint32_t d = 0;
#pragma unroll
    for (int i = 0; i < 32; ++i)
        d |= out[i];
    return d ? 0 : -1;
}

// point == nullptr: the base point u = 9 (crypto_scalarmult_base; never fails)
__global__ __launch_bounds__(64) void k_scalarmult(uint32_t n, const uint8_t *__restrict__ scalar,
                                                   const uint8_t *__restrict__ point, uint8_t *__restrict__ out,
                                                   int32_t *__restrict__ status)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    uint8_t s[32], u[32], q[32];
#pragma unroll
    for (int b = 0; b < 32; ++b) {
        s[b] = scalar[32ull * i + b];
        u[b] = point ? point[32ull * i + b] : (b == 0 ? 9 : 0);
    }
    const int rc = x25519(q, s, u);
#pragma unroll
    for (int b = 0; b < 32; ++b)
        out[32ull * i + b] = q[b];
    status[i] = point ? rc : 0;
}

// crypto_box_beforenm(k, pk, sk) = HSalsa20(X25519(sk, pk), 0^16); on
// failure k is not written (libsodium returns before the core)
__global__ __launch_bounds__(64) void k_beforenm(uint32_t n, const uint8_t *__restrict__ pk,
                                                 const uint8_t *__restrict__ sk, uint8_t *__restrict__ k_out,
                                                 int32_t *__restrict__ status)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    uint8_t s[32], u[32], q[32];
#pragma unroll
    for (int b = 0; b < 32; ++b) {
        s[b] = sk[32ull * i + b];
        u[b] = pk[32ull * i + b];
    }
    const int rc = x25519(q, s, u);
    status[i] = rc;
    if (rc != 0)
        return;
    uint32_t kw[8], zero[4] = {0, 0, 0, 0}, o[8];
#pragma unroll
    for (int w = 0; w < 8; ++w)
        kw[w] = (uint32_t) q[4 * w] | ((uint32_t) q[4 * w + 1] << 8) | ((uint32_t) q[4 * w + 2] << 16) |
                ((uint32_t) q[4 * w + 3] << 24);
    hsalsa20(o, kw, zero);
#pragma unroll
    for (int w = 0; w < 8; ++w)
#pragma unroll
        for (int b = 0; b < 4; ++b)
            k_out[32ull * i + 4 * w + b] = (uint8_t) (o[w] >> (8 * b));
}

} // namespace zmqg
