/*
 * keys_oracle.c -- CPU restatement of the key-handling helpers around the
 * CURVE path.  TEST INFRASTRUCTURE ONLY: the
 * checker for the device kernels, never linked into the product.
 *
 *   oracle_z85_encode / oracle_z85_decode
 *       zmq_z85_encode / zmq_z85_decode, reference src/zmq_utils.cpp:100-180
 *       (encoder / decoder tables :58-96).  Pinned by the reference's own
 *       vectors (tests/test_base85.cpp, tests/test_sodium.cpp key pair).
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#define EXPORT __attribute__((visibility("default")))

static const char z85_enc[86] = "0123456789abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ.-:+=^!/*?&<>()[]{}@%$#";

/* 0xff = not a digit; index = character - 32, as the reference's table */
static uint8_t z85_dec[96];
static int z85_ready;

static void z85_init(void)
{
    if (z85_ready)
        return;
    memset(z85_dec, 0xff, sizeof z85_dec);
    for (int i = 0; i < 85; ++i)
        z85_dec[(uint8_t) z85_enc[i] - 32] = (uint8_t) i;
    z85_ready = 1;
}

/* 0, or EINVAL (22) when size % 4 != 0 (nothing written) */
EXPORT int oracle_z85_encode(char *dest, const uint8_t *data, uint64_t size)
{
    if (size % 4 != 0)
        return 22;
    uint64_t c = 0;
    for (uint64_t b = 0; b < size; b += 4) {
        uint32_t v = ((uint32_t) data[b] << 24) | ((uint32_t) data[b + 1] << 16) | ((uint32_t) data[b + 2] << 8) |
                     data[b + 3];
        uint32_t div = 85u * 85u * 85u * 85u;
        while (div) {
            dest[c++] = z85_enc[v / div % 85u];
            div /= 85u;
        }
    }
    dest[c] = 0;
    return 0;
}

/* 0, or EINVAL (22); `len` is strlen(string).  Groups before an invalid one
 * are written, as the reference's loop writes each group as it completes. */
EXPORT int oracle_z85_decode(uint8_t *dest, const char *string, uint64_t len)
{
    z85_init();
    if (len < 5 || len % 5 != 0)
        return 22;
    uint64_t byte_nbr = 0, char_nbr = 0;
    uint32_t value = 0;
    while (char_nbr < len) {
        if (UINT32_MAX / 85 < value)
            return 22;
        value *= 85;
        const uint8_t index = (uint8_t) ((uint8_t) string[char_nbr++] - 32);
        if (index >= sizeof z85_dec)
            return 22;
        const uint32_t summand = z85_dec[index];
        if (summand == 0xff || summand > UINT32_MAX - value)
            return 22;
        value += summand;
        if (char_nbr % 5 == 0) {
            dest[byte_nbr++] = (uint8_t) (value >> 24);
            dest[byte_nbr++] = (uint8_t) (value >> 16);
            dest[byte_nbr++] = (uint8_t) (value >> 8);
            dest[byte_nbr++] = (uint8_t) value;
            value = 0;
        }
    }
    return 0;
}

/*
 *   oracle_x25519 / oracle_box_beforenm
 *       crypto_scalarmult_curve25519 and crypto_box_beforenm of libsodium
 *       1.0.18 (the third-party library behind the reference's
 *       src/curve_client_tools.hpp:105 and src/curve_server.cpp:382-383;
 *       its source is not in /root/reference): RFC 7748 section 5 X25519
 *       with libsodium's all-zero-result rejection, then HSalsa20 of the
 *       shared point with a zero input block.  Radix 2^51 with 128-bit
 *       products -- a different representation from the device's ten
 *       26/25-bit limbs, so the two cross-check each other.  Pinned by the
 *       RFC 7748 vectors, the NaCl crypto_box key and the reference's
 *       CURVE key pairs (tests/golden/x25519_vectors.json).
 */
typedef unsigned __int128 u128;
typedef struct {
    uint64_t v[5];
} fe51;

static const uint64_t M51 = (1ull << 51) - 1;

static void fe51_carry(fe51 *h, u128 t[5])
{
    uint64_t c;
    for (int i = 0; i < 4; ++i) {
        t[i + 1] += (uint64_t) (t[i] >> 51);
        t[i] &= M51;
    }
    c = (uint64_t) (t[4] >> 51);
    t[4] &= M51;
    t[0] += (u128) c * 19;
    c = (uint64_t) (t[0] >> 51);
    t[0] &= M51;
    t[1] += c;
    for (int i = 0; i < 5; ++i)
        h->v[i] = (uint64_t) t[i];
}

static void fe51_mul(fe51 *h, const fe51 *f, const fe51 *g)
{
    u128 t[5] = {0, 0, 0, 0, 0};
    for (int i = 0; i < 5; ++i)
        for (int j = 0; j < 5; ++j) {
            const u128 p = (u128) f->v[i] * g->v[j];
            if (i + j < 5)
                t[i + j] += p;
            else
                t[i + j - 5] += p * 19;
        }
    fe51_carry(h, t);
}

static void fe51_add(fe51 *h, const fe51 *f, const fe51 *g)
{
    for (int i = 0; i < 5; ++i)
        h->v[i] = f->v[i] + g->v[i];
}

/* f - g + 4p (limbs stay positive) */
static void fe51_sub(fe51 *h, const fe51 *f, const fe51 *g)
{
    static const uint64_t p4[5] = {0x1fffffffffffb4ull, 0x1ffffffffffffcull, 0x1ffffffffffffcull,
                                   0x1ffffffffffffcull, 0x1ffffffffffffcull};
    for (int i = 0; i < 5; ++i)
        h->v[i] = f->v[i] + p4[i] - g->v[i];
}

static void fe51_frombytes(fe51 *h, const uint8_t s[32])
{
    uint64_t w[4];
    for (int k = 0; k < 4; ++k) {
        uint64_t x = 0;
        for (int b = 0; b < 8; ++b)
            x |= (uint64_t) s[8 * k + b] << (8 * b);
        w[k] = x;
    }
    w[3] &= 0x7fffffffffffffffull; /* bit 255 ignored */
    h->v[0] = w[0] & M51;
    h->v[1] = ((w[0] >> 51) | (w[1] << 13)) & M51;
    h->v[2] = ((w[1] >> 38) | (w[2] << 26)) & M51;
    h->v[3] = ((w[2] >> 25) | (w[3] << 39)) & M51;
    h->v[4] = (w[3] >> 12) & M51;
}

static void fe51_tobytes(uint8_t s[32], const fe51 *f)
{
    u128 t[5];
    for (int i = 0; i < 5; ++i)
        t[i] = f->v[i];
    fe51 h;
    fe51_carry(&h, t);
    fe51_carry(&h, (u128[5]){h.v[0], h.v[1], h.v[2], h.v[3], h.v[4]});
    /* now h < 2^255 + small: subtract p if h >= p */
    uint64_t q = (h.v[0] + 19) >> 51;
    q = (h.v[1] + q) >> 51;
    q = (h.v[2] + q) >> 51;
    q = (h.v[3] + q) >> 51;
    q = (h.v[4] + q) >> 51;
    h.v[0] += 19 * q;
    for (int i = 0; i < 4; ++i) {
        h.v[i + 1] += h.v[i] >> 51;
        h.v[i] &= M51;
    }
    h.v[4] &= M51;
    const uint64_t w0 = h.v[0] | (h.v[1] << 51), w1 = (h.v[1] >> 13) | (h.v[2] << 38),
                   w2 = (h.v[2] >> 26) | (h.v[3] << 25), w3 = (h.v[3] >> 39) | (h.v[4] << 12);
    const uint64_t w[4] = {w0, w1, w2, w3};
    for (int k = 0; k < 4; ++k)
        for (int b = 0; b < 8; ++b)
            s[8 * k + b] = (uint8_t) (w[k] >> (8 * b));
}

static void fe51_cswap(fe51 *f, fe51 *g, uint64_t b)
{
    const uint64_t m = 0 - b;
    for (int i = 0; i < 5; ++i) {
        const uint64_t x = (f->v[i] ^ g->v[i]) & m;
        f->v[i] ^= x;
        g->v[i] ^= x;
    }
}

static void fe51_pow_p2(fe51 *out, const fe51 *z)
{
    /* z^(p-2) by square-and-multiply over the exponent bits 2^255 - 21 */
    fe51 r = {{1, 0, 0, 0, 0}};
    for (int bit = 254; bit >= 0; --bit) {
        fe51_mul(&r, &r, &r);
        /* p - 2 = 2^255 - 21: bits 254..5 set, bits 4..0 = 01011 */
        const int set = bit >= 5 ? 1 : ((0x0b >> bit) & 1);
        if (set)
            fe51_mul(&r, &r, z);
    }
    *out = r;
}

EXPORT int oracle_x25519(uint8_t out[32], const uint8_t scalar[32], const uint8_t u[32])
{
    uint8_t k[32];
    memcpy(k, scalar, 32);
    k[0] &= 248;
    k[31] &= 127;
    k[31] |= 64;
    fe51 x1, x2 = {{1, 0, 0, 0, 0}}, z2 = {{0, 0, 0, 0, 0}}, x3, z3 = {{1, 0, 0, 0, 0}};
    fe51_frombytes(&x1, u);
    x3 = x1;
    uint64_t swap = 0;
    const fe51 a24 = {{121665, 0, 0, 0, 0}};
    for (int t = 254; t >= 0; --t) {
        const uint64_t kt = (k[t >> 3] >> (t & 7)) & 1;
        swap ^= kt;
        fe51_cswap(&x2, &x3, swap);
        fe51_cswap(&z2, &z3, swap);
        swap = kt;
        fe51 A, AA, B, BB, E, C, D, DA, CB, t0;
        fe51_add(&A, &x2, &z2);
        fe51_mul(&AA, &A, &A);
        fe51_sub(&B, &x2, &z2);
        fe51_mul(&BB, &B, &B);
        fe51_sub(&E, &AA, &BB);
        fe51_add(&C, &x3, &z3);
        fe51_sub(&D, &x3, &z3);
        fe51_mul(&DA, &D, &A);
        fe51_mul(&CB, &C, &B);
        fe51_add(&t0, &DA, &CB);
        fe51_mul(&x3, &t0, &t0);
        fe51_sub(&t0, &DA, &CB);
        fe51_mul(&t0, &t0, &t0);
        fe51_mul(&z3, &x1, &t0);
        fe51_mul(&x2, &AA, &BB);
        fe51_mul(&t0, &a24, &E);
        fe51_add(&t0, &AA, &t0);
        fe51_mul(&z2, &E, &t0);
    }
    fe51_cswap(&x2, &x3, swap);
    fe51_cswap(&z2, &z3, swap);
    fe51 zi, r;
    fe51_pow_p2(&zi, &z2);
    fe51_mul(&r, &x2, &zi);
    fe51_tobytes(out, &r);
    uint8_t d = 0;
    for (int i = 0; i < 32; ++i)
        d |= out[i];
    return d ? 0 : -1;
}

void oracle_hsalsa20(uint8_t out[32], const uint8_t in[16], const uint8_t k[32]);

/* crypto_box_beforenm(k, pk, sk): -1 (k untouched) when the scalar
 * multiplication fails */
EXPORT int oracle_box_beforenm(uint8_t k[32], const uint8_t pk[32], const uint8_t sk[32])
{
    uint8_t s[32];
    static const uint8_t zero[16] = {0};
    if (oracle_x25519(s, sk, pk) != 0)
        return -1;
    oracle_hsalsa20(k, zero, s);
    return 0;
}
