/*
 * curve_oracle.c -- CPU restatement of the CurveZMQ MESSAGE AEAD path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py load this library, and only as the checker /
 * the timed CPU baseline.  The product (libzmq_amd/, libzmqg_curve.so) never
 * links or calls it.
 *
 * What it restates
 *   - curve_encoding_t::encode          reference src/curve_mechanism_base.cpp:111-205
 *   - curve_encoding_t::decode          reference src/curve_mechanism_base.cpp:207-284
 *   - curve_encoding_t::check_validity  reference src/curve_mechanism_base.cpp:80-109
 *   - mechanism_base_t::check_basic_command_structure
 *                                       reference src/mechanism_base.cpp:14-25
 *   - big-endian nonce helpers          reference src/wire.hpp:51-73
 *   - the crypto the reference calls (src/curve_mechanism_base.cpp:172-174,
 *     226-228): libsodium 1.0.18 crypto_box_easy_afternm /
 *     crypto_box_open_easy_afternm.  libsodium is a third-party dependency not
 *     present in /root/reference; its published algorithm is restated here:
 *     XSalsa20 (HSalsa20 subkey + Salsa20/20, Bernstein "Extending the Salsa20
 *     nonce" and "The Salsa20 family of stream ciphers") and Poly1305
 *     (Bernstein, "The Poly1305-AES message-authentication code"), composed
 *     as NaCl's crypto_secretbox: keystream bytes 0..31 are the one-time
 *     Poly1305 key, plaintext byte i is XORed with keystream byte 32+i, and
 *     the box is tag(16) || ciphertext.
 *
 * Parity pin: tests/golden/curve_golden.json (libsodium 1.0.18 outputs, the
 * NaCl box KAT, and the wire prefix the survey recorded from the compiled
 * reference).  See tests/test_oracle_golden.py.
 *
 * Batch layout mirrors include/zmqg_curve.h so tests can compare the GPU path
 * and this oracle on identical descriptor arrays.
 */
#include <dlfcn.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define EXPORT __attribute__((visibility("default")))

/* include/zmq.h:424-437 */
#define ERR_UNEXPECTED_COMMAND 0x10000001
#define ERR_INVALID_SEQUENCE 0x10000002
#define ERR_MALFORMED_UNSPECIFIED 0x10000011
#define ERR_MALFORMED_MESSAGE 0x10000012
#define ERR_CRYPTOGRAPHIC 0x11000001

/* src/msg.hpp:16, 55-62, 30-31 */
#define F_MORE 1
#define F_COMMAND 2
#define F_SUBSCRIBE 12
#define F_CANCEL 16
#define CMD_TYPE_MASK 0x1c
static const uint8_t SUB_CMD[10] = {9, 'S', 'U', 'B', 'S', 'C', 'R', 'I', 'B', 'E'};
static const uint8_t CANCEL_CMD[7] = {6, 'C', 'A', 'N', 'C', 'E', 'L'};
static const uint8_t MESSAGE_CMD[8] = {7, 'M', 'E', 'S', 'S', 'A', 'G', 'E'};

/* ------------------------------------------------------------------ */
/* deterministic test bytes (splitmix64), mirrored in tests/golden     */
/* ------------------------------------------------------------------ */
EXPORT void oracle_splitmix_bytes(uint64_t seed, uint8_t *out, uint64_t n)
{
    uint64_t x = seed;
    uint64_t i = 0;
    while (i < n) {
        x += 0x9E3779B97F4A7C15ull;
        uint64_t z = x;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        for (int b = 0; b < 8 && i < n; ++b, ++i)
            out[i] = (uint8_t) (z >> (8 * b));
    }
}

/* ------------------------------------------------------------------ */
/* Salsa20 / HSalsa20                                                  */
/* ------------------------------------------------------------------ */
static uint32_t ld32(const uint8_t *p)
{
    return (uint32_t) p[0] | ((uint32_t) p[1] << 8) | ((uint32_t) p[2] << 16)
           | ((uint32_t) p[3] << 24);
}
static void st32(uint8_t *p, uint32_t v)
{
    p[0] = (uint8_t) v;
    p[1] = (uint8_t) (v >> 8);
    p[2] = (uint8_t) (v >> 16);
    p[3] = (uint8_t) (v >> 24);
}
#define ROTL(v, c) (((v) << (c)) | ((v) >> (32 - (c))))

/* 20 rounds over x[16] in place (10 column/row double rounds). */
static void salsa_rounds(uint32_t x[16])
{
    for (int i = 0; i < 10; ++i) {
        x[4] ^= ROTL(x[0] + x[12], 7);   x[8] ^= ROTL(x[4] + x[0], 9);
        x[12] ^= ROTL(x[8] + x[4], 13);  x[0] ^= ROTL(x[12] + x[8], 18);
        x[9] ^= ROTL(x[5] + x[1], 7);    x[13] ^= ROTL(x[9] + x[5], 9);
        x[1] ^= ROTL(x[13] + x[9], 13);  x[5] ^= ROTL(x[1] + x[13], 18);
        x[14] ^= ROTL(x[10] + x[6], 7);  x[2] ^= ROTL(x[14] + x[10], 9);
        x[6] ^= ROTL(x[2] + x[14], 13);  x[10] ^= ROTL(x[6] + x[2], 18);
        x[3] ^= ROTL(x[15] + x[11], 7);  x[7] ^= ROTL(x[3] + x[15], 9);
        x[11] ^= ROTL(x[7] + x[3], 13);  x[15] ^= ROTL(x[11] + x[7], 18);

        x[1] ^= ROTL(x[0] + x[3], 7);    x[2] ^= ROTL(x[1] + x[0], 9);
        x[3] ^= ROTL(x[2] + x[1], 13);   x[0] ^= ROTL(x[3] + x[2], 18);
        x[6] ^= ROTL(x[5] + x[4], 7);    x[7] ^= ROTL(x[6] + x[5], 9);
        x[4] ^= ROTL(x[7] + x[6], 13);   x[5] ^= ROTL(x[4] + x[7], 18);
        x[11] ^= ROTL(x[10] + x[9], 7);  x[8] ^= ROTL(x[11] + x[10], 9);
        x[9] ^= ROTL(x[8] + x[11], 13);  x[10] ^= ROTL(x[9] + x[8], 18);
        x[12] ^= ROTL(x[15] + x[14], 7); x[13] ^= ROTL(x[12] + x[15], 9);
        x[14] ^= ROTL(x[13] + x[12], 13); x[15] ^= ROTL(x[14] + x[13], 18);
    }
}

/* "expand 32-byte k" */
static const uint32_t SIGMA[4] = {0x61707865, 0x3320646e, 0x79622d32, 0x6b206574};

static void salsa_input(uint32_t in[16], const uint8_t k[32], const uint8_t mid[16])
{
    in[0] = SIGMA[0];
    in[5] = SIGMA[1];
    in[10] = SIGMA[2];
    in[15] = SIGMA[3];
    for (int i = 0; i < 4; ++i) {
        in[1 + i] = ld32(k + 4 * i);
        in[11 + i] = ld32(k + 16 + 4 * i);
        in[6 + i] = ld32(mid + 4 * i);
    }
}

EXPORT void oracle_hsalsa20(uint8_t out[32], const uint8_t in16[16], const uint8_t k[32])
{
    uint32_t x[16];
    salsa_input(x, k, in16);
    salsa_rounds(x);
    static const int pick[8] = {0, 5, 10, 15, 6, 7, 8, 9};
    for (int i = 0; i < 8; ++i)
        st32(out + 4 * i, x[pick[i]]);
}

/* One 64-byte Salsa20 block: key k, 8-byte nonce n, 64-bit block counter. */
static void salsa20_block(uint8_t out[64], const uint8_t k[32], const uint8_t n[8], uint64_t ctr)
{
    uint8_t mid[16];
    memcpy(mid, n, 8);
    for (int i = 0; i < 8; ++i)
        mid[8 + i] = (uint8_t) (ctr >> (8 * i));
    uint32_t in[16], x[16];
    salsa_input(in, k, mid);
    memcpy(x, in, sizeof x);
    salsa_rounds(x);
    for (int i = 0; i < 16; ++i)
        st32(out + 4 * i, x[i] + in[i]);
}

EXPORT void oracle_salsa20_stream(uint8_t *out, uint64_t len, const uint8_t n[8], const uint8_t k[32])
{
    uint8_t blk[64];
    for (uint64_t off = 0, ctr = 0; off < len; off += 64, ++ctr) {
        salsa20_block(blk, k, n, ctr);
        uint64_t take = len - off < 64 ? len - off : 64;
        memcpy(out + off, blk, take);
    }
}

/* ------------------------------------------------------------------ */
/* Poly1305, radix 2^26                                               */
/* ------------------------------------------------------------------ */
typedef struct {
    uint32_t r[5], h[5], pad[4];
} poly_state;

static void poly_init(poly_state *st, const uint8_t key[32])
{
    /* clamp r: r &= 0x0ffffffc0ffffffc0ffffffc0fffffff */
    st->r[0] = (ld32(key + 0)) & 0x3ffffff;
    st->r[1] = (ld32(key + 3) >> 2) & 0x3ffff03;
    st->r[2] = (ld32(key + 6) >> 4) & 0x3ffc0ff;
    st->r[3] = (ld32(key + 9) >> 6) & 0x3f03fff;
    st->r[4] = (ld32(key + 12) >> 8) & 0x00fffff;
    memset(st->h, 0, sizeof st->h);
    for (int i = 0; i < 4; ++i)
        st->pad[i] = ld32(key + 16 + 4 * i);
}

/* h = (h + block) * r mod 2^130-5.  hibit = 2^128 for full blocks; a final
 * partial block is padded with 0x01 then zeros and carries no 2^128 bit. */
static void poly_block(poly_state *st, const uint8_t m[16], uint32_t hibit)
{
    const uint32_t r0 = st->r[0], r1 = st->r[1], r2 = st->r[2], r3 = st->r[3], r4 = st->r[4];
    const uint32_t s1 = r1 * 5, s2 = r2 * 5, s3 = r3 * 5, s4 = r4 * 5;
    uint32_t h0 = st->h[0], h1 = st->h[1], h2 = st->h[2], h3 = st->h[3], h4 = st->h[4];
    h0 += (ld32(m + 0)) & 0x3ffffff;
    h1 += (ld32(m + 3) >> 2) & 0x3ffffff;
    h2 += (ld32(m + 6) >> 4) & 0x3ffffff;
    h3 += (ld32(m + 9) >> 6) & 0x3ffffff;
    h4 += (ld32(m + 12) >> 8) | hibit;
    uint64_t d0 = (uint64_t) h0 * r0 + (uint64_t) h1 * s4 + (uint64_t) h2 * s3 + (uint64_t) h3 * s2 + (uint64_t) h4 * s1;
    uint64_t d1 = (uint64_t) h0 * r1 + (uint64_t) h1 * r0 + (uint64_t) h2 * s4 + (uint64_t) h3 * s3 + (uint64_t) h4 * s2;
    uint64_t d2 = (uint64_t) h0 * r2 + (uint64_t) h1 * r1 + (uint64_t) h2 * r0 + (uint64_t) h3 * s4 + (uint64_t) h4 * s3;
    uint64_t d3 = (uint64_t) h0 * r3 + (uint64_t) h1 * r2 + (uint64_t) h2 * r1 + (uint64_t) h3 * r0 + (uint64_t) h4 * s4;
    uint64_t d4 = (uint64_t) h0 * r4 + (uint64_t) h1 * r3 + (uint64_t) h2 * r2 + (uint64_t) h3 * r1 + (uint64_t) h4 * r0;
    uint32_t c;
    c = (uint32_t) (d0 >> 26); h0 = (uint32_t) d0 & 0x3ffffff;
    d1 += c; c = (uint32_t) (d1 >> 26); h1 = (uint32_t) d1 & 0x3ffffff;
    d2 += c; c = (uint32_t) (d2 >> 26); h2 = (uint32_t) d2 & 0x3ffffff;
    d3 += c; c = (uint32_t) (d3 >> 26); h3 = (uint32_t) d3 & 0x3ffffff;
    d4 += c; c = (uint32_t) (d4 >> 26); h4 = (uint32_t) d4 & 0x3ffffff;
    h0 += c * 5; c = h0 >> 26; h0 &= 0x3ffffff;
    h1 += c;
    st->h[0] = h0; st->h[1] = h1; st->h[2] = h2; st->h[3] = h3; st->h[4] = h4;
}

static void poly_update(poly_state *st, const uint8_t *m, uint64_t len)
{
    while (len >= 16) {
        poly_block(st, m, 1u << 24);
        m += 16;
        len -= 16;
    }
    if (len) {
        uint8_t last[16] = {0};
        memcpy(last, m, len);
        last[len] = 1;
        poly_block(st, last, 0);
    }
}

static void poly_finish(poly_state *st, uint8_t tag[16])
{
    uint32_t h0 = st->h[0], h1 = st->h[1], h2 = st->h[2], h3 = st->h[3], h4 = st->h[4], c;
    c = h1 >> 26; h1 &= 0x3ffffff;
    h2 += c; c = h2 >> 26; h2 &= 0x3ffffff;
    h3 += c; c = h3 >> 26; h3 &= 0x3ffffff;
    h4 += c; c = h4 >> 26; h4 &= 0x3ffffff;
    h0 += c * 5; c = h0 >> 26; h0 &= 0x3ffffff;
    h1 += c;
    /* g = h + 5 - 2^130; select g when it did not borrow (h >= p) */
    uint32_t g0 = h0 + 5; c = g0 >> 26; g0 &= 0x3ffffff;
    uint32_t g1 = h1 + c; c = g1 >> 26; g1 &= 0x3ffffff;
    uint32_t g2 = h2 + c; c = g2 >> 26; g2 &= 0x3ffffff;
    uint32_t g3 = h3 + c; c = g3 >> 26; g3 &= 0x3ffffff;
    uint32_t g4 = h4 + c - (1u << 26);
    uint32_t mask = (g4 >> 31) - 1; /* all ones when g4 did not go negative */
    h0 = (h0 & ~mask) | (g0 & mask);
    h1 = (h1 & ~mask) | (g1 & mask);
    h2 = (h2 & ~mask) | (g2 & mask);
    h3 = (h3 & ~mask) | (g3 & mask);
    h4 = (h4 & ~mask) | (g4 & mask);
    /* to 4 x 32 bits, then + pad mod 2^128 */
    uint64_t f0 = ((h0) | (h1 << 26)) + (uint64_t) st->pad[0];
    uint64_t f1 = ((h1 >> 6) | (h2 << 20)) + (uint64_t) st->pad[1];
    uint64_t f2 = ((h2 >> 12) | (h3 << 14)) + (uint64_t) st->pad[2];
    uint64_t f3 = ((h3 >> 18) | (h4 << 8)) + (uint64_t) st->pad[3];
    st32(tag + 0, (uint32_t) f0); f1 += f0 >> 32;
    st32(tag + 4, (uint32_t) f1); f2 += f1 >> 32;
    st32(tag + 8, (uint32_t) f2); f3 += f2 >> 32;
    st32(tag + 12, (uint32_t) f3);
}

EXPORT void oracle_poly1305(uint8_t tag[16], const uint8_t *m, uint64_t len, const uint8_t key[32])
{
    poly_state st;
    poly_init(&st, key);
    poly_update(&st, m, len);
    poly_finish(&st, tag);
}

/* ------------------------------------------------------------------ */
/* crypto_box_easy_afternm / crypto_box_open_easy_afternm restatement  */
/* (= crypto_secretbox_easy with subkey HSalsa20(k, n[0:16]))          */
/* ------------------------------------------------------------------ */
/* Keystream XOR for bytes [0, len) of the message, starting at keystream
 * byte 32 of the XSalsa20 stream (block 0 bytes 0..31 are the Poly1305 key). */
static void xsalsa_xor(uint8_t *dst, const uint8_t *src, uint64_t len,
                       const uint8_t subkey[32], const uint8_t n8[8], uint8_t polykey[32])
{
    uint8_t blk[64];
    salsa20_block(blk, subkey, n8, 0);
    memcpy(polykey, blk, 32);
    uint64_t first = len < 32 ? len : 32;
    for (uint64_t i = 0; i < first; ++i)
        dst[i] = src[i] ^ blk[32 + i];
    uint64_t ctr = 1;
    for (uint64_t off = first; off < len; off += 64, ++ctr) {
        salsa20_block(blk, subkey, n8, ctr);
        uint64_t take = len - off < 64 ? len - off : 64;
        for (uint64_t i = 0; i < take; ++i)
            dst[off + i] = src[off + i] ^ blk[i];
    }
}

/* c = tag(16) || ct(mlen) */
EXPORT int oracle_box_easy_afternm(uint8_t *c, const uint8_t *m, uint64_t mlen,
                                   const uint8_t n[24], const uint8_t k[32])
{
    uint8_t subkey[32], polykey[32];
    oracle_hsalsa20(subkey, n, k);
    xsalsa_xor(c + 16, m, mlen, subkey, n + 16, polykey);
    oracle_poly1305(c, c + 16, mlen, polykey);
    return 0;
}

/* m(clen-16) from c = tag || ct; verifies before decrypting; -1 on forgery. */
EXPORT int oracle_box_open_easy_afternm(uint8_t *m, const uint8_t *c, uint64_t clen,
                                        const uint8_t n[24], const uint8_t k[32])
{
    if (clen < 16)
        return -1;
    uint8_t subkey[32], blk[64], tag[16];
    oracle_hsalsa20(subkey, n, k);
    salsa20_block(blk, subkey, n + 16, 0);
    oracle_poly1305(tag, c + 16, clen - 16, blk);
    uint8_t diff = 0;
    for (int i = 0; i < 16; ++i)
        diff |= (uint8_t) (tag[i] ^ c[i]);
    if (diff)
        return -1;
    uint8_t polykey[32];
    xsalsa_xor(m, c + 16, clen - 16, subkey, n + 16, polykey);
    return 0;
}

/* ------------------------------------------------------------------ */
/* CURVE MESSAGE framing                                              */
/* ------------------------------------------------------------------ */
static void put_u64_be(uint8_t *p, uint64_t v) /* src/wire.hpp:51-61 */
{
    for (int i = 0; i < 8; ++i)
        p[i] = (uint8_t) (v >> (56 - 8 * i));
}
static uint64_t get_u64_be(const uint8_t *p) /* src/wire.hpp:63-73 */
{
    uint64_t v = 0;
    for (int i = 0; i < 8; ++i)
        v = (v << 8) | p[i];
    return v;
}

/* Plaintext header restated from src/curve_mechanism_base.cpp:118-158:
 * byte 0 = flags & (more|command); SUBSCRIBE/CANCEL either downgrade to one
 * 0/1 byte or get the command bit and the "\x09SUBSCRIBE"/"\x06CANCEL" name. */
EXPORT uint32_t oracle_plaintext_header(uint8_t hdr[11], uint8_t msg_flags, int downgrade_sub)
{
    const int is_sub = (msg_flags & CMD_TYPE_MASK) == F_SUBSCRIBE;
    const int is_cancel = (msg_flags & CMD_TYPE_MASK) == F_CANCEL;
    hdr[0] = msg_flags & (F_MORE | F_COMMAND);
    if (!(is_sub || is_cancel))
        return 1;
    if (downgrade_sub) {
        hdr[1] = is_sub ? 1 : 0;
        return 2;
    }
    hdr[0] |= F_COMMAND;
    if (is_cancel) {
        memcpy(hdr + 1, CANCEL_CMD, sizeof CANCEL_CMD);
        return 1 + sizeof CANCEL_CMD;
    }
    memcpy(hdr + 1, SUB_CMD, sizeof SUB_CMD);
    return 1 + sizeof SUB_CMD;
}

/* Wire size of one encoded message: "\x07MESSAGE"(8) + nonce(8) + tag(16) + mlen. */
EXPORT uint64_t oracle_wire_size(uint8_t msg_flags, int downgrade_sub, uint64_t payload_len)
{
    uint8_t hdr[11];
    return 32 + oracle_plaintext_header(hdr, msg_flags, downgrade_sub) + payload_len;
}

typedef int (*box_fn)(uint8_t *, const uint8_t *, unsigned long long, const uint8_t *, const uint8_t *);

static int box_portable(uint8_t *c, const uint8_t *m, unsigned long long mlen, const uint8_t *n, const uint8_t *k)
{
    return oracle_box_easy_afternm(c, m, mlen, n, k);
}
static int open_portable(uint8_t *m, const uint8_t *c, unsigned long long clen, const uint8_t *n, const uint8_t *k)
{
    return oracle_box_open_easy_afternm(m, c, clen, n, k);
}

/* curve_encoding_t::encode for one message (src/curve_mechanism_base.cpp:111-205).
 * scratch must hold >= 11 + len bytes (the reference's std::vector plaintext). */
static void curve_encode_one(box_fn box, uint8_t *wire, uint8_t *scratch, const uint8_t precom[32],
                             const uint8_t prefix[16], uint64_t nonce, uint8_t msg_flags,
                             int downgrade_sub, const uint8_t *payload, uint64_t len)
{
    uint8_t n24[24];
    memcpy(n24, prefix, 16);
    put_u64_be(n24 + 16, nonce);
    uint32_t hl = oracle_plaintext_header(scratch, msg_flags, downgrade_sub);
    if (len)
        memcpy(scratch + hl, payload, len);
    box(wire + 16, scratch, hl + len, n24, precom);
    memcpy(wire, MESSAGE_CMD, 8);
    memcpy(wire + 8, n24 + 16, 8);
}

/* curve_mechanism_base_t::decode (src/curve_mechanism_base.cpp:38-52) for one
 * message: basic structure check, check_validity, open, flags.  Returns the
 * status (0 or a ZMQ_PROTOCOL_ERROR_* code) and updates *peer_nonce exactly as
 * the reference does (before the MAC check).  scratch >= wire_len bytes. */
static int32_t curve_decode_one(box_fn open, uint8_t *payload_out, uint8_t *flags_out, uint8_t *scratch,
                                const uint8_t precom[32], const uint8_t prefix[16], uint64_t *peer_nonce,
                                const uint8_t *wire, uint64_t wire_len)
{
    *flags_out = 0;
    if (wire_len <= 1 || wire_len <= wire[0])
        return ERR_MALFORMED_UNSPECIFIED; /* src/mechanism_base.cpp:16-22 */
    if (wire_len < 8 || memcmp(wire, MESSAGE_CMD, 8) != 0)
        return ERR_UNEXPECTED_COMMAND; /* :85-90 */
    if (wire_len < 16 + 16 + 1)
        return ERR_MALFORMED_MESSAGE; /* :92-96 */
    const uint64_t nonce = get_u64_be(wire + 8);
    if (nonce <= *peer_nonce)
        return ERR_INVALID_SEQUENCE; /* :99-104 */
    *peer_nonce = nonce; /* :105, before the MAC check */
    uint8_t n24[24];
    memcpy(n24, prefix, 16);
    memcpy(n24 + 16, wire + 8, 8);
    if (open(scratch, wire + 16, wire_len - 16, n24, precom) != 0)
        return ERR_CRYPTOGRAPHIC; /* :277-281 */
    *flags_out = scratch[0] & (F_MORE | F_COMMAND);
    if (wire_len - 33)
        memcpy(payload_out, scratch + 1, wire_len - 33);
    return 0;
}

/* ------------------------------------------------------------------ */
/* Batch entry points (layout of include/zmqg_curve.h)                 */
/* ------------------------------------------------------------------ */
typedef struct {
    uint8_t precom[32];
    uint8_t enc_prefix[16];
    uint8_t dec_prefix[16];
    int32_t downgrade_sub;
} oracle_session;

EXPORT uint64_t oracle_session_size(void) { return sizeof(oracle_session); }

EXPORT int oracle_encode_batch(const oracle_session *sessions, uint64_t n, const uint32_t *sid,
                               const uint64_t *nonce, const uint8_t *flags, const uint64_t *in_off,
                               const uint32_t *len, const uint8_t *in, const uint64_t *out_off,
                               uint8_t *out)
{
    uint64_t maxlen = 0;
    for (uint64_t i = 0; i < n; ++i)
        if (len[i] > maxlen)
            maxlen = len[i];
    uint8_t *scratch = (uint8_t *) malloc(maxlen + 16);
    if (!scratch)
        return -1;
    for (uint64_t i = 0; i < n; ++i) {
        const oracle_session *s = &sessions[sid[i]];
        curve_encode_one(box_portable, out + out_off[i], scratch, s->precom, s->enc_prefix, nonce[i],
                         flags[i], s->downgrade_sub, in + in_off[i], len[i]);
    }
    free(scratch);
    return 0;
}

/* Messages are decoded in batch order, as the engine would call
 * curve_encoding_t::decode one by one.  peer_nonce[sid] is read and updated. */
EXPORT int oracle_decode_batch(const oracle_session *sessions, uint64_t *peer_nonce, uint64_t n,
                               const uint32_t *sid, const uint64_t *in_off, const uint32_t *wire_len,
                               const uint8_t *in, const uint64_t *out_off, uint8_t *out,
                               uint8_t *flags_out, int32_t *status_out)
{
    uint64_t maxlen = 0;
    for (uint64_t i = 0; i < n; ++i)
        if (wire_len[i] > maxlen)
            maxlen = wire_len[i];
    uint8_t *scratch = (uint8_t *) malloc(maxlen + 16);
    if (!scratch)
        return -1;
    for (uint64_t i = 0; i < n; ++i) {
        const oracle_session *s = &sessions[sid[i]];
        status_out[i] = curve_decode_one(open_portable, out + out_off[i], &flags_out[i], scratch, s->precom,
                                         s->dec_prefix, &peer_nonce[sid[i]], in + in_off[i], wire_len[i]);
    }
    free(scratch);
    return 0;
}

/* ------------------------------------------------------------------ */
/* Timed CPU baseline: encode+decode round trips on T threads.         */
/* Sessions are partitioned across threads (one engine/I-O thread owns */
/* a connection, src/stream_engine_base.cpp).  Crypto either the       */
/* portable restatement above or the box's libsodium via dlopen.       */
/* ------------------------------------------------------------------ */
typedef struct {
    box_fn box, open;
    const oracle_session *sessions;
    uint64_t n;
    const uint32_t *sid;
    const uint64_t *nonce;
    const uint8_t *flags;
    const uint64_t *in_off;
    const uint32_t *len;
    const uint8_t *in;
    const uint64_t *wire_off;
    uint8_t *wire;
    uint8_t *back;
    uint32_t nthreads, tid;
    uint64_t ok;
} bench_arg;

static void *bench_worker(void *p)
{
    bench_arg *a = (bench_arg *) p;
    uint64_t maxlen = 0;
    for (uint64_t i = 0; i < a->n; ++i)
        if (a->len[i] > maxlen)
            maxlen = a->len[i];
    uint8_t *scratch = (uint8_t *) malloc(maxlen + 64);
    uint64_t ok = 0;
    for (uint64_t i = 0; i < a->n; ++i) {
        if (a->sid[i] % a->nthreads != a->tid)
            continue;
        const oracle_session *s = &a->sessions[a->sid[i]];
        uint8_t *w = a->wire + a->wire_off[i];
        curve_encode_one(a->box, w, scratch, s->precom, s->enc_prefix, a->nonce[i], a->flags[i],
                         s->downgrade_sub, a->in + a->in_off[i], a->len[i]);
        /* the peer decodes with the mirrored prefix (enc_prefix of the sender) */
        uint64_t peer = a->nonce[i] - 1;
        uint8_t fl;
        uint64_t wl = 32 + 1 + a->len[i];
        if (curve_decode_one(a->open, a->back + a->in_off[i], &fl, scratch, s->precom, s->enc_prefix,
                             &peer, w, wl) == 0)
            ++ok;
    }
    free(scratch);
    a->ok = ok;
    return NULL;
}

/* Returns seconds of wall clock for one encode+decode pass over the batch;
 * *ok_out = messages that round-tripped.  use_sodium: 0 portable, 1 dlopen
 * libsodium (fails with -1.0 if absent).  Plain (non-sub/cancel) flags only. */
EXPORT double oracle_bench_roundtrip(int use_sodium, uint32_t nthreads, const oracle_session *sessions, uint64_t n,
                                     const uint32_t *sid, const uint64_t *nonce, const uint8_t *flags,
                                     const uint64_t *in_off, const uint32_t *len, const uint8_t *in,
                                     const uint64_t *wire_off, uint8_t *wire, uint8_t *back, uint64_t *ok_out)
{
    box_fn box = box_portable, open = open_portable;
    if (use_sodium) {
        void *h = dlopen("libsodium.so.23", RTLD_NOW);
        if (!h)
            h = dlopen("libsodium.so.26", RTLD_NOW);
        if (!h)
            h = dlopen("/opt/conda/lib/libsodium.so.23", RTLD_NOW);
        if (!h)
            return -1.0;
        int (*init)(void) = (int (*)(void)) dlsym(h, "sodium_init");
        box = (box_fn) dlsym(h, "crypto_box_easy_afternm");
        open = (box_fn) dlsym(h, "crypto_box_open_easy_afternm");
        if (!init || !box || !open || init() < 0)
            return -1.0;
    }
    if (nthreads < 1)
        nthreads = 1;
    pthread_t *th = (pthread_t *) calloc(nthreads, sizeof(pthread_t));
    bench_arg *args = (bench_arg *) calloc(nthreads, sizeof(bench_arg));
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (uint32_t t = 0; t < nthreads; ++t) {
        bench_arg a = {box, open, sessions, n, sid, nonce, flags, in_off, len, in, wire_off, wire, back,
                       nthreads, t, 0};
        args[t] = a;
        pthread_create(&th[t], NULL, bench_worker, &args[t]);
    }
    uint64_t ok = 0;
    for (uint32_t t = 0; t < nthreads; ++t) {
        pthread_join(th[t], NULL);
        ok += args[t].ok;
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    free(th);
    free(args);
    *ok_out = ok;
    return (double) (t1.tv_sec - t0.tv_sec) + 1e-9 * (double) (t1.tv_nsec - t0.tv_nsec);
}
