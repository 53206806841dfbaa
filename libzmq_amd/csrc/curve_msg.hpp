// curve_msg.hpp -- one CURVE MESSAGE per launch (zmqg_encode_msg /
// zmqg_decode_msg): the drop-in codec's per-message path, i.e. what
// src/stream_engine_base.cpp:613 / :622 call for every message.
//
// The batch kernels are built for many frames: descriptors are read from
// memory (over PCIe when they sit in mapped host memory, each a dependent
// round trip before the keystream can start), a lane walks its frame's
// windows one after the other, and a workgroup takes part in the call-state
// and look-back protocol.  For one message of at most kMsgMaxStream stream
// bytes none of that is needed: the descriptors travel as kernel arguments,
// the session key comes from HBM, and one wave spreads the message over its
// lanes --
//   1. the whole input (payload / wire frame) is loaded into LDS at its
//      stream position (stream byte 32 + j = message byte j) by all lanes at
//      once, so the only PCIe latency before the keystream is one round trip;
//   2. lane b computes Salsa20 block b (stream bytes 64b .. 64b+63) and XORs
//      its window;
//   3. Poly1305 over the ciphertext in parallel: with N 16-byte blocks and
//      nl = ceil(N/4) lanes holding 4 blocks each, the lanes are placed at the
//      END of the wave (zero segments in front of a Horner sum change
//      nothing), each lane's Horner value is worth r^(4*(63-lane)), and six
//      shuffle levels combine h_v*r^(4*2^s) + h_(v+2^s);
//   4. encode writes "\x07MESSAGE" || BE64(nonce) || tag || ciphertext;
//      decode checks the header (src/mechanism_base.cpp:14-25,
//      src/curve_mechanism_base.cpp:80-97), the replay rule (:98-106, the
//      peer nonce advances before the MAC check) and the tag, and only then
//      writes the payload (verified) or zeros (failed) -- libsodium's
//      verify-then-decrypt order (:226-228).
// Same bytes, statuses and session-state updates as the batch path with
// n = 1 (tests/test_gpu_msg.py checks both against the oracle).
#pragma once

#include "curve_device.hpp"

namespace zmqg {

constexpr uint32_t kMsgMaxStream = 4096; // 64 lanes x one Salsa20 block

struct MsgArgs {
    const uint8_t *in;             // encode: payload (len bytes); decode: wire frame (len bytes)
    uint8_t *out;                  // encode: wire frame; decode: payload (len - 33 bytes)
    const DevSession *sessions;
    unsigned long long *peer;      // decode: _cn_peer_nonce per session
    uint8_t *flags_out;            // decode
    int32_t *status;               // decode: 0 / ZMQG_ERR_*; encode: 0 / ZMQG_ERR_SESSION
    uint32_t *done;                // set to 1 (system scope) after every other write of the launch
    uint64_t nonce;                // encode
    uint32_t sid, len, max_sessions, flags;
};

// Copies between global memory and LDS.  The message sits in mapped host
// memory, so a load is a PCIe round trip: a 16-byte-aligned message (the
// per-message buffer always is) is read with all of a lane's loads in
// flight at once -- up to four dwordx4 per lane, 4 KiB per wave -- before any
// of them is used; other alignments take the general byte/word form.
typedef u32x4 msg_u32x4_u1 __attribute__((aligned(1)));
__device__ __forceinline__ void msg_load_lds(uint8_t *lds, const uint8_t *g, uint32_t n, uint32_t lane)
{
    if (((uintptr_t) g & 15u) == 0 && n <= kMsgMaxStream) {
        const uint32_t ng = n >> 4, tail = n & 15u;
        u32x4 v[kMsgMaxStream / 16 / 64];
#pragma unroll
        for (uint32_t j = 0; j < kMsgMaxStream / 16 / 64; ++j)
            if (lane + 64u * j < ng)
                v[j] = *(const GCU4 *) (uintptr_t) (g + 16u * (lane + 64u * j));
        const uint8_t tb = lane < tail ? g[16u * ng + lane] : 0;
#pragma unroll
        for (uint32_t j = 0; j < kMsgMaxStream / 16 / 64; ++j)
            if (lane + 64u * j < ng)
                *(msg_u32x4_u1 *) (lds + 16u * (lane + 64u * j)) = v[j];
        if (lane < tail)
            lds[16u * ng + lane] = tb;
        return;
    }
    const uint32_t head = (4u - ((uint32_t) (uintptr_t) g & 3u)) & 3u;
    const uint32_t h = head < n ? head : n;
    for (uint32_t k = lane; k < h; k += 64)
        lds[k] = g[k];
    const uint32_t nw = (n - h) >> 2;
    const uint32_t *gw = (const uint32_t *) (uintptr_t) (g + h);
    for (uint32_t k = lane; k < nw; k += 64) {
        const uint32_t v = gw[k];
        uint8_t *p = lds + h + 4 * k;
        p[0] = (uint8_t) v;
        p[1] = (uint8_t) (v >> 8);
        p[2] = (uint8_t) (v >> 16);
        p[3] = (uint8_t) (v >> 24);
    }
    for (uint32_t k = h + 4 * nw + lane; k < n; k += 64)
        lds[k] = g[k];
}

__device__ __forceinline__ void msg_store_g(uint8_t *g, const uint8_t *lds, uint32_t n, uint32_t lane)
{
    const uint32_t head = (4u - ((uint32_t) (uintptr_t) g & 3u)) & 3u;
    const uint32_t h = head < n ? head : n;
    for (uint32_t k = lane; k < h; k += 64)
        g[k] = lds[k];
    const uint32_t nw = (n - h) >> 2;
    uint32_t *gw = (uint32_t *) (uintptr_t) (g + h);
    for (uint32_t k = lane; k < nw; k += 64) {
        const uint8_t *p = lds + h + 4 * k;
        gw[k] = (uint32_t) p[0] | ((uint32_t) p[1] << 8) | ((uint32_t) p[2] << 16) | ((uint32_t) p[3] << 24);
    }
    for (uint32_t k = h + 4 * nw + lane; k < n; k += 64)
        g[k] = lds[k];
}

__device__ __forceinline__ void msg_zero_g(uint8_t *g, uint32_t n, uint32_t lane)
{
    for (uint32_t k = lane; k < n; k += 64)
        g[k] = 0;
}

// Carry a sum of two partially reduced elements (limbs below 2^28) back to
// limbs below 2^26 (limb 1 below 2^26 + 1): fe_mul's inputs must stay below
// 2^27, or its last fold (c * 5 in 32 bits) wraps.
__device__ __forceinline__ void fe_carry(fe &h)
{
    uint32_t c;
    c = h.l[0] >> 26;
    h.l[0] &= M26;
    h.l[1] += c;
    c = h.l[1] >> 26;
    h.l[1] &= M26;
    h.l[2] += c;
    c = h.l[2] >> 26;
    h.l[2] &= M26;
    h.l[3] += c;
    c = h.l[3] >> 26;
    h.l[3] &= M26;
    h.l[4] += c;
    c = h.l[4] >> 26;
    h.l[4] &= M26;
    h.l[0] += c * 5;
    c = h.l[0] >> 26;
    h.l[0] &= M26;
    h.l[1] += c;
}

__device__ __forceinline__ fe fe_shfl_down(const fe &x, uint32_t d)
{
    fe y;
#pragma unroll
    for (int i = 0; i < 5; ++i)
        y.l[i] = (uint32_t) __shfl_down((int) x.l[i], d, 64);
    return y;
}

// The launch's completion word: every lane's writes reach memory (system
// scope: the results sit in mapped host memory), then lane 0 sets it.  The
// host polls it instead of waiting for the stream (zmqg_*_msg).
#ifndef ZMQG_MSG_ABLATE
#define ZMQG_MSG_ABLATE 0 // (diagnostic builds only: 1 release-only fence, 2 no fence, 4 no Salsa20,
                          // 8 no Poly1305 tree, 16 no output stores, 32 no input loads)
#endif
__device__ __forceinline__ void msg_done(uint32_t *done)
{
    if (ZMQG_MSG_ABLATE & 2) {
        __syncthreads();
        if (threadIdx.x == 0)
            __hip_atomic_store(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return;
    }
    if (ZMQG_MSG_ABLATE & 1) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        __syncthreads();
        if (threadIdx.x == 0)
            __hip_atomic_store(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return;
    }
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0)
        __hip_atomic_store(done, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// salsa20_block with the double rounds in a loop: a single launch executes
// it once per lane, so a tenth of the code (fewer instruction-cache misses
// on a cold CU) costs only the loop's scalar branch.
__device__ __forceinline__ void salsa20_block_rolled(uint32_t out[16], const uint32_t k[8], uint32_t n0, uint32_t n1,
                                                     uint32_t ctr)
{
    uint32_t x[16] = {SIGMA0, k[0], k[1], k[2], k[3], SIGMA1, n0, n1, ctr, 0, SIGMA2, k[4], k[5], k[6], k[7], SIGMA3};
#pragma unroll 1
    for (int rr = 0; rr < 10; ++rr) {
        ZMQG_QR(x[0], x[4], x[8], x[12]);
        ZMQG_QR(x[5], x[9], x[13], x[1]);
        ZMQG_QR(x[10], x[14], x[2], x[6]);
        ZMQG_QR(x[15], x[3], x[7], x[11]);
        ZMQG_QR(x[0], x[1], x[2], x[3]);
        ZMQG_QR(x[5], x[6], x[7], x[4]);
        ZMQG_QR(x[10], x[11], x[8], x[9]);
        ZMQG_QR(x[15], x[12], x[13], x[14]);
    }
    const uint32_t in[16] = {SIGMA0, k[0], k[1], k[2], k[3], SIGMA1, n0, n1, ctr, 0, SIGMA2, k[4], k[5], k[6], k[7], SIGMA3};
#pragma unroll
    for (int i = 0; i < 16; ++i)
        out[i] = x[i] + in[i];
}

// The message itself as a kernel argument (CAP bytes, zero-padded to a
// whole word): kernel arguments reach the GPU with the dispatch, so the
// kernel reads them at HBM latency instead of pulling the message over PCIe
// from mapped host memory (a 4,000-byte message cost ~5 us of PCIe reads).
template <uint32_t CAP>
struct MsgInline {
    uint32_t w[CAP ? CAP / 4 : 1];
};
constexpr uint32_t kMsgInlineMax = 3968; // kernel arguments are limited to 4 KiB in all

// LDS <- the inline message (n bytes) at byte offset lds (any alignment)
typedef uint32_t msg_u32_u1 __attribute__((aligned(1)));
template <uint32_t CAP>
__device__ __forceinline__ void msg_inline_lds(uint8_t *lds, const MsgInline<CAP> &d, uint32_t n, uint32_t lane)
{
    const uint32_t nw = (n + 3) >> 2;
#pragma unroll
    for (uint32_t j = 0; j < (CAP / 4 + 63) / 64; ++j) {
        const uint32_t i = lane + 64u * j;
        if (i < nw)
            *(msg_u32_u1 *) (lds + 4u * i) = d.w[i];
    }
}

template <bool DEC, uint32_t CAP>
__global__ __launch_bounds__(64) void k_msg(MsgArgs a, MsgInline<CAP> d)
{
    __shared__ uint32_t st_w[kMsgMaxStream / 4 + 16]; // the stream image: 32 bytes, then the message bytes
    uint8_t *const st = (uint8_t *) st_w;
    const uint32_t lane = threadIdx.x;
    const bool sid_ok = a.sid < a.max_sessions;
    const DevSession &ses = a.sessions[sid_ok ? a.sid : 0u];
    uint32_t key[8];
#pragma unroll
    for (int t = 0; t < 8; ++t)
        key[t] = DEC ? ses.dec_key[t] : ses.enc_key[t];
    // decode: the peer nonce is read now, beside the message's PCIe round
    // trip, not after it
    const unsigned long long peer = DEC && sid_ok ? a.peer[a.sid] : 0ull;

    // ---- 1. the message into LDS at its stream position; header checks
    uint32_t m = 0; // ciphertext bytes
    int32_t status = 0;
    uint32_t n0 = 0, n1 = 0;
    uint64_t nc = 0;
    if (!DEC) {
        uint32_t hw[3];
        const uint32_t hl = plaintext_header(a.flags, ses.downgrade_sub, hw);
        m = hl + a.len;
        if (lane < 8)
            st_w[lane] = 0;
        if (lane < hl)
            st[32 + lane] = (uint8_t) (hw[lane >> 2] >> (8 * (lane & 3)));
        if (CAP)
            msg_inline_lds(st + 32 + hl, d, a.len, lane);
        else if (!(ZMQG_MSG_ABLATE & 32))
            msg_load_lds(st + 32 + hl, a.in, a.len, lane);
        nc = a.nonce;
        n0 = bswap32((uint32_t) (nc >> 32));
        n1 = bswap32((uint32_t) nc);
        if (!sid_ok)
            status = ZMQG_ERR_SESSION;
    } else {
        const uint32_t L = a.len;
        if (CAP)
            msg_inline_lds(st, d, L, lane);
        else if (!(ZMQG_MSG_ABLATE & 32))
            msg_load_lds(st, a.in, L, lane);
        __syncthreads();
        // mechanism_base.cpp:14-25, curve_mechanism_base.cpp:80-97
        const uint32_t b0 = L ? st[0] : 0u;
        const uint32_t w0 = L >= 8 ? st_w[0] : 0u, w1 = L >= 8 ? st_w[1] : 0u;
        if (L <= 1u || L <= b0)
            status = ZMQG_ERR_MALFORMED_UNSPECIFIED;
        else if (L < 8u || w0 != 0x53454d07u || w1 != 0x45474153u)
            status = ZMQG_ERR_UNEXPECTED_COMMAND;
        else if (L < 33u)
            status = ZMQG_ERR_MALFORMED_MESSAGE;
        if (!sid_ok)
            status = ZMQG_ERR_SESSION;
        m = L >= 33u ? L - 32u : 0u;
        if (status == 0) {
            n0 = st_w[2];
            n1 = st_w[3];
            nc = ((uint64_t) bswap32(n0) << 32) | bswap32(n1);
            // curve_mechanism_base.cpp:98-106: a nonce not above the peer's
            // is a replay; a valid one becomes the peer nonce before the MAC
            if (nc <= peer)
                status = ZMQG_ERR_INVALID_SEQUENCE;
        }
    }
    // zero the bytes after the message up to the next 16-byte block (Poly1305
    // pads a partial last block with zeros)
    const uint32_t end = 32 + m;
    if (lane < 16 && end + lane < kMsgMaxStream + 64)
        st[end + lane] = 0;
    __syncthreads();
    if (DEC && status == 0 && lane == 0)
        a.peer[a.sid] = nc;

    // ---- 2. keystream block `lane`, XOR of its window
    const uint32_t nb = (end + 63) >> 6;
    uint32_t ks[16];
    if (ZMQG_MSG_ABLATE & 4) {
#pragma unroll
        for (int k = 0; k < 16; ++k)
            ks[k] = key[k & 7] ^ (lane * 0x9e3779b9u + k);
    } else {
        salsa20_block_rolled(ks, key, n0, n1, lane);
    }
    uint32_t w[16];
#pragma unroll
    for (int k = 0; k < 16; ++k)
        w[k] = st_w[16 * lane + k];
    // the Poly1305 key: keystream bytes 0..31 of block 0
    uint32_t pk[8];
#pragma unroll
    for (int k = 0; k < 8; ++k)
        pk[k] = __builtin_amdgcn_readfirstlane(ks[k]);
    uint32_t o[16];
#pragma unroll
    for (int k = 0; k < 16; ++k)
        o[k] = (lane == 0 && k < 8) ? 0u : w[k] ^ ks[k];
    // bytes past the message stay zero in the image (the Poly1305 padding)
    if (lane < nb) {
        const int nv = (int) end - 64 * (int) lane;
        if (nv < 64)
            mask_tail(o, nv);
    }
    if (!DEC) { // the ciphertext image replaces the plaintext
        __syncthreads();
        if (lane < nb)
#pragma unroll
            for (int k = 0; k < 16; ++k)
                st_w[16 * lane + k] = o[k];
        __syncthreads();
    }

    // ---- 3. Poly1305 over the ciphertext (stream bytes 32 .. 32+m)
    const fe r = poly_r_from_key(pk[0], pk[1], pk[2], pk[3]);
    // nl lanes of four blocks each, right-aligned in the smallest power-of-
    // two span S that holds them (a short message needs few or no levels)
    const uint32_t N = (m + 15) >> 4, nl = (N + 3) >> 2, pad = 4 * nl - N;
    uint32_t levels = 0;
    while ((1u << levels) < nl)
        ++levels;
    const uint32_t S = 1u << levels;
    fe h = fe_zero();
    const int seg = (int) lane - (int) (S - nl);
    if (seg >= 0 && lane < S) {
        const uint32_t s1 = r.l[1] * 5, s2 = r.l[2] * 5, s3 = r.l[3] * 5, s4 = r.l[4] * 5;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int k = 4 * seg + t - (int) pad;
            if (k >= 0) {
                const uint32_t *b = st_w + 8 + 4 * k;
                uint32_t b0 = b[0], b1 = b[1], b2 = b[2], b3 = b[3], hib = 1u << 24;
                const uint32_t rem = m - 16u * (uint32_t) k;
                if (rem < 16u) { // partial last block: 0x01 after the data, no 2^128
                    const uint32_t sh = 8u * (rem & 3u), wi = rem >> 2, one = 1u << sh;
                    b0 |= wi == 0 ? one : 0u;
                    b1 |= wi == 1 ? one : 0u;
                    b2 |= wi == 2 ? one : 0u;
                    b3 |= wi == 3 ? one : 0u;
                    hib = 0;
                }
                fe_add_block(h, b0, b1, b2, b3, hib);
                fe_mul_s(h, r, s1, s2, s3, s4);
            }
        }
    }
    if (levels && !(ZMQG_MSG_ABLATE & 8)) {
        fe p = r;
        fe_mul(p, r);
        fe_mul(p, p); // r^4
        // (a rolled loop: one launch runs this once, from a cold instruction cache)
#pragma unroll 1
        for (uint32_t s = 0; s < levels; ++s) {
            const fe hn = fe_shfl_down(h, 1u << s);
            if ((lane & ((2u << s) - 1u)) == 0) {
                fe_mul(h, p);
                fe_add(h, hn);
                fe_carry(h); // (the next level multiplies it again)
            }
            if (s + 1 < levels)
                fe_mul(p, p);
        }
    }
    uint32_t tag[4];
    poly_finish(h, pk + 4, tag);

    // ---- 4. results
    if (!DEC) {
        if (lane == 0) {
            st_w[0] = 0x53454d07u; // "\x07MES"
            st_w[1] = 0x45474153u; // "SAGE"
            st_w[2] = n0;
            st_w[3] = n1;
#pragma unroll
            for (int k = 0; k < 4; ++k)
                st_w[4 + k] = tag[k];
        }
        __syncthreads();
        if (status == 0)
            if (!(ZMQG_MSG_ABLATE & 16))
                msg_store_g(a.out, st, end, lane);
        if (lane == 0 && a.status)
            *a.status = status;
        msg_done(a.done);
        return;
    }
    if (status == 0) {
        const uint32_t t0 = __builtin_amdgcn_readfirstlane(tag[0]), t1 = __builtin_amdgcn_readfirstlane(tag[1]),
                       t2 = __builtin_amdgcn_readfirstlane(tag[2]), t3 = __builtin_amdgcn_readfirstlane(tag[3]);
        if ((t0 ^ st_w[4]) | (t1 ^ st_w[5]) | (t2 ^ st_w[6]) | (t3 ^ st_w[7]))
            status = ZMQG_ERR_CRYPTOGRAPHIC;
    }
    const uint32_t P = a.len >= 33u ? a.len - 33u : 0u;
    if (status == 0) {
        // the plaintext image: flags byte at stream byte 32, payload after it
        __syncthreads();
        if (lane < nb)
#pragma unroll
            for (int k = 0; k < 16; ++k)
                st_w[16 * lane + k] = o[k];
        __syncthreads();
        if (!(ZMQG_MSG_ABLATE & 16))
            msg_store_g(a.out, st + 33, P, lane);
        if (lane == 0)
            *a.flags_out = st[32] & 3u; // msg_t::more | msg_t::command (curve_mechanism_base.cpp:276)
    } else {
        if (!(ZMQG_MSG_ABLATE & 16))
            msg_zero_g(a.out, P, lane);
        if (lane == 0)
            *a.flags_out = 0;
    }
    if (lane == 0)
        *a.status = status;
    msg_done(a.done);
}

} // namespace zmqg
