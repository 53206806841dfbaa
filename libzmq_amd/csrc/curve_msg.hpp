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
// the session key comes from HBM, and one workgroup of four waves spreads
// the message over its lanes --
//   1. the whole input (payload / wire frame) is laid out in LDS at its
//      stream position (stream byte 32 + j = message byte j) from the kernel
//      arguments (or, above kMsgInlineMax, from memory in one round trip);
//   2. the quad of lanes 4b .. 4b+3 computes Salsa20 block b (stream bytes
//      64b .. 64b+63, salsa20_quad) and each lane XORs its four words;
//   3. Poly1305 over the ciphertext on wave 0: a Horner sum of c = ceil(N/64)
//      blocks per lane, each lane's sum times its power of r^c, which wave 3
//      computes meanwhile by a DPP prefix product over its lanes, and a DPP
//      row sum;
//   4. meanwhile waves 1 and 2 store encode's "\x07MESSAGE" || BE64(nonce) ||
//      ciphertext and wave 0 adds the tag; decode checks the header
//      (src/mechanism_base.cpp:14-25, src/curve_mechanism_base.cpp:80-97)
//      and the replay rule (:98-106, the peer nonce advances before the MAC
//      check) first, stores the payload while the tag is computed, and a
//      frame whose tag then fails gets zeros over it before the completion
//      word -- the batch kernels' order; the caller sees the payload
//      (verified) or zeros (failed), as after libsodium's verify-then-decrypt
//      (:226-228).
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
constexpr uint32_t kMsgThreads = 256; // four waves: one Salsa20 block per quad of lanes (salsa20_quad)

__device__ __forceinline__ void msg_load_lds(uint8_t *lds, const uint8_t *g, uint32_t n, uint32_t tid)
{
    constexpr uint32_t T = kMsgThreads;
    if (((uintptr_t) g & 15u) == 0 && n <= kMsgMaxStream) {
        const uint32_t ng = n >> 4, tail = n & 15u;
        u32x4 v[kMsgMaxStream / 16 / T];
#pragma unroll
        for (uint32_t j = 0; j < kMsgMaxStream / 16 / T; ++j)
            if (tid + T * j < ng)
                v[j] = *(const GCU4 *) (uintptr_t) (g + 16u * (tid + T * j));
        const uint8_t tb = tid < tail ? g[16u * ng + tid] : 0;
#pragma unroll
        for (uint32_t j = 0; j < kMsgMaxStream / 16 / T; ++j)
            if (tid + T * j < ng)
                *(msg_u32x4_u1 *) (lds + 16u * (tid + T * j)) = v[j];
        if (tid < tail)
            lds[16u * ng + tid] = tb;
        return;
    }
    const uint32_t head = (4u - ((uint32_t) (uintptr_t) g & 3u)) & 3u;
    const uint32_t h = head < n ? head : n;
    for (uint32_t k = tid; k < h; k += T)
        lds[k] = g[k];
    const uint32_t nw = (n - h) >> 2;
    const uint32_t *gw = (const uint32_t *) (uintptr_t) (g + h);
    for (uint32_t k = tid; k < nw; k += T) {
        const uint32_t v = gw[k];
        uint8_t *p = lds + h + 4 * k;
        p[0] = (uint8_t) v;
        p[1] = (uint8_t) (v >> 8);
        p[2] = (uint8_t) (v >> 16);
        p[3] = (uint8_t) (v >> 24);
    }
    for (uint32_t k = h + 4 * nw + tid; k < n; k += T)
        lds[k] = g[k];
}

template <uint32_t T = kMsgThreads>
__device__ __forceinline__ void msg_store_g(uint8_t *g, const uint8_t *lds, uint32_t n, uint32_t tid)
{
    const uint32_t head = (4u - ((uint32_t) (uintptr_t) g & 3u)) & 3u;
    const uint32_t h = head < n ? head : n;
    for (uint32_t k = tid; k < h; k += T)
        g[k] = lds[k];
    const uint32_t nw = (n - h) >> 2;
    uint32_t *gw = (uint32_t *) (uintptr_t) (g + h);
    for (uint32_t k = tid; k < nw; k += T) {
        const uint8_t *p = lds + h + 4 * k;
        gw[k] = (uint32_t) p[0] | ((uint32_t) p[1] << 8) | ((uint32_t) p[2] << 16) | ((uint32_t) p[3] << 24);
    }
    for (uint32_t k = h + 4 * nw + tid; k < n; k += T)
        g[k] = lds[k];
}

template <uint32_t T = kMsgThreads>
__device__ __forceinline__ void msg_zero_g(uint8_t *g, uint32_t n, uint32_t tid)
{
    for (uint32_t k = tid; k < n; k += T)
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

// x times the element DPP control CTRL brings from another lane; lanes
// outside ROWS, or whose source lane does not exist, multiply by one.  The
// steps of an inclusive prefix product over a wave: row_shr 1, 2, 4, 8
// within rows of 16, then row_bcast 15 and 31 across them (MUL_ROWS 0xa,
// 0xc) -- DPP moves instead of LDS permutes, so a level costs the multiply.
template <int CTRL, int ROWS>
__device__ __forceinline__ void fe_mul_dpp(fe &x)
{
    fe y;
#pragma unroll
    for (int i = 0; i < 5; ++i)
        y.l[i] = (uint32_t) __builtin_amdgcn_update_dpp(i == 0 ? 1 : 0, (int) x.l[i], CTRL, ROWS, 0xf, false);
    fe_mul(x, y);
}

// The sum of the wave's elements (limbs below 2^26 + 64, fe_mul's output):
// 32-bit row sums by DPP (16 of them stay below 2^31), the four rows added in
// 64 bits and folded back; every lane gets the total.
__device__ __forceinline__ fe fe_wave_sum(const fe &x)
{
    uint64_t w[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        int v = (int) x.l[i];
        v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true); // row_shr:1
        v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true); // row_shr:2
        v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true); // row_shr:4
        v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true); // row_shr:8
        w[i] = (uint64_t) (uint32_t) __builtin_amdgcn_readlane(v, 15) + (uint32_t) __builtin_amdgcn_readlane(v, 31) +
               (uint32_t) __builtin_amdgcn_readlane(v, 47) + (uint32_t) __builtin_amdgcn_readlane(v, 63);
    }
    return fe_from_wide(w);
}

// The launch's completion word: every lane's writes reach memory (system
// scope: the results sit in mapped host memory), then lane 0 sets it.  The
// host polls it instead of waiting for the stream (zmqg_*_msg).
#ifndef ZMQG_MSG_ABLATE
#define ZMQG_MSG_ABLATE 0 // (diagnostic builds only: 1 full system fence, 2 no fence, 4 no Salsa20,
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
    if (ZMQG_MSG_ABLATE & 1) { // (the round-4 default before: a full system fence, acquire side included)
        __threadfence_system();
        __syncthreads();
        if (threadIdx.x == 0)
            __hip_atomic_store(done, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        return;
    }
    // every thread's writes released at system scope (the host reads them
    // after seeing the word; nothing is read back here, so no acquire), then
    // the word
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    __syncthreads();
    if (threadIdx.x == 0)
        __hip_atomic_store(done, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// One Salsa20 block on a quad of lanes (round 4): lane q of the quad holds
// column q's quarter-round (a, b, c, d) = x[5q], x[5q+4], x[5q+8], x[5q+12]
// (indices mod 16), so a column round is one quarter-round per lane.  Row q's
// quarter-round (x[5q], x[5q+1], x[5q+2], x[5q+3], within row q) finds its b,
// c, d in lanes q+1, q+2, q+3 of the quad, as their d, c, b: three quad
// permutations (DPP quad_perm) before the row round and their inverses after.
// A block costs a lane 240 VALU operations instead of 960, so the keystream
// of a one-message launch takes a quarter of the time (the launch spends four
// waves instead of one).
template <int CTRL>
__device__ __forceinline__ uint32_t quad_perm(uint32_t v)
{
    return (uint32_t) __builtin_amdgcn_mov_dpp((int) v, CTRL, 0xf, 0xf, false);
}
constexpr int kQuadNext = 0x39, kQuadHalf = 0x4e, kQuadPrev = 0x93; // lane q reads q+1 / q+2 / q+3 (mod 4)

__device__ __forceinline__ void salsa20_quad(uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d)
{
    // (a rolled loop: one launch runs it once, from a cold instruction cache)
#pragma unroll 1
    for (int r = 0; r < 10; ++r) {
        ZMQG_QR(a, b, c, d); // column round
        uint32_t B = quad_perm<kQuadNext>(d), C = quad_perm<kQuadHalf>(c), D = quad_perm<kQuadPrev>(b);
        ZMQG_QR(a, B, C, D); // row round
        d = quad_perm<kQuadPrev>(B);
        c = quad_perm<kQuadHalf>(C);
        b = quad_perm<kQuadNext>(D);
    }
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
__device__ __forceinline__ void msg_inline_lds(uint8_t *lds, const MsgInline<CAP> &d, uint32_t n, uint32_t tid)
{
    const uint32_t nw = (n + 3) >> 2;
#pragma unroll
    for (uint32_t j = 0; j < (CAP / 4 + kMsgThreads - 1) / kMsgThreads; ++j) {
        const uint32_t i = tid + kMsgThreads * j;
        if (i < nw)
            *(msg_u32_u1 *) (lds + 4u * i) = d.w[i];
    }
}

template <bool DEC, uint32_t CAP>
__global__ __launch_bounds__(kMsgThreads) void k_msg(MsgArgs a, MsgInline<CAP> d)
{
    __shared__ uint32_t st_w[kMsgMaxStream / 4 + 16]; // the stream image: 32 bytes, then the message bytes
    __shared__ uint32_t pt_w[DEC ? kMsgMaxStream / 4 + 16 : 1]; // decode: the plaintext image
    __shared__ uint32_t sh_pk[4];     // Poly1305 r words (wave 0 -> wave 3)
    __shared__ uint32_t sh_pw[5 * 64]; // lane u's power of r^c, limb-major (wave 3 -> wave 0)
    uint8_t *const st = (uint8_t *) st_w;
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const bool sid_ok = a.sid < a.max_sessions;
    const DevSession &ses = a.sessions[sid_ok ? a.sid : 0u];
    uint32_t key[8];
#pragma unroll
    for (int t = 0; t < 8; ++t)
        key[t] = DEC ? ses.dec_key[t] : ses.enc_key[t];
    // decode: the peer nonce is read now, beside the key's round trip
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
        if (tid < 8)
            st_w[tid] = 0;
        if (tid < hl)
            st[32 + tid] = (uint8_t) (hw[tid >> 2] >> (8 * (tid & 3)));
        if (CAP)
            msg_inline_lds(st + 32 + hl, d, a.len, tid);
        else if (!(ZMQG_MSG_ABLATE & 32))
            msg_load_lds(st + 32 + hl, a.in, a.len, tid);
        nc = a.nonce;
        n0 = bswap32((uint32_t) (nc >> 32));
        n1 = bswap32((uint32_t) nc);
        if (!sid_ok)
            status = ZMQG_ERR_SESSION;
    } else {
        const uint32_t L = a.len;
        if (CAP)
            msg_inline_lds(st, d, L, tid);
        else if (!(ZMQG_MSG_ABLATE & 32))
            msg_load_lds(st, a.in, L, tid);
        m = L >= 33u ? L - 32u : 0u;
    }
    // zero the bytes after the message up to the next 16-byte block (Poly1305
    // pads a partial last block with zeros; below a 33-byte frame, bytes 32..
    // -- past the message either way)
    const uint32_t end = 32 + m;
    if (tid < 16 && end + tid < kMsgMaxStream + 64)
        st[end + tid] = 0;
    __syncthreads();
    if (DEC) {
        const uint32_t L = a.len;
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
    if (DEC && status == 0 && tid == 0)
        a.peer[a.sid] = nc;

    // ---- 2. keystream block blk on its quad of lanes, XOR of its window's
    // four words of the quad's lane
    const uint32_t nb = (end + 63) >> 6, blk = tid >> 2, q = tid & 3u;
    // (a, b, c, d) = x[5q], x[5q+4], x[5q+8], x[5q+12] of block blk
    const uint32_t sig = q == 0 ? SIGMA0 : q == 1 ? SIGMA1 : q == 2 ? SIGMA2 : SIGMA3;
    const uint32_t ib = q == 0 ? key[3] : q == 1 ? 0u : q == 2 ? key[7] : key[2];
    const uint32_t ic = q == 0 ? blk : q == 1 ? key[6] : q == 2 ? key[1] : n1;
    const uint32_t id = q == 0 ? key[5] : q == 1 ? key[0] : q == 2 ? n0 : key[4];
    uint32_t ka = sig, kb = ib, kc = ic, kd = id;
    if (ZMQG_MSG_ABLATE & 4) {
        ka ^= blk * 0x9e3779b9u;
        kc ^= kb;
    } else {
        salsa20_quad(ka, kb, kc, kd);
    }
    ka += sig;
    kb += ib;
    kc += ic;
    kd += id;
    // the Poly1305 key: keystream words 0..7 of block 0 (lanes 0-3: words 0
    // 4 8 12 / 5 9 13 1 / 10 14 2 6 / 15 3 7 11; meaningful in wave 0 only)
    uint32_t pk[8];
    pk[0] = __builtin_amdgcn_readlane(ka, 0);
    pk[1] = __builtin_amdgcn_readlane(kd, 1);
    pk[2] = __builtin_amdgcn_readlane(kc, 2);
    pk[3] = __builtin_amdgcn_readlane(kb, 3);
    pk[4] = __builtin_amdgcn_readlane(kb, 0);
    pk[5] = __builtin_amdgcn_readlane(ka, 1);
    pk[6] = __builtin_amdgcn_readlane(kd, 2);
    pk[7] = __builtin_amdgcn_readlane(kc, 3);
    const uint32_t ia = (5u * q) & 15u; // word index of register a; b, c, d follow at +4, +8, +12 (mod 16)
    uint32_t o[4];                      // this lane's output words (ciphertext or plaintext) of block blk
    {
        const uint32_t ks[4] = {ka, kb, kc, kd};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t wi = (ia + 4u * k) & 15u;
            const int nv = (int) end - (int) (64u * blk + 4u * wi); // valid bytes of this word
            const uint32_t mk = nv >= 4 ? 0xffffffffu : (nv <= 0 ? 0u : ((1u << (8 * nv)) - 1u));
            const uint32_t x = blk < nb ? st_w[16u * blk + wi] : 0u;
            o[k] = (blk == 0 && wi < 8) ? 0u : ((x ^ ks[k]) & mk);
        }
    }
    if (tid == 0) {
#pragma unroll
        for (int k = 0; k < 4; ++k)
            sh_pk[k] = pk[k];
    }
    if (!DEC) { // the ciphertext image replaces the plaintext
        __syncthreads();
        if (blk < nb)
#pragma unroll
            for (int k = 0; k < 4; ++k)
                st_w[16u * blk + ((ia + 4u * k) & 15u)] = o[k];
        __syncthreads();
    } else { // the plaintext image beside the ciphertext (flags byte at stream byte 32, payload after it)
        if (status == 0 && blk < nb)
#pragma unroll
            for (int k = 0; k < 4; ++k)
                pt_w[16u * blk + ((ia + 4u * k) & 15u)] = o[k];
        __syncthreads();
    }

    // ---- 3. Poly1305 over the ciphertext (stream bytes 32 .. 32+m): c =
    // ceil(N/64) blocks per lane (a Horner sum) over nl = ceil(N/c) groups of
    // c blocks, group g on lane nl-1-g of wave 0 (the message's last group on
    // lane 0), the first group padded by zero blocks in front (zero blocks
    // ahead of a Horner sum change nothing); lane u's sum is worth x^u, x =
    // r^c, which wave 3 computes meanwhile as an inclusive prefix product over
    // its lanes (one on lane 0, x elsewhere; log2(nl) DPP levels of one
    // multiply each) and hands over in LDS; wave 0 then sums its lanes' terms
    // (tests/test_poly_tree_model.py models it).  Waves 1 and 2 store
    // everything but the tag meanwhile, so the stores' round trips to the
    // mapped destination overlap the MAC instead of following it.
    const uint32_t N = (m + 15) >> 4, c = N ? (N + 63) >> 6 : 1u, nl = (N + c - 1) / c, pad = c * nl - N;
    uint32_t levels = 0;
    while ((1u << levels) < nl)
        ++levels;
    const bool scan = levels && !(ZMQG_MSG_ABLATE & 8);
    const uint32_t wv = tid >> 6;
    const uint32_t P = DEC && a.len >= 33u ? a.len - 33u : 0u;
    fe h = fe_zero();
    if (wv == 0) {
        const fe r = poly_r_from_key(pk[0], pk[1], pk[2], pk[3]);
        if (lane < nl) {
            const uint32_t g = nl - 1u - lane;
            const uint32_t s1 = r.l[1] * 5, s2 = r.l[2] * 5, s3 = r.l[3] * 5, s4 = r.l[4] * 5;
#pragma unroll
            for (uint32_t t = 0; t < 4; ++t) {
                const int k = (int) (c * g + t) - (int) pad;
                if (t < c && k >= 0) {
                    const uint32_t *bp = st_w + 8 + 4 * k;
                    uint32_t b0 = bp[0], b1 = bp[1], b2 = bp[2], b3 = bp[3], hib = 1u << 24;
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
    } else if (wv == 3) {
        if (scan) {
            const fe r = poly_r_from_key(sh_pk[0], sh_pk[1], sh_pk[2], sh_pk[3]);
            // x = r^c (c uniform, 1..4)
            fe x = r;
            if (c > 1) {
                fe r2 = r;
                fe_mul(r2, r);
                x = r2;
                if (c == 3)
                    fe_mul(x, r);
                else if (c == 4)
                    fe_mul(x, r2);
            }
            fe pw = x;
            if (lane == 0) {
                pw = fe_zero();
                pw.l[0] = 1;
            }
            fe_mul_dpp<0x111, 0xf>(pw); // row_shr:1
            if (levels > 1)
                fe_mul_dpp<0x112, 0xf>(pw); // row_shr:2
            if (levels > 2)
                fe_mul_dpp<0x114, 0xf>(pw); // row_shr:4
            if (levels > 3)
                fe_mul_dpp<0x118, 0xf>(pw); // row_shr:8
            if (levels > 4)
                fe_mul_dpp<0x142, 0xa>(pw); // row_bcast:15
            if (levels > 5)
                fe_mul_dpp<0x143, 0xc>(pw); // row_bcast:31
#pragma unroll
            for (int i = 0; i < 5; ++i)
                sh_pw[64 * i + lane] = pw.l[i];
        }
    } else if (status == 0 && !(ZMQG_MSG_ABLATE & 16)) { // waves 1 and 2
        const uint32_t j = tid - 64;
        if (!DEC) {
            // "\x07MESSAGE" || nonce, then the ciphertext
            msg_store_g<128>(a.out + 32, st + 32, m, j);
            if (j < 16) {
                const uint32_t w = j < 4 ? 0x53454d07u : j < 8 ? 0x45474153u : j < 12 ? n0 : n1;
                a.out[j] = (uint8_t) (w >> (8 * (j & 3u)));
            }
        } else {
            // header, session and replay checks passed: the payload goes out
            // now, and is zeroed below if the tag fails
            msg_store_g<128>(a.out, (const uint8_t *) pt_w + 33, P, j);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); // landed before any zeroing below
        }
    }
    __syncthreads();
    uint32_t tag[4] = {0, 0, 0, 0};
    if (wv == 0) {
        if (scan) {
            fe pw;
#pragma unroll
            for (int i = 0; i < 5; ++i)
                pw.l[i] = sh_pw[64 * i + lane];
            fe_mul(h, pw);
            h = fe_wave_sum(h);
        }
        poly_finish(h, pk + 4, tag);
        // (the same on every lane; lane 0's where there was one lane)
#pragma unroll
        for (int k = 0; k < 4; ++k)
            tag[k] = __builtin_amdgcn_readlane(tag[k], 0);
    }

    // ---- 4. results
    if (!DEC) {
        if (status == 0 && !(ZMQG_MSG_ABLATE & 16) && tid < 16) {
            const uint32_t w = tid < 4 ? tag[0] : tid < 8 ? tag[1] : tid < 12 ? tag[2] : tag[3];
            a.out[16 + tid] = (uint8_t) (w >> (8 * (tid & 3u)));
        }
        if (tid == 0 && a.status)
            *a.status = status;
        msg_done(a.done);
        return;
    }
    // wave 0 decides: the tag check, and zeros over a forged frame's payload
    // (waves 1 and 2 drained their speculative stores before the barrier
    // above, so these land after them)
    if (wv == 0) {
        if (status == 0 && ((tag[0] ^ st_w[4]) | (tag[1] ^ st_w[5]) | (tag[2] ^ st_w[6]) | (tag[3] ^ st_w[7])))
            status = ZMQG_ERR_CRYPTOGRAPHIC; // src/curve_mechanism_base.cpp:277-281
        if (status != 0 && !(ZMQG_MSG_ABLATE & 16))
            msg_zero_g<64>(a.out, P, lane);
        if (tid == 0) {
            // msg_t::more | msg_t::command (curve_mechanism_base.cpp:276)
            *a.flags_out = status == 0 ? ((const uint8_t *) pt_w)[32] & 3u : 0u;
            *a.status = status;
        }
    }
    msg_done(a.done);
}

} // namespace zmqg
