// curve_frames_st.hpp -- the one-lane-per-frame kernel with its global
// traffic moved in coalesced 128-byte runs through LDS by a second wave on
// each SIMD (k_frames_st).
//
// Same frame semantics as k_frames_seq / k_frames_lds (curve_frames.hpp,
// curve_frames_lds.hpp): one lane owns one frame and walks its 64-byte
// keystream windows in order with the sequential radix-2^32 Poly1305; the
// decode header checks and replay rule of src/curve_mechanism_base.cpp:80-284
// and src/mechanism_base.cpp:14-25; encode per :111-205.
//
// Why.  In k_frames_seq every lane loads and stores its own frame, so each
// dwordx4 instruction touches 64 different 64-byte pieces; the address unit
// takes ~700 (load) and ~970 (store) cycles per such instruction
// (profiles/valu_rates_r02.md, vmem_issue): memory alone ran as long as the
// whole kernel.  Moving the bytes in 128-byte runs
// (8 or 9 lanes per piece) makes that cheap, but a single wave per SIMD that
// also issues the moves and waits for them exposes every wait: a first
// version of this kernel with one wave per SIMD doing both took 65 us at
// config 2 against seq's 59 (memory and LDS work alone 42 us, compute alone
// 51, ablations in DESIGN.md section 3.1).  So each SIMD holds two waves of
// one 512-thread workgroup (waves w and w + 4 share a SIMD): a compute wave
// (keystream, Poly1305, XOR; LDS reads and writes only) and its memory wave
// (LDS-DMA loads, ring-to-global stores, the frames' edge bytes), meeting at
// one workgroup barrier per super-step.  While one waits the other issues.
//
// Super-steps.  Super-step K covers stream bytes [128K, 128K + 128), i.e.
// windows 2K and 2K + 1 (window 0, with the header, nonce and tag, is read
// by its lane directly).  Between barriers B_K and B_K+1:
//   * compute wave: windows 2K, 2K+1 from input buffer K & 1 (the frame's
//     16-byte-aligned cover of the super-step: 9 granules = 144 bytes at
//     phase va; 17 aligned ds_read_b32 per window, shifted in registers);
//     each window's 64 output bytes go, shifted to the destination's 4-byte
//     phase, as aligned dwords into the frame's ring half K & 1; bytes past
//     the half's end (the first bytes of super-step K+1's first granule) go
//     to overflow slot K & 3.
//   * memory wave: LDS-DMA of super-step K+1's covers into buffer (K+1) & 1
//     (9 instructions, consecutive lanes on consecutive granules of a frame);
//     super-step K-1's output granules from ring half (K-1) & 1 (granule 0
//     completed from overflow slot (K-2) & 3) to memory as 8 dwordx4
//     instructions of 8 lanes per 128-byte piece, whole granules only; after
//     super-step 0 also each frame's partial first granule (head); then it
//     waits for the DMA, so the compute wave finds the covers at B_K+1.
// After the last super-step the memory wave stores the last granules and each
// frame's partial last granule (tail), drains its stores and leaves; the
// compute waves finish the MACs and the replay look-back (256 threads).
// Only naturally aligned DS accesses (gfx950 replays misaligned b128 at ~64
// cycles, cdna_hip_programming.md Guideline 17).
// LDS per pair: 2 x 9,216 (input) + 64 x 336 (ring 256 + overflow 4 x 16 +
// pad) = 39,936 bytes; four pairs per workgroup, one workgroup per CU.
#pragma once

#include "curve_frames_lds.hpp"

#ifndef ZMQG_ST_ABLATE
#define ZMQG_ST_ABLATE 0 // timing experiments only (outputs wrong): 1 no ring->global stores, 2 no DMA, 4 no ring
                         // writes, 8 no window reads from LDS, 16 no Salsa20, 32 no Poly1305
#endif

#ifndef ZMQG_ST_REGSTAGE
#define ZMQG_ST_REGSTAGE 0 // 1: covers move by global_load_dwordx4 into the memory wave's registers and
                           // ds_write_b128, instead of LDS-DMA
#endif

#ifndef ZMQG_ST_STORE
#define ZMQG_ST_STORE 0 // cache policy of the ring-to-global stores: 0 default, 1 nt, 2 sc1 (write-through),
                        // 3 sc0 sc1
#endif

#ifndef ZMQG_ST_MEMPRIO
#define ZMQG_ST_MEMPRIO 2 // s_setprio of the memory waves (0: same as the compute waves)
#endif

#ifndef ZMQG_ST_STAMPS
#define ZMQG_ST_STAMPS 0 // diagnostic builds only (tools/st_stamps.hip): per-wave s_memtime stamps into rp.clk
#endif
#if ZMQG_ST_STAMPS
#define ST_STAMP(slot)                                                                                        \
    do {                                                                                                      \
        if (rp.clk && (threadIdx.x & 63u) == 0 && (slot) < 64u)                                               \
            rp.clk[64ull * (blockIdx.x * (kSxThreads / 64) + (threadIdx.x >> 6)) + (slot)] =                  \
                __builtin_amdgcn_s_memtime();                                                                 \
    } while (0)
#define ST_RTSTAMP(slot)                                                                                      \
    do {                                                                                                      \
        if (rp.clk && (threadIdx.x & 63u) == 0)                                                               \
            rp.clk[64ull * (blockIdx.x * (kSxThreads / 64) + (threadIdx.x >> 6)) + (slot)] =                  \
                __builtin_amdgcn_s_memrealtime();                                                             \
    } while (0)
#else
#define ST_STAMP(slot) do { } while (0)
#define ST_RTSTAMP(slot) do { } while (0)
#endif

namespace zmqg {

constexpr uint32_t kSxThreads = 2 * kFramesBS;             // compute waves 0..3, memory waves 4..7
constexpr uint32_t kSxCover = 144;                         // a super-step's 16-byte-aligned input cover per frame
constexpr uint32_t kSxInBuf = 64 * kSxCover;               // one input buffer per pair (9 DMA instructions)
constexpr uint32_t kSxRing = 336;                          // ring per frame: halves [0,256), overflow [256,320), pad
constexpr uint32_t kSxPair = 2 * kSxInBuf + 64 * kSxRing;  // 39,936 bytes
static_assert(kFramesWaves * kSxPair + 256 <= 160u * 1024u, "LDS of one workgroup");

// byte mask of bytes [0, nb) of dword d of a granule (nb 0..16)
__device__ __forceinline__ uint32_t lead_mask(uint32_t nb, uint32_t d)
{
    const int32_t b = (int32_t) nb - 4 * (int32_t) d;
    return b >= 4 ? 0xffffffffu : b <= 0 ? 0u : (1u << (8 * b)) - 1u;
}

template <bool DEC, class BigOp>
__global__ __launch_bounds__(kSxThreads) void k_frames_st(
    uint32_t n, const uint32_t *__restrict__ sid, const uint64_t *__restrict__ nonce, const uint8_t *__restrict__ flags,
    const uint64_t *__restrict__ in_off, const uint32_t *__restrict__ len, const uint8_t *__restrict__ in,
    const uint64_t *__restrict__ out_off, uint8_t *__restrict__ out, const DevSession *__restrict__ sessions,
    uint32_t max_sessions, uint32_t max_stream, uint8_t *__restrict__ flags_out, int32_t *__restrict__ status_out,
    ReplayOut rp, BigOp big, ZState *__restrict__ zs, FrameCtl ctl)
{
    __shared__ __attribute__((aligned(16))) uint8_t sx_lds[kFramesWaves * kSxPair];
    __shared__ unsigned long long sh_wmax[kFramesWaves];
    __shared__ CallState sh_cs;
    __shared__ uint32_t sh_steps[2 * kFramesWaves]; // per wave, both roles
    const bool lb = DEC && rp.lb_flag != nullptr;
    const bool use_ticket = lb && !rp.ordered; // (kernel-uniform)
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const bool mem = wave >= kFramesWaves;          // (wave-uniform) the memory wave of pair wave & 3
    const uint32_t wv = wave & (kFramesWaves - 1u); // the pair (= its compute wave)
    uint8_t *const pl = sx_lds + wv * kSxPair;
    const uint32_t pl_off = __builtin_amdgcn_readfirstlane((uint32_t) (uintptr_t) (StLdsVoid *) pl);
    uint8_t *const ring = pl + 2u * kSxInBuf;
    uint8_t *const myring = ring + kSxRing * lane;
    ST_STAMP(0u);
    ST_RTSTAMP(62u);
    if (mem && ZMQG_ST_MEMPRIO) // the memory wave's few VALU instructions go ahead of its partner's
        __builtin_amdgcn_s_setprio(ZMQG_ST_MEMPRIO);

    // ---- compute waves: the frame's descriptors, session key, first window
    uint32_t i = 0, ii = 0, s = 0, L_in = 0;
    bool valid = false, sid_ok = false, over = false;
    const uint8_t *src = nullptr;
    uint8_t *dst = nullptr;
    uint32_t key[8];
    uint32_t S = 0, n0 = 0, n1 = 0, hl = 1;
    uint64_t A = 0, B = 0;
    int32_t status = 0;
    uint32_t hw[3] = {0, 0, 0};
    uint32_t x0[16]; // window 0's stream words (decode: the wire; encode: payload bytes 0..31)
    auto fetch = [&](uint32_t wgv) {
        i = wgv * kFramesBS + wv * 64u + lane;
        valid = i < n;
        ii = valid ? i : n - 1;
        sid_ok = sid[ii] < max_sessions;
        s = sid_ok ? sid[ii] : 0u; // (a frame of an unknown session is not processed)
        const DevSession &ses = sessions[s];
#pragma unroll
        for (int t = 0; t < 8; ++t)
            key[t] = DEC ? ses.dec_key[t] : ses.enc_key[t];
        src = in + in_off[ii];
        dst = out + out_off[ii];
        L_in = len[ii];
        over = ctl.max_len != 0 && L_in > ctl.max_len; // the caller's bound broken
        if (!DEC) {
            hl = plaintext_header(flags[ii], ses.downgrade_sub, hw);
            S = sid_ok && !over ? 32u + hl + L_in : 0u;
            A = (uint64_t) (uintptr_t) src - 32u - hl;
            B = (uint64_t) (uintptr_t) dst;
            if (L_in >= 32u) { // payload bytes 0..31: two dwordx4 (and a dword when unaligned)
                load_bytes_c<32>(src, x0);
#pragma unroll
                for (int k = 8; k < 16; ++k)
                    x0[k] = 0;
            } else {
                load_window(src, (int) L_in, x0);
            }
        } else {
            A = (uint64_t) (uintptr_t) src;
            uint32_t d[17];
            frame_load_raw(A, 0, L_in, d);
#pragma unroll
            for (int k = 0; k < 16; ++k)
                x0[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], (uint32_t) A & 3u);
            B = (uint64_t) (uintptr_t) dst - 33u;
        }
    };
    // memory waves: the same frame's descriptors without the key and window
    // 0; decode's S is provisional (before the header checks, which only
    // ever zero it) -- enough to load the covers, and the same on both roles
    auto fetch_mem = [&](uint32_t wgv) {
        i = wgv * kFramesBS + wv * 64u + lane;
        valid = i < n;
        ii = valid ? i : n - 1;
        sid_ok = sid[ii] < max_sessions;
        s = sid_ok ? sid[ii] : 0u;
        const uint8_t *const sp = in + in_off[ii];
        uint8_t *const dp = out + out_off[ii];
        L_in = len[ii];
        over = ctl.max_len != 0 && L_in > ctl.max_len;
        if (!DEC) {
            hl = plaintext_header(flags[ii], sessions[s].downgrade_sub, hw);
            S = sid_ok && !over ? 32u + hl + L_in : 0u;
            A = (uint64_t) (uintptr_t) sp - 32u - hl;
            B = (uint64_t) (uintptr_t) dp;
        } else {
            S = sid_ok && !over ? L_in : 0u;
            A = (uint64_t) (uintptr_t) sp;
            B = (uint64_t) (uintptr_t) dp - 33u;
        }
    };
    // every wave's provisional window count -> sh_steps (the workgroup's
    // super-step count: every wave meets every barrier)
    auto publish_steps = [&]() {
        const uint32_t Sp = (DEC && !mem) ? (sid_ok && !over ? L_in : 0u) : S;
        uint32_t w = valid && Sp <= max_stream ? (Sp + 63u) >> 6 : 0u;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            const uint32_t o = __shfl_xor(w, d);
            w = o > w ? o : w;
        }
        if (lane == 0)
            sh_steps[wave] = w;
    };
    // memory waves: DMA lanes -- instruction j, lane -> granule k of frame f
    // (idx = 64 j + lane = 9 f + k); the first covers go out at once
    uint64_t dga[9];
    int32_t dlim[9];
    uint32_t dlow = 0; // bit j: granule k < 4 (window 0's part of super-step 0: read by its lane)
    u32x4 stg[ZMQG_ST_REGSTAGE ? 9 : 1]; // (register staging) the covers in flight
    auto dma = [&](uint32_t K) { // super-step K's covers -> input buffer K & 1 (no wait)
        const uint32_t b = pl_off + (K & 1u) * kSxInBuf;
#pragma unroll
        for (uint32_t j = 0; j < 9; ++j)
            if (!(ZMQG_ST_ABLATE & 2) && (int32_t) (128u * K) < dlim[j] && (K > 0u || !((dlow >> j) & 1u))) {
                if (ZMQG_ST_REGSTAGE)
                    stg[ZMQG_ST_REGSTAGE ? j : 0] = *(const GCU4 *) (uintptr_t) (dga[j] + 128ull * K);
                else
                    lds_dma16(dga[j] + 128ull * K, b + 1024u * j);
            }
    };
    auto land = [&](uint32_t K) { // (register staging) the covers loaded by dma(K) -> input buffer K & 1
        if (ZMQG_ST_REGSTAGE) {
            uint8_t *const b = pl + (K & 1u) * kSxInBuf + 16u * lane;
#pragma unroll
            for (uint32_t j = 0; j < 9; ++j)
                if (!(ZMQG_ST_ABLATE & 2) && (int32_t) (128u * K) < dlim[j] && (K > 0u || !((dlow >> j) & 1u)))
                    *(u32x4 *) (b + 1024u * j) = stg[ZMQG_ST_REGSTAGE ? j : 0];
        }
    };
    auto mem_start = [&]() {
        const uint32_t vv = (uint32_t) A & 15u;
        const uint64_t A16 = A - vv;
        const int32_t lim = valid && S <= max_stream && S ? (int32_t) (S + vv) : 0;
#pragma unroll
        for (uint32_t j = 0; j < 9; ++j) {
            const uint32_t idx = 64u * j + lane, f = idx / 9u, k = idx - 9u * f;
            dga[j] = shfl_u64(A16, f) + 16u * k;
            dlim[j] = __shfl(lim, (int) f) - (int32_t) (16u * k);
            dlow |= (k < 4u ? 1u : 0u) << j;
        }
        dma(0u); // window 1's covers
    };
    CallState c0{};
    if (threadIdx.x == 0) {
        c0.epoch = __hip_atomic_load(&zs->epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        c0.ticket = use_ticket ? atomicAdd(&zs->ticket, 1u) : 0u;
        c0.nbase = DEC ? 0ull : nonce_base(ctl);
    }
    if (!use_ticket) {
        if (mem) {
            fetch_mem(blockIdx.x);
            mem_start();
        } else {
            fetch(blockIdx.x);
        }
        publish_steps();
    }
    if (threadIdx.x == 0)
        sh_cs = c0;
    __syncthreads();
    const CallState cs = sh_cs;
    const uint32_t epoch = cs.epoch;
    const uint32_t wg = use_ticket ? cs.ticket : blockIdx.x;
    if (use_ticket) {
        if (mem) {
            fetch_mem(wg);
            mem_start();
        } else {
            fetch(wg);
        }
        publish_steps();
        __syncthreads();
    }
    uint32_t KS = 0; // super-steps of the workgroup
#pragma unroll
    for (uint32_t k = 0; k < 2 * kFramesWaves; ++k)
        KS = sh_steps[k] > KS ? sh_steps[k] : KS;
    KS = __builtin_amdgcn_readfirstlane((KS + 1u) >> 1);
    const uint32_t stw = __builtin_amdgcn_readfirstlane(sh_steps[wv]); // this pair's windows (provisional)
    ST_STAMP(1u);
    const uint64_t nbase = cs.nbase;
    unsigned long long *const list_ctr = zs->list_ctr + (epoch & 1u);
    if (blockIdx.x == 0 && threadIdx.x == 0)
        zs->list_ctr[(epoch & 1u) ^ 1u] = 0;

    if (!mem) {
        if (!DEC) {
            const uint64_t nc = frame_nonce(nonce, ctl, nbase, ii);
            n0 = bswap32((uint32_t) (nc >> 32));
            n1 = bswap32((uint32_t) nc);
        } else {
            if (L_in < 64u)
                mask_tail(x0, (int) L_in);
            // mechanism_base.cpp:14-25, curve_mechanism_base.cpp:80-97
            const uint32_t b0 = x0[0] & 0xffu;
            if (L_in <= 1u || L_in <= b0)
                status = ZMQG_ERR_MALFORMED_UNSPECIFIED;
            else if (L_in < 8u || x0[0] != 0x53454d07u || x0[1] != 0x45474153u)
                status = ZMQG_ERR_UNEXPECTED_COMMAND;
            else if (L_in < 33u)
                status = ZMQG_ERR_MALFORMED_MESSAGE;
            if (!sid_ok)
                status = ZMQG_ERR_SESSION;
            if (over)
                status = ZMQG_ERR_BOUND;
            n0 = x0[2];
            n1 = x0[3];
            S = status == 0 ? L_in : 0u;
        }
    }
    const bool small = valid && S <= max_stream;
    unsigned long long vn = 0, wexcl = 0, psn = 0, wagg = 0;
    if (DEC) {
        if (!mem) {
            vn = valid && status == 0 ? (((unsigned long long) bswap32(n0) << 32) | bswap32(n1)) : 0ull;
            psn = rp.peer[s];
            if (valid && !lb) { // (several sessions: the replay tables' input)
                rp.vout[i] = vn;
                rp.psnap[i] = psn;
                if (rp.iota)
                    rp.iota[i] = i;
            }
        }
        if (lb) { // (the barrier is the whole workgroup's)
            unsigned long long sc = vn;
            if (!mem) {
#pragma unroll
                for (int d = 1; d < 64; d <<= 1) {
                    const unsigned long long o = __shfl_up(sc, d);
                    if ((int) lane >= d)
                        sc = o > sc ? o : sc;
                }
                if (lane == 63)
                    sh_wmax[wv] = sc;
            }
            const unsigned long long up = __shfl_up(sc, 1);
            __syncthreads();
            if (!mem) {
                for (uint32_t k = 0; k < kFramesWaves; ++k) {
                    if (k < wv)
                        wexcl = sh_wmax[k] > wexcl ? sh_wmax[k] : wexcl;
                    wagg = sh_wmax[k] > wagg ? sh_wmax[k] : wagg;
                }
                if (lane > 0)
                    wexcl = up > wexcl ? up : wexcl;
                if (threadIdx.x == 0)
                    lookback_publish(rp.lb_flag + wg, rp.lb_agg + wg, wagg, epoch, 1);
            }
        }
    }
    const bool is_big = valid && !small && S > 0;
    if (!small)
        S = 0;
    // compute waves hand the frame's final stream length (decode: 0 after a
    // failed header check) to the memory wave through overflow slot 2 (first
    // written in super-step 2; read in super-step 0)
    if (!mem)
        *(uint32_t *) (myring + 288u) = S;
    uint32_t nw = (S + 63u) >> 6;
    const uint32_t va = (uint32_t) A & 15u; // input phase: stream byte 0 at cover byte va
    const uint32_t ub = (uint32_t) B & 15u; // output phase: output byte q = ub + stream byte
    const uint32_t u4 = ub & 3u, up = u4 ? u4 : 4u;

    PolyKey32 pk;
    Poly32 h = {0, 0, 0, 0, 0};
    uint32_t spad[4], wtag[4] = {0, 0, 0, 0}, fl = 0;

    if (mem) {
        // ================================================================ memory wave
        const uint32_t lo = DEC ? 33u : 32u; // first stream byte of the ring-stored output
        const uint64_t Bg = B - ub;
        // output q ranges (q = ub + stream byte, from the 16-byte boundary
        // Bg): head [hs, he) and tail [ts, te) by this lane, whole granules
        // [ga, gb) by the wave; from the final S (super-step 0)
        const uint32_t hs = ub + lo, hr = (hs + 15u) & ~15u;
        uint32_t te = 0, he = 0, ts = 0, ga = 0, gb = 0;
        // store lanes: instruction j, lane -> granule k = lane & 7 of frame f = 8 j + lane / 8
        const uint32_t sk = lane & 7u;
        uint64_t sga[8];
        uint32_t srg[8];
        int32_t sglo[8], sghi[8];
        uint32_t smask[8][4]; // k = 0 lanes: the bytes of granule 0 that come from the overflow slot
        auto setup_out = [&]() { // (super-step 0, after the hand-off of the final S)
            S = *(const uint32_t *) (myring + 288u);
            nw = (S + 63u) >> 6;
            te = S > lo ? ub + S : 0u;
            he = te ? (hr < te ? hr : te) : 0u;
            if (te && (te >> 4) > (hr >> 4)) {
                ga = hr >> 4;
                gb = te >> 4;
            }
            const uint32_t tsf = te & ~15u;
            ts = te ? (tsf > he ? tsf : he) : 0u;
#pragma unroll
            for (uint32_t j = 0; j < 8; ++j) {
                const uint32_t f = 8u * j + (lane >> 3);
                sga[j] = shfl_u64(Bg, f) + 16u * sk;
                srg[j] = kSxRing * f + 16u * sk;
                sglo[j] = __shfl((int) ga, (int) f) - (int32_t) sk;
                sghi[j] = __shfl((int) gb, (int) f) - (int32_t) sk;
                const uint32_t ubf = (uint32_t) __shfl((int) ub, (int) f);
#pragma unroll
                for (uint32_t d = 0; d < 4; ++d)
                    smask[j][d] = lead_mask(ubf, d);
            }
        };
        // super-step K's ring granules -> memory (granule 0 completed from
        // super-step K-1's overflow slot)
        auto coop = [&](uint32_t K) {
            const uint32_t half = 128u * (K & 1u), ovf = 256u + 16u * ((K - 1u) & 3u);
            u32x4 sv[8];
#pragma unroll
            for (uint32_t j = 0; j < 8; ++j)
                sv[j] = *(const u32x4 *) (ring + srg[j] + half);
            if (K > 0u && sk == 0u) {
#pragma unroll
                for (uint32_t j = 0; j < 8; ++j) {
                    const u32x4 o = *(const u32x4 *) (ring + srg[j] + ovf);
                    sv[j].x = (o.x & smask[j][0]) | (sv[j].x & ~smask[j][0]);
                    sv[j].y = (o.y & smask[j][1]) | (sv[j].y & ~smask[j][1]);
                    sv[j].z = (o.z & smask[j][2]) | (sv[j].z & ~smask[j][2]);
                    sv[j].w = (o.w & smask[j][3]) | (sv[j].w & ~smask[j][3]);
                }
            }
            const int32_t g = (int32_t) (8u * K);
#if ZMQG_ST_STAMPS
            if (K == 2u) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                ST_STAMP(55u);
            }
#endif
#pragma unroll
            for (uint32_t j = 0; j < 8; ++j)
                if (!(ZMQG_ST_ABLATE & 1) && g >= sglo[j] && g < sghi[j]) {
                    const uint64_t a = sga[j] + 128ull * K;
                    if (ZMQG_ST_STORE == 1)
                        __builtin_nontemporal_store(sv[j], (GU4 *) (uintptr_t) a);
                    else if (ZMQG_ST_STORE == 2) // (counted by the explicit vmcnt(0) waits; s_nop: data hazard)
                        asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(a), "v"(sv[j]) : "memory");
                    else if (ZMQG_ST_STORE == 3)
                        asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1" ::"v"(a), "v"(sv[j])
                                     : "memory");
                    else
                        *(GU4 *) (uintptr_t) a = sv[j];
                }
#if ZMQG_ST_STAMPS
            if (K == 2u)
                ST_STAMP(56u);
#endif
        };
        auto head = [&]() { // output bytes [hs, he) of granule hs / 16 (super-step 0, k >= 2)
            if (__builtin_amdgcn_ballot_w64(he > hs) != 0) {
                if (he > hs) {
                    const uint32_t g = hs & ~15u;
                    const u32x4 v = *(const u32x4 *) (myring + g);
                    granule_store_part(Bg + g, hs - g, he - g, v);
                }
            }
        };

        land(0u);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); // super-step 0's covers (issued at entry)
        ST_STAMP(2u);
#pragma unroll 1
        for (uint32_t K = 0; K < KS; ++K) {
            __syncthreads(); // B_K: super-step K's covers are in; super-step K-1's ring is complete
            ST_STAMP(3u + (K < 16u ? K : 16u));
            if (K == 0u)
                setup_out();
            if (K + 1u < KS)
                dma(K + 1u);
            if (K == 3u)
                ST_STAMP(54u);
            if (K > 0u)
                coop(K - 1u);
            if (K == 1u)
                head();
            ST_STAMP(20u + (K < 16u ? K : 16u));
            if (K + 1u < KS)
                land(K + 1u);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); // the DMA, before B_K+1
            ST_STAMP(37u + (K < 16u ? K : 16u));
        }
        __syncthreads(); // B_KS: the last super-step's ring is complete
        ST_STAMP(58u);
        if (KS > 0u) {
            coop(KS - 1u);
            if (KS == 1u)
                head();
            if (__builtin_amdgcn_ballot_w64(te > ts) != 0) {
                if (te > ts) { // output bytes [ts, te) of granule ts / 16
                    const uint32_t G = ts >> 4, Kg = G >> 3, k = G & 7u;
                    u32x4 v = *(const u32x4 *) (myring + 128u * (Kg & 1u) + 16u * k);
                    if (k == 0u) {
                        const u32x4 o = *(const u32x4 *) (myring + 256u + 16u * ((Kg - 1u) & 3u));
                        const uint32_t m0 = lead_mask(ub, 0), m1 = lead_mask(ub, 1), m2 = lead_mask(ub, 2),
                                       m3 = lead_mask(ub, 3);
                        v.x = (o.x & m0) | (v.x & ~m0);
                        v.y = (o.y & m1) | (v.y & ~m1);
                        v.z = (o.z & m2) | (v.z & ~m2);
                        v.w = (o.w & m3) | (v.w & ~m3);
                    }
                    granule_store_part(Bg + ts, 0u, te - ts, v);
                }
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); // every store of the frames drained before B_fin
        ST_STAMP(59u);
        __syncthreads();                                 // B_fin
        ST_STAMP(60u);
        ST_STAMP(61u);
        ST_RTSTAMP(63u);
        return;
    }

    // ==================================================================== compute wave
    // window w's output words y (ycarry: the previous window's last word) ->
    // ring half K & 1 as aligned dwords at the destination's 4-byte phase
    // (the first only when it merges the carry); a second window's dwords
    // past the half's end -> overflow slot K & 3
    auto ring_put = [&](uint32_t K, uint32_t hh, const uint32_t y[16], uint32_t ycarry) {
        if (ZMQG_ST_ABLATE & 4)
            return;
        const uint32_t P0 = 128u * (K & 1u) + 64u * hh + ub - up; // dword 0's position
        const uint32_t hend = 128u * (K & 1u) + 128u, ovf = 256u + 16u * (K & 3u);
        const uint32_t sft = 4u - up;
        uint32_t o[17];
        o[0] = __builtin_amdgcn_alignbyte(y[0], ycarry, sft);
#pragma unroll
        for (int m = 1; m < 16; ++m)
            o[m] = __builtin_amdgcn_alignbyte(y[m], y[m - 1], sft);
        o[16] = __builtin_amdgcn_alignbyte(0u, y[15], sft);
        if (up != 4u)
            *(uint32_t *) (myring + P0) = o[0];
#pragma unroll
        for (uint32_t m = 1; m < 17; ++m) {
            uint32_t p = P0 + 4u * m;
            if (hh == 1u && m >= 13u) // (dwords 0..12 of a second window never pass the half's end)
                p = p >= hend ? p - hend + ovf : p;
            *(uint32_t *) (myring + p) = o[m];
        }
    };

    uint32_t cp[16];                // ciphertext of the window whose MAC is absorbed next step
    uint32_t cp_j0 = 2, cp_len = 0; // its first block slot and ciphertext bytes
    uint32_t ycarry = 0;
    // ---- window 0 (Poly1305 key, first 32 ciphertext bytes, header)
    {
        uint32_t ks[16];
        salsa20_block(ks, key, n0, n1, 0, 0);
        pk = poly32_key(ks[0], ks[1], ks[2], ks[3]);
#pragma unroll
        for (int k = 0; k < 4; ++k)
            spad[k] = ks[4 + k];
        uint32_t x[16];
        if (DEC) {
#pragma unroll
            for (int k = 0; k < 16; ++k)
                x[k] = x0[k];
#pragma unroll
            for (int k = 0; k < 4; ++k)
                wtag[k] = x[4 + k];
        } else {
            // plaintext bytes 0..31 = header || payload[0 .. 32-hl)
            uint32_t pt[8];
            switch (hl) {
            case 1: shift_in<1>(x0, pt); break;
            case 2: shift_in<2>(x0, pt); break;
            case 8: shift_in<8>(x0, pt); break;
            default: shift_in<11>(x0, pt); break;
            }
            pt[0] |= hw[0];
            pt[1] |= hw[1];
            pt[2] |= hw[2];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                x[k] = 0;
                x[8 + k] = pt[k];
            }
        }
        uint32_t y[16];
#pragma unroll
        for (int k = 0; k < 16; ++k)
            y[k] = x[k] ^ ks[k];
        if (!DEC && S < 64u)
            mask_tail(y, (int) S);
#pragma unroll
        for (int k = 0; k < 16; ++k)
            cp[k] = DEC ? x[k] : y[k];
        cp_len = (S < 64u ? S : 64u) - 32u; // (S = 0: unused)
        if (DEC)
            fl = y[8] & 3u;
        if (nw > 0u)
            ring_put(0u, 0u, y, 0u); // (the carry lands below the output: never stored)
        ycarry = y[15];
    }
    call_state_count(zs);
    ST_STAMP(2u);

    // ---- windows 1 ..
    auto window = [&](uint32_t K, uint32_t hh) {
        const uint32_t t = 2u * K + hh;
        const bool act = t < nw;
        uint32_t d[17];
        {
            const uint32_t *const p =
                (const uint32_t *) (pl + (K & 1u) * kSxInBuf + kSxCover * lane + ((va + 64u * hh) & ~3u));
#pragma unroll
            for (int m = 0; m < 17; ++m)
                d[m] = (ZMQG_ST_ABLATE & 8) ? key[m & 7] + t * 0x9e3779b9u + (uint32_t) m : p[m];
        }
        if (K == 3u && hh == 0u)
            ST_STAMP(54u);
        uint32_t ks[16];
        if (ZMQG_ST_ABLATE & 16) {
#pragma unroll
            for (int k = 0; k < 16; ++k)
                ks[k] = key[k & 7] ^ (t * 0x9e3779b9u + k);
        } else {
            salsa20_block(ks, key, n0, n1, t, 0);
        }
        // The previous window's MAC, the four-block form for every lane in the
        // keystream's basic block (see k_frames_seq); lanes whose window was
        // not four full blocks keep h and take the general form below.
        const bool pv = t - 1u < nw;
        const bool full = pv && cp_j0 == 0u && cp_len == 64u;
        {
            Poly32 hf = h;
            if (ZMQG_ST_ABLATE & 32)
                hf.h0 ^= cp[0] ^ cp[5] ^ cp[11];
            else
                poly32_window_full(hf, pk, cp);
            h.h0 = full ? hf.h0 : h.h0;
            h.h1 = full ? hf.h1 : h.h1;
            h.h2 = full ? hf.h2 : h.h2;
            h.h3 = full ? hf.h3 : h.h3;
            h.h4 = full ? hf.h4 : h.h4;
        }
#pragma unroll
        for (int k = 0; k < 16; ++k)
            asm volatile("" : "+v"(ks[k]));
        asm volatile("" : "+v"(h.h0), "+v"(h.h1), "+v"(h.h2), "+v"(h.h3), "+v"(h.h4));
        if (!(ZMQG_ST_ABLATE & 32) && __builtin_amdgcn_ballot_w64(pv && !full) != 0) {
            if (pv && !full)
                poly32_window(h, pk, cp, cp_j0, cp_len);
        }
        if (K == 3u && hh == 0u)
            ST_STAMP(55u);
        uint32_t x[16];
        const uint32_t sa = va & 3u;
#pragma unroll
        for (int k = 0; k < 16; ++k)
            x[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], sa);
        const bool tail = act && S < 64u * t + 64u;
        if (DEC && __builtin_amdgcn_ballot_w64(tail) != 0) {
            if (tail)
                mask_tail(x, (int) (S - 64u * t));
        }
        uint32_t y[16];
#pragma unroll
        for (int k = 0; k < 16; ++k)
            y[k] = x[k] ^ ks[k];
        if (!DEC && __builtin_amdgcn_ballot_w64(tail) != 0) {
            if (tail)
                mask_tail(y, (int) (S - 64u * t));
        }
#pragma unroll
        for (int k = 0; k < 16; ++k)
            cp[k] = DEC ? x[k] : y[k];
        cp_j0 = 0;
        cp_len = act ? (S - 64u * t < 64u ? S - 64u * t : 64u) : 0u;
        if (K == 3u && hh == 0u)
            ST_STAMP(56u);
        if (act)
            ring_put(K, hh, y, ycarry);
        if (K == 3u && hh == 0u)
            ST_STAMP(57u);
        ycarry = y[15];
    };

#pragma unroll 1
    for (uint32_t K = 0; K < KS; ++K) {
        __syncthreads(); // B_K: super-step K's covers have landed; the ring half is free
        ST_STAMP(3u + (K < 16u ? K : 16u));
        if (K > 0u && 2u * K < stw)
            window(K, 0u);
        ST_STAMP(20u + (K < 16u ? K : 16u));
        if (2u * K + 1u < stw)
            window(K, 1u);
        ST_STAMP(37u + (K < 16u ? K : 16u));
    }
    __syncthreads(); // B_KS
    ST_STAMP(58u);
    // the last window's MAC
    if (stw > 0u && nw == stw)
        poly32_window(h, pk, cp, cp_j0, cp_len);
    ST_STAMP(59u);
    __syncthreads(); // B_fin: the memory waves' stores of these frames are done; they have left
    ST_STAMP(60u);

    unsigned long long excl = 0;
    if (lb) {
        const unsigned long long P = lookback_excl(wg, epoch, rp.lb_flag, rp.lb_agg, rp.lb_inc);
        if (threadIdx.x == 0) {
            const unsigned long long inc = P > wagg ? P : wagg;
            // (a grid of at most kFramesBS workgroups looks back over every
            // aggregate in one round and needs no inclusive values)
            if (gridDim.x > kFramesBS)
                lookback_publish(rp.lb_flag + wg, rp.lb_inc + wg, inc, epoch, 2);
            if (wg + 1 == gridDim.x) {
                *rp.peer = inc > psn ? inc : psn;
                if (rp.smax)
                    *rp.smax = inc;
            }
        }
        excl = P > wexcl ? P : wexcl;
        if (excl < psn)
            excl = psn;
    }
    if (is_big && !ctl.no_body) {
        if (lb) { // the body's finisher applies the rule to this frame
            rp.excl[i] = excl;
            rp.psnap[i] = psn;
        }
        big(i, list_ctr, nbase);
    }
    call_state_end<DEC>(zs, ctl, cs, n);
    if (!DEC && valid && ctl.enc_status)
        ctl.enc_status[i] = !sid_ok ? ZMQG_ERR_SESSION : over ? ZMQG_ERR_BOUND : 0;
    if (!valid || !small)
        return;
    if (S == 0) { // decode: header failure (encode: a frame not processed)
        if (DEC)
            fail_unprocessed(status, L_in, dst, flags_out + i, status_out + i, zs, ctl);
        return;
    }
    uint32_t tag[4];
    poly32_finish(h, spad, tag);
    if (!DEC) {
        // "\x07MESSAGE" || nonce || tag: wire bytes 0..31 (the rest went out through the ring)
        const uint32_t o[16] = {0x53454d07u, 0x45474153u, n0, n1, tag[0], tag[1], tag[2], tag[3]};
        store_bytes_c<32>(dst, o);
    } else {
        if (lb && !(vn > excl))
            status = ZMQG_ERR_INVALID_SEQUENCE; // src/curve_mechanism_base.cpp:99-104 (before the MAC)
        else if ((tag[0] ^ wtag[0]) | (tag[1] ^ wtag[1]) | (tag[2] ^ wtag[2]) | (tag[3] ^ wtag[3]))
            status = ZMQG_ERR_CRYPTOGRAPHIC; // src/curve_mechanism_base.cpp:277-281
        status_out[i] = status;
        flags_out[i] = status == 0 ? (uint8_t) fl : 0;
        if (status != 0) // (the memory wave drained its stores of this frame before B_fin)
            zero_bytes(dst, S - 33u);
    }
    ST_STAMP(61u);
    ST_RTSTAMP(63u);
}

} // namespace zmqg
