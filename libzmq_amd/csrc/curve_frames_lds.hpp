// curve_frames_lds.hpp -- the one-lane-per-frame kernel with its global
// traffic staged through LDS (k_frames_lds).
//
// Same frame semantics as k_frames_seq (curve_frames.hpp): one lane owns one
// frame, walks its 64-byte keystream windows in order with the sequential
// radix-2^32 Poly1305, and applies the decode header checks and replay rule
// (src/curve_mechanism_base.cpp:80-284, src/mechanism_base.cpp:14-25).  What
// changes is how a wave moves its 64 frames' bytes.  In k_frames_seq every
// lane loads and stores its own frame, so each dwordx4 instruction touches 64
// different cache lines; profiles of that kernel showed a quarter of each
// window's time in load waits and store issue, and the load latency stretched
// to a whole window (tools/seq_stamps.hip).  Here the wave moves the bytes
// cooperatively, each instruction covering whole 64- and 80-byte runs:
//   * input: window t's 16-byte-aligned cover (5 granules, 80 bytes) of each
//     of the 64 frames comes in by LDS-DMA (global_load_lds_dwordx4): pair
//     idx = 64j + lane of instruction j moves granule idx % 5 of frame
//     idx / 5, so consecutive lanes read consecutive granules of a frame.  It
//     is issued one window ahead into the other of two buffers; the owning
//     lane reads its 64 stream bytes from LDS at the frame's byte offset
//     (unaligned ds_read_b128, supported on gfx950).
//   * output: the owning lane writes its 64 output bytes into a per-frame
//     ring at the destination's byte alignment; one window later the wave
//     stores the ring's aligned granules, pair idx = 64j + lane moving
//     granule lane % 4 of frame 16j + lane / 4 (four dwordx4 per window),
//     whole granules with dwordx4 and the at most two partial granules at a
//     frame's edges byte-exact, so neighbouring frames are never touched.
//     A frame's output range [u, u + S) spans ceil((u + S) / 64) granule
//     windows: the last window's final u bytes go out in one step more.
// Ring slot (128 + 16 bytes) of a frame whose output starts at byte u = B & 15
// of a granule: window t is written at [64(t&1) + u, +64); an odd window's
// bytes beyond 128 are copied to [0, 16) before the next (even) window is
// written, so [64(t&1), +64) always holds window t's aligned granules (its
// first u bytes from window t-1).
// Measured alternatives: 64-byte-aligned runs
// (ZMQG_LDS_SECTOR=64) cut the write traffic WRITE_SIZE reports from 1.71x to
// 1.38x the payload but were 5-10 % slower (the ring copies grow to 64
// bytes); one input buffer refilled right after it is read (ZMQG_LDS_INBUF=1)
// was slower again (the LDS reads are waited for before the DMA).
#pragma once

#include "curve_frames.hpp"

namespace zmqg {

#ifndef ZMQG_LDS_SECTOR
#define ZMQG_LDS_SECTOR 16 // output runs are aligned to this many bytes (16 or 64)
#endif
// Issue priority by phase.  Two waves share each SIMD here (two workgroups
// per CU) and the arbiter favours the older one, so a wave that reaches its
// descriptor and key loads, a step's DMA and stores, or its epilogue while the
// other is deep in a keystream waits behind that keystream to issue them, and
// its memory latency starts late.  With s_setprio 3 over those stretches and
// 0 over the keystream the memory work of either wave goes out at once and
// the other's VALU stream fills the wait: config 4 (16 Mi x 256 B, 1,024
// sessions) 9.87-9.89 ms per encode+decode against 11.12-11.18 for no
// priorities on one box; 3/1 gave 9.91-10.26, 2/0 10.52-10.56
// (DESIGN.md section 3.1).
#ifndef ZMQG_LDS_PRIO
#define ZMQG_LDS_PRIO 2 // priority while issuing memory work / during the keystream: 0 none, 1 3/1, 2 3/0, 3 2/0
#endif
#define LDS_PRIO_MEM (ZMQG_LDS_PRIO == 3 ? 2 : 3)
#define LDS_PRIO_KS (ZMQG_LDS_PRIO == 1 ? 1 : 0)
// (s_setprio takes an immediate)
#define LDS_PRIO(lv)                                                                                   \
    do {                                                                                               \
        if (ZMQG_LDS_PRIO)                                                                             \
            __builtin_amdgcn_s_setprio(lv);                                                            \
    } while (0)
#ifndef ZMQG_LDS_ALIGN64
#define ZMQG_LDS_ALIGN64 1 // cooperative stores as 64-byte-aligned pieces (0: the windows' own granules)
#endif
#ifndef ZMQG_LDS_INBUF
#define ZMQG_LDS_INBUF 2 // input buffers per wave (1: refilled right after it is read)
#endif
constexpr uint32_t kStSector = ZMQG_LDS_SECTOR;
constexpr uint32_t kStNIn = ZMQG_LDS_INBUF;
static_assert(kStSector == 16 || kStSector == 64, "output sector");
static_assert(kStNIn == 1 || kStNIn == 2, "input buffers");
constexpr uint32_t kStRing = 128 + kStSector;                   // output ring slot
constexpr uint32_t kStInBuf = 64 * kStIn;                       // one input buffer per wave
constexpr uint32_t kStWave = kStNIn * kStInBuf + 64 * kStRing;  // 19,456 bytes per wave (16, 2)

typedef __attribute__((address_space(1))) void StGVoid;

// bytes [lo, hi) (0 <= lo < hi <= 16) of granule v at the 16-byte aligned
// address a: the bytes before the first whole word (up to 3), the whole
// words (up to 4), the bytes after the last (up to 3) -- ten lane-predicated
// stores at most (a frame's edge granules; the per-byte form issued twenty).
__device__ __forceinline__ void granule_store_part(uint64_t a, uint32_t lo, uint32_t hi, const u32x4 &v)
{
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    const uint32_t fa = (lo + 3u) >> 2, la = hi >> 2; // whole words [fa, la)
    const uint32_t le = (4u * fa < hi ? 4u * fa : hi); // leading bytes [lo, le)
    uint32_t wl = w[0], wt = w[0];                      // the words holding them / the trailing bytes
#pragma unroll
    for (uint32_t q = 1; q < 4; ++q) {
        if (q == (lo >> 2))
            wl = w[q];
        if (q == la)
            wt = w[q];
    }
#pragma unroll
    for (uint32_t b = 0; b < 3; ++b)
        if (lo + b < le)
            *(GU8 *) (uintptr_t) (a + lo + b) = (uint8_t) (wl >> (8u * ((lo + b) & 3u)));
#pragma unroll
    for (uint32_t q = 0; q < 4; ++q)
        if (q >= fa && q < la)
            *(GU32 *) (uintptr_t) (a + 4u * q) = w[q];
    const uint32_t ts = 4u * la > le ? 4u * la : le; // trailing bytes [ts, hi), inside word la
#pragma unroll
    for (uint32_t b = 0; b < 3; ++b)
        if (ts + b < hi && la < 4u)
            *(GU8 *) (uintptr_t) (a + ts + b) = (uint8_t) (wt >> (8u * ((ts + b) & 3u)));
}

template <bool DEC, class BigOp>
__global__ __launch_bounds__(kFramesBS) void k_frames_lds(
    uint32_t n, const uint32_t *__restrict__ sid, const uint64_t *__restrict__ nonce, const uint8_t *__restrict__ flags,
    const uint64_t *__restrict__ in_off, const uint32_t *__restrict__ len, const uint8_t *__restrict__ in,
    const uint64_t *__restrict__ out_off, uint8_t *__restrict__ out, const DevSession *__restrict__ sessions,
    uint32_t max_sessions, uint32_t max_stream, uint8_t *__restrict__ flags_out, int32_t *__restrict__ status_out,
    ReplayOut rp, BigOp big, ZState *__restrict__ zs, FrameCtl ctl)
{
    __shared__ __attribute__((aligned(16))) uint8_t st_lds[kFramesWaves * kStWave];
    const bool lb = DEC && rp.lb_flag != nullptr;
    SEQ_STAMP(0u);
    LDS_PRIO(LDS_PRIO_MEM);
    __shared__ unsigned long long sh_wmax[kFramesWaves];
    __shared__ CallState sh_cs;
    const bool use_ticket = lb && !rp.ordered; // (kernel-uniform)
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;

    // The frame's descriptors, session key and first window (as in
    // k_frames_seq): without a look-back ticket to take, the workgroup's
    // frames are known at entry, so these loads go out before the call
    // state's round trip instead of after it.
    uint32_t i = 0, ii = 0, s = 0, L_in = 0;
    bool valid = false, sid_ok = false, over = false;
    const uint8_t *src = nullptr;
    uint8_t *dst = nullptr;
    uint32_t key[8];
    uint32_t S = 0, n0 = 0, n1 = 0, hl = 1;
    uint64_t A = 0, B = 0, nc = 0;
    unsigned long long psn = 0; // decode: the session's peer nonce before the batch
    int32_t status = 0;
    uint32_t hw[3] = {0, 0, 0};
    uint32_t x0[16]; // window 0's stream words (decode: the wire; encode: payload bytes 0..31)
    auto fetch = [&](uint32_t wgv) {
        i = wgv * kFramesBS + threadIdx.x;
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
        over = frame_over<DEC>(ctl, L_in, out_off[ii]); // the caller's bounds broken
        if (!DEC) {
            if (!ctl.nonce_ctr) // (device-assigned nonces need the call state's base)
                nc = nonce[ii];
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
            // the wire frame's first window: header, nonce, tag, 32 ciphertext bytes
            A = (uint64_t) (uintptr_t) src;
            uint32_t d[17];
            frame_load_raw(A, 0, L_in, d);
#pragma unroll
            for (int k = 0; k < 16; ++k)
                x0[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], (uint32_t) A & 3u);
            B = (uint64_t) (uintptr_t) dst - 33u;
            psn = rp.peer[s];
        }
    };
    // the call state (see call_state_begin): thread 0's reads go out first,
    // the frame's loads behind them, and the reads are waited for (to publish
    // them in LDS) only after both are in flight
    CallState c0{};
    if (threadIdx.x == 0) {
        c0.epoch = __hip_atomic_load(&zs->epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        c0.ticket = use_ticket ? atomicAdd(&zs->ticket, 1u) : 0u;
        c0.nbase = DEC ? 0ull : nonce_base(ctl);
    }
    if (!use_ticket)
        fetch(blockIdx.x);
    if (threadIdx.x == 0)
        sh_cs = c0;
    __syncthreads();
    const CallState cs = sh_cs;
    const uint32_t epoch = cs.epoch;
    const uint32_t wg = use_ticket ? cs.ticket : blockIdx.x;
    if (use_ticket)
        fetch(wg);
    const uint64_t nbase = cs.nbase;
    unsigned long long *const list_ctr = zs->list_ctr + (epoch & 1u);
    if (blockIdx.x == 0 && threadIdx.x == 0)
        zs->list_ctr[(epoch & 1u) ^ 1u] = 0;

    if (!DEC) {
        if (ctl.nonce_ctr)
            nc = nbase + ii;
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
        B = (uint64_t) (uintptr_t) dst - 33u;
    }
    const bool small = valid && S <= max_stream;
    unsigned long long vn = 0, wexcl = 0, wagg = 0;
    if (DEC) {
        vn = valid && status == 0 ? (((unsigned long long) bswap32(n0) << 32) | bswap32(n1)) : 0ull;
        if (valid && !lb) { // (several sessions: the replay tables' input)
            rp.vout[i] = vn;
            rp.psnap[i] = psn;
            if (rp.iota)
                rp.iota[i] = i;
        }
        if (lb) {
            const unsigned long long sc = wave_scan_max_u64(vn);
            const unsigned long long up = wave_prev_u64(sc);
            if (lane == 63)
                sh_wmax[wv] = sc;
            __syncthreads();
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
    const bool is_big = valid && !small && S > 0;
    if (!small)
        S = 0;
    const uint32_t nw = (S + 63u) >> 6;
    const uint32_t steps = __builtin_amdgcn_readfirstlane(wave_max_u32(nw));

    // ---- the wave's staging areas and its lanes' share of the cooperative moves
    uint8_t *const wlds = st_lds + wv * kStWave;
    uint8_t *const ring = wlds + kStNIn * kStInBuf;
    uint8_t *const myring = ring + kStRing * lane;
    const uint32_t va = (uint32_t) A & 15u;
    const uint32_t ub = (uint32_t) B & (kStSector - 1u);
    // load pair j: granule lk of frame lf; loaded at step t when 64t + 16 lk is
    // below that frame's va + S (the granule holds a stream byte)
    uint64_t la[5];
    uint32_t lrel[5], llim[5];
    {
        const uint64_t Ab = A - va;
        const uint32_t lim = S ? va + S : 0u;
#pragma unroll
        for (uint32_t j = 0; j < 5; ++j) {
            const uint32_t idx = 64u * j + lane, f = idx / 5u, k = idx - 5u * f;
            lrel[j] = 16u * k;
            la[j] = shfl_u64(Ab, f) + lrel[j];
            llim[j] = (uint32_t) __shfl((int) lim, (int) f);
            const int fva = __shfl((int) va, (int) f); // (k_frames_seq's notes)
            if (ZMQG_SEQ_SKIP5 && k == 4u && fva == 0)
                llim[j] = 0;
        }
    }
    // Encode into back-to-back frames (every lane's frame processed, at least
    // 80 stream bytes, all of the wave's length in windows, each starting
    // where the lane before's ends: packed
    // wire output, wave-uniform): the granule a frame boundary falls in is
    // written whole, once, by the later frame's lane at the end (its wire
    // bytes 0..15 after the earlier frame's last bytes, read from that
    // lane's ring), and so are the 16-byte granules of the header, nonce,
    // tag and first ciphertext bytes -- the cooperative stores cover only
    // whole granules, and no byte-exact edge stores remain but the wave's
    // own two ends (without this, an encode wave issued ~3x the store
    // instructions of a decode wave, and partial granules cost write traffic
    // beyond the wire bytes: DESIGN.md section 3.1).
    bool merge = false;
    uint32_t pend = 0; // merge: ring-relative end (ub + S) of the lane before's frame
    if (!DEC) {
        const uint32_t pl = lane ? lane - 1u : 0u;
        const uint64_t Bp = shfl_u64(B, pl);
        const uint32_t Sp = (uint32_t) __shfl((int) S, (int) pl);
        pend = ((uint32_t) Bp & (kStSector - 1u)) + Sp;
        // (every frame's last window the wave's last: a lane past its frame
        // would overwrite its ring, and the tail read below, with later steps)
        const bool ok = valid && S >= 80u && nw == steps && (lane == 0 || Bp + Sp == B);
        merge = kStSector == 16 && __builtin_amdgcn_ballot_w64(!ok) == 0;
    }
    // store pair j: granule lane % 4 of frame 16j + lane / 4 of each window; its
    // frame's cooperatively stored bytes are ring-relative [slo, shi) (decode:
    // the payload, stream bytes 33..S; encode: the ciphertext, 32..S; merged
    // encode: the whole granules inside it, and the last lane's tail)
    // Each step stores one 64-byte piece of each frame that is 64-byte
    // aligned in memory: ring-relative [64u + sh, +64) at step u + 1, sh = 0
    // when the frame's base granule is 64-byte aligned, else sh = d - 64 with
    // d the ring offset of the first 64-byte boundary (16, 32 or 48) when d >
    // ub (the piece then ends inside the window before the one just computed)
    // -- whole 64-byte segments, so no segment is written in two halves by
    // two steps (WRITE_SIZE counted those twice: 1.5-1.7x the bytes).  The
    // ring holds ring-relative granule r at r mod 128 for the two windows it
    // keeps (the spill copy keeps that true across the odd windows' overflow).
    uint64_t sa[4];
    uint32_t sro[4], slo4[4], shi4[4];
    int32_t ssh4[4];
    const uint32_t srel = 16u * (lane & 3u);
    {
        const uint64_t Gb = B - ub;
        const uint32_t d = (64u - ((uint32_t) Gb & 63u)) & 63u;
        const int32_t sh = ZMQG_LDS_ALIGN64 && d > ub ? (int32_t) d - 64 : 0;
        uint32_t slo = ub + (DEC ? 33u : 32u), shi = S ? ub + S : 0u;
        if (merge) {
            slo = (slo + 15u) & ~15u;
            if (lane != 63u)
                shi &= ~15u;
        }
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
            const uint32_t f = 16u * j + (lane >> 2);
            sa[j] = shfl_u64(Gb, f) + srel;
            sro[j] = kStRing * f;
            slo4[j] = (uint32_t) __shfl((int) slo, (int) f);
            shi4[j] = (uint32_t) __shfl((int) shi, (int) f);
            ssh4[j] = __shfl(sh, (int) f);
        }
    }
    // window t's input cover -> input buffer t & 1 (no wait)
    const uint32_t wlds_off =
        __builtin_amdgcn_readfirstlane((uint32_t) (uintptr_t) (StLdsVoid *) wlds); // the wave's LDS byte offset
    auto dma = [&](uint32_t t) {
        const uint32_t b = wlds_off + (kStNIn == 2 ? (t & 1u) * kStInBuf : 0u);
#pragma unroll
        for (uint32_t j = 0; j < 5; ++j)
            if (64u * t + lrel[j] < llim[j])
                lds_dma16(la[j] + 64ull * t, b + 1024u * j);
    };
    // window t's output granules from the ring: the four reads first, then
    // the whole granules, then (rarely, a wave-uniform branch) the partial ones
    // piece t's granules (ring-relative 64t + sh + 16 (lane % 4)); a piece
    // before the frame's first byte (t = 0 with sh < 0) stores nothing
    auto ring_get = [&](uint32_t t, u32x4 (&g)[4]) {
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
            const int32_t r = (int32_t) (64u * t + srel) + ssh4[j];
            g[j] = *(const u32x4 *) (ring + sro[j] + ((uint32_t) r & 127u));
        }
    };
    auto ring_store = [&](uint32_t t, const u32x4 (&g)[4]) {
        uint32_t partm = 0;
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
            const int32_t rs = (int32_t) (64u * t + srel) + ssh4[j];
            const uint32_t r = (uint32_t) rs;
            const bool in = rs >= 0;
            const bool full = in && r >= slo4[j] && r + 16u <= shi4[j];
            const bool part = in && !full && r < shi4[j] && r + 16u > slo4[j];
            if (full)
                *(GU4 *) (uintptr_t) (sa[j] + (int64_t) (64 * (int32_t) t + ssh4[j])) = g[j];
            partm |= part ? 1u << j : 0u;
        }
        if (!(ZMQG_FRAMES_ABLATE & 512) && __builtin_amdgcn_ballot_w64(partm != 0) != 0) {
#pragma unroll
            for (uint32_t j = 0; j < 4; ++j)
                if ((partm >> j) & 1u) {
                    const uint32_t r = (uint32_t) ((int32_t) (64u * t + srel) + ssh4[j]);
                    granule_store_part(sa[j] + (int64_t) (64 * (int32_t) t + ssh4[j]), slo4[j] > r ? slo4[j] - r : 0u,
                                       shi4[j] - r < 16u ? shi4[j] - r : 16u, g[j]);
                }
        }
    };
    auto store_window_t = [&](uint32_t t) {
        u32x4 g[4];
        ring_get(t, g);
        ring_store(t, g);
    };
    auto ring_spill = [&]() {
        u32x4 o[kStSector / 16];
#pragma unroll
        for (uint32_t q = 0; q < kStSector / 16; ++q)
            o[q] = *(const u32x4 *) (myring + 128 + 16 * q);
#pragma unroll
        for (uint32_t q = 0; q < kStSector / 16; ++q)
            *(u32x4 *) (myring + 16 * q) = o[q];
    };
    // window t's output bytes y -> the ring
    auto ring_put = [&](uint32_t t, const uint32_t y[16]) {
        if ((t & 1u) == 0 && t > 0) // the odd window before: its bytes beyond 128 -> [0, kStSector)
            ring_spill();
        uint8_t *const p = myring + 64u * (t & 1u) + ub;
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q)
            *(u32x4_u1 *) (p + 16u * q) = (u32x4){y[4 * q], y[4 * q + 1], y[4 * q + 2], y[4 * q + 3]};
    };
    if (steps > 1)
        dma(1u);

    SEQ_STAMP(1u);
    LDS_PRIO(LDS_PRIO_KS);
    // ---- step 0: window 0 (Poly1305 key, first 32 ciphertext bytes, header)
    PolyKey32 pk;
    Poly32 h = {0, 0, 0, 0, 0};
    uint32_t spad[4], wtag[4] = {0, 0, 0, 0}, fl = 0;
    uint32_t cp[16];                // ciphertext of the window whose MAC is absorbed next step
    uint32_t cp_j0 = 2, cp_len = 0; // its first block slot and ciphertext bytes
    uint32_t ct0[4];                // merged encode: ciphertext bytes 0..15 (wire 32..47)
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
#pragma unroll
        for (int k = 0; k < 4; ++k)
            ct0[k] = y[8 + k];
        if (DEC)
            fl = y[8] & 3u;
        // stream bytes 0..31 (decode: header/nonce/tag; encode: the Poly1305
        // key) are outside the cooperatively stored range
        ring_put(0u, y);
    }
    SEQ_STAMP(2u);
    call_state_count(zs);

    // ---- steps 1 ..: window t
#pragma unroll 1
    for (uint32_t t = 1; t < steps; ++t) {
        SEQ_STAMP(3u + (t < 20u ? t : 20u));
        // window t's input has landed (and the stores issued a step ago are
        // out of the way); the next window's DMA and the previous window's
        // stores go out before the keystream, so a whole window hides them
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        LDS_PRIO(LDS_PRIO_MEM);
        if (t < 8u)
            SEQ_STAMP(44u + t);
        const bool act = t < nw;
        uint32_t x[16];
        {
            const uint8_t *const p = wlds + (kStNIn == 2 ? (t & 1u) * kStInBuf : 0u) + kStIn * lane + va;
#pragma unroll
            for (uint32_t q = 0; q < 4; ++q) {
                const u32x4 v = *(const u32x4_u1 *) (p + 16u * q);
                x[4 * q] = v.x;
                x[4 * q + 1] = v.y;
                x[4 * q + 2] = v.z;
                x[4 * q + 3] = v.w;
            }
        }
        u32x4 g[4];
        ring_get(t - 1u, g);
        if (kStNIn == 1) // the input buffer is read before the next window's DMA refills it
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (t + 1u < steps)
            dma(t + 1u);
        ring_store(t - 1u, g);
        LDS_PRIO(LDS_PRIO_KS);
        if (t < 8u)
            SEQ_STAMP(52u + t);
        uint32_t ks[16];
        if (ZMQG_FRAMES_ABLATE & 32) {
#pragma unroll
            for (int k = 0; k < 16; ++k)
                ks[k] = key[k & 7] ^ (t * 0x9e3779b9u + k);
        } else {
            salsa20_block(ks, key, n0, n1, t, 0);
        }
        // The previous window's MAC (its ciphertext is in cp), the four-block
        // form for every lane, unconditionally, in the keystream's basic block
        // (see k_frames_seq); lanes whose window was not four full blocks keep
        // h and take the general form below.
        const bool pv = t - 1u < nw;
        const bool full = pv && cp_j0 == 0u && cp_len == 64u;
        {
            Poly32 hf = h;
            if (ZMQG_FRAMES_ABLATE & 64)
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
        if (!(ZMQG_FRAMES_ABLATE & 64) && __builtin_amdgcn_ballot_w64(pv && !full) != 0) {
            if (pv && !full)
                poly32_window(h, pk, cp, cp_j0, cp_len);
        }
        if (t < 12u)
            SEQ_STAMP(24u + t);
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
        ring_put(t, y);
        if (t < 8u)
            SEQ_STAMP(36u + t);
    }
    SEQ_STAMP(60u);
    LDS_PRIO(LDS_PRIO_MEM);
    if (steps > 0) {
        // the last window's granules, and the granules its last ub bytes
        // spill into (odd window: bytes beyond ring byte 128, copied first)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        store_window_t(steps - 1u);
        if ((steps & 1u) == 0)
            ring_spill();
        store_window_t(steps);
        // then the last window's MAC
        if (nw == steps)
            poly32_window(h, pk, cp, cp_j0, cp_len);
    }

    unsigned long long excl = 0;
    if (lb) {
        const unsigned long long P = lookback_excl(wg, epoch, rp.lb_flag, rp.lb_agg, rp.lb_inc);
        if (threadIdx.x == 0) {
            const unsigned long long inc = P > wagg ? P : wagg;
            // (a grid of at most kFramesBS workgroups looks back over every
            // aggregate in one round and needs no inclusive values: no
            // publish, and no drain of this wave's last stores for it)
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
    frame_result_copy<DEC>(big);
    SEQ_STAMP(61u);
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
    if (!DEC && merge) {
        // wire bytes 0..47 ("\x07MESSAGE", nonce, tag, ciphertext 0..15) laid
        // out at the frame's byte offset ub in the granules [G, G + 48)
        const uint32_t o[12] = {0x53454d07u, 0x45474153u, n0,     n1,     tag[0], tag[1],
                                tag[2],      tag[3],      ct0[0], ct0[1], ct0[2], ct0[3]};
        const uint32_t m0 = ub >> 2, sb = ub & 3u;
        uint32_t gw[12];
#pragma unroll
        for (int j = 0; j < 12; ++j) {
            // (compile-time indices for each word shift; ub picks one)
            const uint32_t h0 = o[j], l0 = j >= 1 ? o[j - 1] : 0u;
            const uint32_t h1 = j >= 1 ? o[j - 1] : 0u, l1 = j >= 2 ? o[j - 2] : 0u;
            const uint32_t h2 = j >= 2 ? o[j - 2] : 0u, l2 = j >= 3 ? o[j - 3] : 0u;
            const uint32_t h3 = j >= 3 ? o[j - 3] : 0u, l3 = j >= 4 ? o[j - 4] : 0u;
            const uint32_t hi = m0 == 0 ? h0 : m0 == 1 ? h1 : m0 == 2 ? h2 : h3;
            const uint32_t lo = m0 == 0 ? l0 : m0 == 1 ? l1 : m0 == 2 ? l2 : l3;
            gw[j] = sb == 0 ? hi : __builtin_amdgcn_alignbyte(hi, lo, 4u - sb);
        }
        const uint64_t G = B - ub;
        u32x4 g0 = {gw[0], gw[1], gw[2], gw[3]};
        if (ub != 0 && lane != 0) {
            // the granule's first ub bytes: the end of the lane before's frame,
            // in its ring at that frame's granule (pend >> 4) mod 8
            const u32x4 pg = *(const u32x4 *) (ring + kStRing * (lane - 1u) + 16u * ((pend >> 4) & 7u));
            const uint32_t pw[4] = {pg.x, pg.y, pg.z, pg.w};
            uint32_t mw[4];
#pragma unroll
            for (uint32_t j = 0; j < 4; ++j) {
                const int nb = (int) ub - 4 * (int) j; // bytes of word j from the lane before
                const uint32_t mask = nb >= 4 ? 0xffffffffu : nb <= 0 ? 0u : (1u << (8 * nb)) - 1u;
                mw[j] = (pw[j] & mask) | (gw[j] & ~mask);
            }
            g0 = (u32x4){mw[0], mw[1], mw[2], mw[3]};
        }
        if (ub == 0 || lane != 0)
            *(GU4 *) (uintptr_t) G = g0;
        else
            granule_store_part(G, ub, 16u, g0);
        *(GU4 *) (uintptr_t) (G + 16u) = (u32x4){gw[4], gw[5], gw[6], gw[7]};
        if (ub != 0)
            *(GU4 *) (uintptr_t) (G + 32u) = (u32x4){gw[8], gw[9], gw[10], gw[11]};
    } else if (!DEC) {
        // "\x07MESSAGE" || nonce || tag: wire bytes 0..31 (the rest went out cooperatively)
        uint32_t o[16] = {0x53454d07u, 0x45474153u, n0, n1, tag[0], tag[1], tag[2], tag[3]};
        if (ZMQG_FRAMES_ABLATE & 1024) { // (timing only: two aligned dwordx4 at the granule below)
            GU4 *q = (GU4 *) (uintptr_t) ((uint64_t) (uintptr_t) dst & ~15ull);
            q[0] = (u32x4){o[0], o[1], o[2], o[3]};
            q[1] = (u32x4){o[4], o[5], o[6], o[7]};
        } else {
            store_bytes_c<32>(dst, o);
        }
    } else {
        if (lb && !(vn > excl))
            status = ZMQG_ERR_INVALID_SEQUENCE; // src/curve_mechanism_base.cpp:99-104 (before the MAC)
        else if ((tag[0] ^ wtag[0]) | (tag[1] ^ wtag[1]) | (tag[2] ^ wtag[2]) | (tag[3] ^ wtag[3]))
            status = ZMQG_ERR_CRYPTOGRAPHIC; // src/curve_mechanism_base.cpp:277-281
        status_out[i] = status;
        flags_out[i] = status == 0 ? (uint8_t) (fl | frame_zbits<DEC>(big, i)) : 0;
        if (status != 0) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); // the wave's stores of this frame first
            zero_bytes(dst, S - 33u);
        }
    }
}

} // namespace zmqg
