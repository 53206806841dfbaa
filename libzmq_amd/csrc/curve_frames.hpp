// curve_frames.hpp -- the frame kernel: whole CURVE MESSAGE frames (encode or
// decode) in one pass, G lanes per frame.
//
// Reference: src/curve_mechanism_base.cpp:111-205 (encode) and :207-284
// (decode, with check_validity :80-109 and mechanism_base.cpp:14-25), i.e.
// libsodium 1.0.18 crypto_box_easy_afternm / crypto_box_open_easy_afternm on
// one frame each.
//
// Stream image.  Stream byte j of a frame is keystream byte j: bytes 0..31
// are the Poly1305 key area, byte 32+p is plaintext byte p.  On the wire,
// stream byte j >= 32 is wire byte j (ciphertext), so encode's output stream
// is the wire frame itself and decode's input stream is the wire frame; the
// plaintext side is offset by the plaintext header (encode: flags byte and
// sub/cancel prefix, src/curve_mechanism_base.cpp:118-164; decode: the flags
// byte, :250-260).  A window is 64 stream bytes = one Salsa20 block = four
// 16-byte Poly1305 blocks of ciphertext (window 0: two, the other two are
// the key area).
//
// Work split.  The G lanes of a frame take windows w = q, q+G, q+2G, ...
// (lane q), so each step a frame's G lanes read and write 64*G contiguous
// bytes.  Lane 0 starts with window 0 (keystream block 0 -> Poly1305 r, s)
// and hands r to its group by a shuffle.  Poly1305 is evaluated in parallel:
// with virtual blocks v = ciphertext block + 2 (two leading zero blocks,
// which do not change the MAC), window w holds v = 4w..4w+3, and for NV
// virtual blocks and L = last window, k = NV - 4L blocks in it,
//     h = sum_{w<L} r^(k + 4(L-1-w)) U_w + U'_L,
//     U_w = sum_j m_{4w+j} r^(4-j),   U'_L = sum_{j<k} m_{4L+j} r^(k-j),
// so lane q keeps H_q = H_q r^(4G) + U_w over its windows below L and scales
// H_q by r^(k + 4(L-1-w_q)) at the end; the group sums the lanes' terms and
// lane 0 finishes the tag (encode: writes it; decode: compares).
//
// Memory.  Loads and stores are 4-byte aligned dwordx4 (aligned 4-byte words
// of arbitrarily aligned frames), shifted in registers with v_alignbyte; an
// output dword straddling two windows is written by the later window, which
// gets the earlier window's last word from the lane that computed it.  Only
// the first output dword of a frame and its tail are byte-exact stores, so
// neighbouring frames are never touched.
#pragma once

#ifndef ZMQG_FRAMES_ABLATE
#define ZMQG_FRAMES_ABLATE 0 // timing/counting experiments only: k_frames: 1 no Poly1305, 2 no stores, 4 no input shift; k_frames_seq: 8 no stores, 16 no loads, 32 no Salsa20, 64 no Poly1305, 128 stores to 64-byte-aligned places (whole lines), 256 loads from 64-byte-aligned places; k_frames_lds: 512 no partial edge granules, 1024 the encode head as two aligned dwordx4
#endif


#ifndef ZMQG_SEQ_STORE
#define ZMQG_SEQ_STORE 0 // k_frames_seq window stores: 0 default policy, 3 sc0 sc1 (experiments)
#endif

// one output dwordx4 of a window (the seq kernel's per-lane stores)
__device__ __forceinline__ void seq_store4(uint64_t a, uint32_t x, uint32_t y, uint32_t z, uint32_t w)
{
    typedef unsigned int v4_ __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(1))) v4_ __attribute__((aligned(4))) G4_;
    if (ZMQG_SEQ_STORE == 3)
        asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1" ::"v"(a), "v"((v4_){x, y, z, w}) : "memory");
    else
        *(G4_ *) (uintptr_t) a = (v4_){x, y, z, w};
}

#ifndef ZMQG_SEQ_LDSIN
#define ZMQG_SEQ_LDSIN 1 // k_frames_seq: each window's input staged by the wave's LDS-DMA one window ahead (1; 0: per-lane loads)
#endif
#ifndef ZMQG_SEQ_COOPST
#define ZMQG_SEQ_COOPST 2 // k_frames_seq decode under ZMQG_OPT_STREAM_OUT, 64-byte-aligned payloads: each step's chunks stored by the wave cooperatively (16 frames x 64 B per instruction) through LDS, a step later (2; 3: at the next step's top) or at once (1); 0: each lane its own always
#endif
#ifndef ZMQG_SEQ_SKIP5
#define ZMQG_SEQ_SKIP5 1 // LDS-DMA input: no fifth granule for 16-byte-aligned frames (k_frames_seq, k_frames_lds)
#endif
#ifndef ZMQG_SEQ_PF
#define ZMQG_SEQ_PF 1 // k_frames_seq: windows requested ahead of the one computed (1; 2 measured slower)
#endif
#ifndef ZMQG_SEQ_AL64
#define ZMQG_SEQ_AL64 1 // k_frames_seq decode: 64-byte payload chunks when every payload of a wave starts 64-byte aligned (0: off, for timing)
#endif

#ifndef ZMQG_FR_BS
#define ZMQG_FR_BS 256 // frame-kernel workgroup size (threads)
#endif

#include "../../include/zmqg_curve.h"
#include "curve_device.hpp"

namespace zmqg {

constexpr uint32_t kFramesBS = ZMQG_FR_BS, kFramesWaves = kFramesBS / 64;
#ifndef ZMQG_SEQ_STAMPS
#define ZMQG_SEQ_STAMPS 0 // diagnostic builds only (tools/seq_stamps.hip): per-wave s_memtime stamps into rp.clk, 64 per wave
#endif

#if ZMQG_SEQ_STAMPS
#define SEQ_STAMP(slot)                                                                            \
    do {                                                                                           \
        if (rp.clk && (threadIdx.x & 63u) == 0 && (slot) < 64u)                                    \
            rp.clk[64ull * (blockIdx.x * kFramesWaves + (threadIdx.x >> 6)) + (slot)] =            \
                __builtin_amdgcn_s_memtime();                                                      \
    } while (0)
#else
#define SEQ_STAMP(slot) do { } while (0)
#endif

struct DevSession {
    uint32_t enc_key[8]; // HSalsa20(precom, enc_prefix)
    uint32_t dec_key[8]; // HSalsa20(precom, dec_prefix)
    uint32_t downgrade_sub;
    uint32_t pad[7];
};

// plaintext header of src/curve_mechanism_base.cpp:118-158 as 3 words
__device__ __forceinline__ uint32_t plaintext_header(uint32_t msg_flags, uint32_t downgrade, uint32_t hw[3])
{
    const uint32_t f = msg_flags & 3u; // more | command
    const uint32_t ct = msg_flags & 0x1c;
    const bool sub = ct == 12u, cancel = ct == 16u;
    hw[1] = hw[2] = 0;
    if (!(sub || cancel)) {
        hw[0] = f;
        return 1;
    }
    if (downgrade) {
        hw[0] = f | ((sub ? 1u : 0u) << 8);
        return 2;
    }
    if (cancel) { // f|2, "\x06CANCEL"
        hw[0] = (f | 2u) | (6u << 8) | ((uint32_t) 'C' << 16) | ((uint32_t) 'A' << 24);
        hw[1] = (uint32_t) 'N' | ((uint32_t) 'C' << 8) | ((uint32_t) 'E' << 16) | ((uint32_t) 'L' << 24);
        return 8;
    }
    // f|2, "\x09SUBSCRIBE"
    hw[0] = (f | 2u) | (9u << 8) | ((uint32_t) 'S' << 16) | ((uint32_t) 'U' << 24);
    hw[1] = (uint32_t) 'B' | ((uint32_t) 'S' << 8) | ((uint32_t) 'C' << 16) | ((uint32_t) 'R' << 24);
    hw[2] = (uint32_t) 'I' | ((uint32_t) 'B' << 8) | ((uint32_t) 'E' << 16);
    return 11;
}

// out[i] = stream bytes of p shifted right by HL bytes (zeros shifted in), 8 words.
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

typedef u32x4 u32x4_a4 __attribute__((aligned(4)));
typedef __attribute__((address_space(1))) const u32x4_a4 GCU4a4;
typedef __attribute__((address_space(1))) u32x4_a4 GU4a4;
typedef __attribute__((address_space(1))) const uint32_t GCU32;

// Raw aligned words for window w of a stream whose byte 0 is at A and whose
// bytes [0, S) may be read: d[k] = the aligned word holding stream byte
// 64w + 4k - (A & 3).  Fast path: four dwordx4 + one dword.  At the stream's
// end only words that hold a stream byte < S are read (such a word never
// crosses into a page the stream does not touch).
__device__ __forceinline__ void frame_load_raw(uint64_t A, uint32_t w, uint32_t S, uint32_t d[17])
{
    const uint32_t v = (uint32_t) A & 3u;
    const uint64_t a4 = (A & ~3ull) + 64ull * w;
    if (64u * w + 68u <= S) {
        const GCU4a4 *p = (const GCU4a4 *) (uintptr_t) a4;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const u32x4 t = p[k];
            d[4 * k] = t.x;
            d[4 * k + 1] = t.y;
            d[4 * k + 2] = t.z;
            d[4 * k + 3] = t.w;
        }
        d[16] = *(GCU32 *) (uintptr_t) (a4 + 64);
    } else {
#pragma unroll
        for (int k = 0; k < 17; ++k)
            d[k] = (64u * w + 4u * k < S + v) ? *(GCU32 *) (uintptr_t) (a4 + 4u * k) : 0u;
    }
}

// Stream words of window w from the raw words (zero at and beyond S).
// The tail mask runs only when some lane of the wave is on its frame's last
// window (a wave-uniform branch): if-converted, its 16 selects per word
// would be paid on every window.
__device__ __forceinline__ void mask_tail_wave(uint32_t x[16], uint32_t w, uint32_t S, bool act)
{
    if (__builtin_amdgcn_ballot_w64(act && S < 64u * w + 64u) != 0) {
        if (S < 64u * w + 64u)
            mask_tail(x, (int) (S - 64u * w));
    }
}

__device__ __forceinline__ void frame_words(const uint32_t d[17], uint32_t v, uint32_t w, uint32_t S, uint32_t x[16],
                                            bool mask, bool act)
{
#pragma unroll
    for (int k = 0; k < 16; ++k)
        x[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], v);
    if (mask)
        mask_tail_wave(x, w, S, act);
}

// Store output stream words y of window w >= 1 (stream byte 0 at B): the 16
// aligned words covering stream [64w - up, 64w + 64 - up), up = B&3 or 4,
// word 0 completed with yprev (word 15 of window w-1); on the frame's last
// window also the tail up to S.  Bytes >= S are never written.
__device__ __forceinline__ void frame_store(uint64_t B, uint32_t w, uint32_t S, const uint32_t y[16], uint32_t yprev,
                                            bool last)
{
    const uint32_t u = (uint32_t) B & 3u, up = u ? u : 4u, sh = 4u - up;
    // (ablation 128, timing only: every window stored whole to a 64-byte-aligned
    // place, so a frame's consecutive windows fill whole 128-byte lines)
    const uint64_t a = (ZMQG_FRAMES_ABLATE & 128) ? ((B + 160ull) & ~127ull) + 64ull * w : B - up + 64ull * w; // aligned
    if (ZMQG_FRAMES_ABLATE & 128) {
        if (a + 64ull > B + S) // (never beyond the frame's own end)
            return;
        S = 0xffffffffu;
        last = false;
    }
    uint32_t o[17];
    o[0] = __builtin_amdgcn_alignbyte(y[0], yprev, sh);
#pragma unroll
    for (int k = 1; k < 16; ++k)
        o[k] = __builtin_amdgcn_alignbyte(y[k], y[k - 1], sh);
    o[16] = __builtin_amdgcn_alignbyte(0u, y[15], sh);
    if (64u * w + 64u <= S) {
#pragma unroll
        for (int k = 0; k < 4; ++k)
            seq_store4(a + 16u * k, o[4 * k], o[4 * k + 1], o[4 * k + 2], o[4 * k + 3]);
        if (last) { // S == 64w + 64: the last `up` bytes
            GU8 *t = (GU8 *) (uintptr_t) (a + 64);
            if (up == 4u) {
                *(GU32 *) t = o[16];
            } else {
#pragma unroll
                for (uint32_t b = 0; b < 3; ++b)
                    if (b < up)
                        t[b] = (uint8_t) (o[16] >> (8 * b));
            }
        }
    } else {
        // the frame's last window: stream bytes [64w - up, S), at most 68
        store_tail(a, S + up - 64u * w, o);
    }
}

// ---------------------------------------------------------------- Poly1305, parallel form
struct fe5 { // an element plus 5x its limbs 1..4 (the reduction multipliers)
    fe e;
    uint32_t s1, s2, s3, s4;
};

__device__ __forceinline__ fe5 fe5_of(const fe &x)
{
    fe5 r;
    r.e = x;
    r.s1 = x.l[1] * 5;
    r.s2 = x.l[2] * 5;
    r.s3 = x.l[3] * 5;
    r.s4 = x.l[4] * 5;
    return r;
}

// a += m * p (m: limbs of a block or an element, p: a power of r)
__device__ __forceinline__ void acc_mul(uint64_t a[5], const uint32_t m[5], const fe5 &p)
{
    const uint32_t p0 = p.e.l[0], p1 = p.e.l[1], p2 = p.e.l[2], p3 = p.e.l[3], p4 = p.e.l[4];
    a[0] = mad64(m[0], p0, mad64(m[1], p.s4, mad64(m[2], p.s3, mad64(m[3], p.s2, mad64(m[4], p.s1, a[0])))));
    a[1] = mad64(m[0], p1, mad64(m[1], p0, mad64(m[2], p.s4, mad64(m[3], p.s3, mad64(m[4], p.s2, a[1])))));
    a[2] = mad64(m[0], p2, mad64(m[1], p1, mad64(m[2], p0, mad64(m[3], p.s4, mad64(m[4], p.s3, a[2])))));
    a[3] = mad64(m[0], p3, mad64(m[1], p2, mad64(m[2], p1, mad64(m[3], p0, mad64(m[4], p.s4, a[3])))));
    a[4] = mad64(m[0], p4, mad64(m[1], p3, mad64(m[2], p2, mad64(m[3], p1, mad64(m[4], p0, a[4])))));
}

// limbs of the 16-byte block in words w[0..3] with the 2^128 bit (full block)
// or, for a partial block of nb < 16 bytes (bytes >= nb already zero), the
// 0x01 pad byte at nb and no 2^128 bit
__device__ __forceinline__ void block_limbs(const uint32_t *w, int nb, uint32_t m[5])
{
    uint32_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3], hib = 1u << 24;
    if (nb < 16) {
        hib = 0;
        const uint32_t pad = 1u << (8 * (nb & 3));
        const int wi = nb >> 2;
        w0 |= wi == 0 ? pad : 0u;
        w1 |= wi == 1 ? pad : 0u;
        w2 |= wi == 2 ? pad : 0u;
        w3 |= wi == 3 ? pad : 0u;
    }
    m[0] = w0 & M26;
    m[1] = __builtin_amdgcn_alignbit(w1, w0, 26) & M26;
    m[2] = __builtin_amdgcn_alignbit(w2, w1, 20) & M26;
    m[3] = __builtin_amdgcn_alignbit(w3, w2, 14) & M26;
    m[4] = (w3 >> 8) | hib;
}

// Replay rule of src/curve_mechanism_base.cpp:98-106 in the decode frame
// kernel.  Per frame: the header-valid nonce vout (0 for a header failure)
// and the session's peer nonce before the batch (psnap).
//   One session (lb_flag != null): workgroups take their frames in ticket
//   order and run a decoupled look-back over the workgroup maxima of vout,
//   so each frame knows excl = max of every earlier header-valid nonce in
//   the batch; small frames apply the rule here, big frames get excl for
//   the body's finisher, and the last workgroup writes the new peer nonce.
//   Several sessions (lb_flag == null): iota for the sort-by-session path;
//   the rule is applied by k_fixup / the body finisher.
struct ReplayOut {
    unsigned long long *vout;
    unsigned long long *psnap;
    uint32_t *iota;
    unsigned long long *peer; // read (psnap); one session: written by the last workgroup
    unsigned long long *excl; // one session: per frame, for the body finisher
    unsigned long long *lb_flag, *lb_agg, *lb_inc; // one session: look-back state per ticket
    uint32_t ordered;         // 1: the whole grid is co-resident, so workgroups use blockIdx as
                              //    their look-back order (no ticket)
    uint32_t dbg;             // timing experiments only (tools/frames_bench): 1 no look-back, 2 no ticket
    unsigned long long *clk;  // diagnostics only: per workgroup {start, end} s_memrealtime, memtime delta, hw ids
    unsigned long long *smax; // one session, optional: the batch's largest header-valid nonce (last workgroup)
};

// Per-context device state that carries from one batch call to the next,
// kept on the device so that a captured hipGraph of calls replays correctly:
// the call epoch (look-back flags of older calls are stale; parity selects
// the big-frame list counter), the workgroup ticket and done counters (the
// last workgroup to finish resets them and advances the epoch).
struct ZState {
    uint32_t epoch;  // >= 1
    uint32_t ticket;
    uint32_t done;
    uint32_t pad;
    unsigned long long list_ctr[2]; // big frames << 40 | body chunks, by epoch parity
    uint32_t post_n;                // decode: entries in the post list (k_post resets it)
    uint32_t post_done;             // k_post: workgroups finished
};

// Decode work after the body kernel (k_post, zmqg_curve.hip): zero-fill a
// failed frame's region, or move an in-place frame's payload from where the
// body wrote it (wire offset 33) to the frame's start (dst = src - 33).
constexpr uint32_t kPostZero = 0, kPostMove = 1;
struct PostOp {
    uint64_t dst;
    uint64_t len;
    uint32_t kind;
    uint32_t p; // move: the frame's big-list position (its scratch for the segment seams)
};

__device__ __forceinline__ void post_append(ZState *zs, PostOp *post, uint64_t dst, uint64_t len, uint32_t kind,
                                            uint32_t p)
{
    const uint32_t e = __hip_atomic_fetch_add(&zs->post_n, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    PostOp o;
    o.dst = dst;
    o.len = len;
    o.kind = kind;
    o.p = p;
    post[e] = o;
}

// Per-call options of the frame kernels (zmqg_batch_opts, include/zmqg_curve.h).
struct FrameCtl {
    int32_t *enc_status; // encode: per-frame 0 / ZMQG_ERR_SESSION / ZMQG_ERR_BOUND (optional)
    PostOp *post;        // decode: header-failed frames too long for one lane to zero-fill
    uint64_t max_len;    // 0, or the caller's bound on len / wire_len
    uint32_t no_body;    // 1: no body kernel follows (every frame within max_len fits this kernel)
    uint32_t out_check;  // decode, ZMQG_OPT_VERIFY_FIRST: payload regions must end within out_limit
    unsigned long long *nonce_ctr; // encode, one session, ZMQG_OPT_NONCE_AUTO: the session's send
                                   // counter; frame i takes *nonce_ctr + i, the last workgroup adds n
    uint64_t out_limit;  // (out_check) the caller's out_bytes: the staging area's extent
    // k_frames_split: workgroups [0, split_wg) run the one-lane-per-frame body
    // on frames [0, split_n) (split_n = split_wg x kFramesBS), the rest run the
    // G-lanes-per-frame body on frames [split_n, n); 0 in every other launch
    uint32_t split_wg, split_n;
    uint32_t stream_out; // decode, ZMQG_OPT_STREAM_OUT (host side: picks k_frames_seq's SO instantiation)
};

// msg_t flags a received ZMTP frame adds to its decoded message: the
// decoder's MORE / COMMAND (src/v2_decoder.cpp:35-41) ORed into the
// plaintext's by set_flags (src/msg.cpp:433-436); 0 without zflags.
__device__ __forceinline__ uint32_t zmtp_msg_bits(const uint8_t *zflags, uint32_t i)
{
    if (!zflags)
        return 0u;
    const uint32_t z = zflags[i];
    return (z & 1u) | ((z & 4u) ? 2u : 0u); // ZMTP MORE (1) / COMMAND (4) -> msg_t more (1) / command (2)
}

// zmqg_decode_zmtp's two additions to a decode, carried by the decode's
// BigOp (DecodeHead: zflags, res_src, res_dst) so that the encode kernels do
// not change: the frames' ZMTP flag bits, and the call's result copied from
// the parse state by one thread of workgroup 0.
template <bool DEC, class BigOp>
__device__ __forceinline__ uint32_t frame_zbits(const BigOp &big, uint32_t i)
{
    if constexpr (DEC)
        return zmtp_msg_bits(big.zflags, i);
    else
        return 0u;
}

template <bool DEC, class BigOp>
__device__ __forceinline__ void frame_result_copy(const BigOp &big)
{
    if constexpr (DEC) {
        if (blockIdx.x == 0 && threadIdx.x == 0 && big.res_src)
            for (int k = 0; k < 4; ++k)
                big.res_dst[k] = big.res_src[k];
    }
}

// A frame the call must not process (status ZMQG_ERR_BOUND, nothing
// written): above the caller's max_len, or -- decode under
// ZMQG_OPT_VERIFY_FIRST, whose staging area is sized from out_bytes -- a
// payload region reaching past out_bytes.
template <bool DEC>
__device__ __forceinline__ bool frame_over(const FrameCtl &ctl, uint32_t L_in, uint64_t ooff)
{
    const bool over_len = ctl.max_len != 0 && L_in > ctl.max_len;
    if (!DEC)
        return over_len;
    return over_len || (ctl.out_check && L_in > 33u && ooff + (L_in - 33u) > ctl.out_limit);
}

// Encode nonce of frame i: the caller's, or (ZMQG_OPT_NONCE_AUTO, one
// session) the send counter read at kernel start plus i, as n calls of
// curve_encoding_t::get_and_inc_nonce (src/curve_mechanism_base.hpp:41) would
// assign them.
__device__ __forceinline__ uint64_t frame_nonce(const uint64_t *nonce, const FrameCtl &ctl, uint64_t nbase,
                                                uint32_t i)
{
    return ctl.nonce_ctr ? nbase + i : nonce[i];
}

__device__ __forceinline__ uint64_t nonce_base(const FrameCtl &ctl)
{
    return ctl.nonce_ctr ? __hip_atomic_load(ctl.nonce_ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
}

// A frame kernel's view of the call state (ZState), taken by thread 0 of
// each workgroup at its start: the epoch, its look-back ticket (ticket:
// true) and the encode nonce base.  Once these reads have been used (after
// its first window) the workgroup counts itself in zs->done with a
// fire-and-forget atomic (call_state_count); workgroup 0, at its end, waits
// for the count to reach the grid and then resets the counters and advances
// the epoch and the send counter for the next call (call_state_end: every
// other workgroup has read them by then; the next call is stream-ordered
// after this one; nothing in this launch reads them after its start).  So no
// workgroup waits on a returning device-scope atomic: round 1 counted at
// every workgroup's end with one (a round trip on each exit path), and
// counting at the start with one serialised the whole grid's first
// workgroups behind 256 atomics on one address (tools/seq_stamps.hip).
// Workgroup 0 is dispatched first, so the count is normally complete when
// it looks, and its one extra load falls inside the other workgroups' time.
struct CallState {
    uint32_t epoch, ticket;
    uint64_t nbase;
};

template <bool DEC>
__device__ __forceinline__ CallState call_state_begin(ZState *zs, const FrameCtl &ctl, bool ticket)
{
    __shared__ CallState sh_cs;
    if (threadIdx.x == 0) {
        CallState c;
        c.epoch = __hip_atomic_load(&zs->epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        c.ticket = ticket ? atomicAdd(&zs->ticket, 1u) : 0u;
        c.nbase = DEC ? 0ull : nonce_base(ctl);
        sh_cs = c;
    }
    __syncthreads();
    return sh_cs;
}

// (called once the CallState values have been used, so its reads are done)
__device__ __forceinline__ void call_state_count(ZState *zs)
{
    if (threadIdx.x == 0)
        (void) __hip_atomic_fetch_add(&zs->done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <bool DEC>
__device__ __forceinline__ void call_state_end(ZState *zs, const FrameCtl &ctl, const CallState &c, uint32_t n)
{
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        while (__hip_atomic_load(&zs->done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < gridDim.x)
            __builtin_amdgcn_s_sleep(2);
        __hip_atomic_store(&zs->done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&zs->ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&zs->epoch, c.epoch + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (!DEC && ctl.nonce_ctr)
            __hip_atomic_store(ctl.nonce_ctr, c.nbase + n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// Frames whose region a failing lane zero-fills itself; longer ones go to
// the post list (k_post spreads them over the whole grid).
constexpr uint32_t kLaneFillMax = 4608;

// Decoupled look-back, whole workgroup: maximum of the aggregates of every
// workgroup ticket < t, reading kFramesBS tickets per round (one per thread) and
// stopping at the nearest one that has published its inclusive value.
// Every earlier ticket has started (tickets are taken at workgroup start)
// and publishes its aggregate right after its header pass, so the spin is
// short; run right after this workgroup's own header pass, so inclusive
// values appear in ticket order early in the kernel.
__device__ __forceinline__ unsigned long long lookback_excl(uint32_t t, uint32_t epoch,
                                                            const unsigned long long *lb_flag,
                                                            const unsigned long long *lb_agg,
                                                            const unsigned long long *lb_inc)
{
    __shared__ uint32_t sh_stop[kFramesWaves];
    __shared__ unsigned long long sh_v[kFramesWaves];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
    unsigned long long P = 0;
    for (int base = (int) t; base > 0; base -= (int) kFramesBS) {
        const int k = base - 1 - (int) tid; // this thread's predecessor
        int state = 2;                      // out of range: an inclusive zero
        if (k >= 0) {
            unsigned long long f;
            do {
                f = __hip_atomic_load(lb_flag + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } while ((uint32_t) (f >> 2) != epoch || (f & 3ull) == 0);
            state = (int) (f & 3ull);
        }
        unsigned long long v = 0;
        if (k >= 0)
            v = __hip_atomic_load((state == 2 ? lb_inc : lb_agg) + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long m = __ballot(state == 2);
        if (lane == 0)
            sh_stop[wv] = m ? 64u * wv + (uint32_t) __builtin_ctzll(m) : kFramesBS;
        __syncthreads();
        uint32_t stop = kFramesBS;
        for (uint32_t w = 0; w < kFramesWaves; ++w)
            stop = sh_stop[w] < stop ? sh_stop[w] : stop;
        if (tid > stop)
            v = 0;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            const unsigned long long o = __shfl_xor(v, d);
            v = o > v ? o : v;
        }
        if (lane == 0)
            sh_v[wv] = v;
        __syncthreads();
        for (uint32_t w = 0; w < kFramesWaves; ++w)
            P = sh_v[w] > P ? sh_v[w] : P;
        __syncthreads();
        if (stop < kFramesBS)
            break;
    }
    return P;
}

// Hand-off without fences (MI355X_MICROARCH.md, "Valid forms": write-through
// sc1 stores drained by s_waitcnt vmcnt(0) before the flag, sc1 loads on the
// reading side).  An agent-scope release would write back the whole XCD L2,
// full of this kernel's output: tens of microseconds per workgroup.
__device__ __forceinline__ void lookback_publish(unsigned long long *flag, unsigned long long *val,
                                                 unsigned long long v, uint32_t epoch, uint32_t state)
{
    __hip_atomic_store(val, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(flag, ((unsigned long long) epoch << 2) | state, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Decode result of a frame whose stream was not processed (header failure,
// unknown session, broken bound): status, flags 0, and the payload region
// zero-filled -- by this lane up to kLaneFillMax bytes, above that by k_post
// over the whole grid (a forged 16 MiB header must not cost one lane 16 MiB
// of stores).  A frame above the caller's bound is left as it was.
__device__ __forceinline__ void fail_unprocessed(int32_t status, uint32_t L_in, uint8_t *dst, uint8_t *flags_out,
                                                 int32_t *status_out, ZState *zs, const FrameCtl &ctl)
{
    *status_out = status;
    *flags_out = 0;
    if (status == ZMQG_ERR_BOUND || L_in < 33u)
        return;
    if (L_in - 33u <= kLaneFillMax || ctl.post == nullptr)
        zero_bytes(dst, L_in - 33u);
    else
        post_append(zs, ctl.post, (uint64_t) (uintptr_t) dst, L_in - 33u, kPostZero, 0);
}

// No big-frame handler (tools, tests): frames above max_stream are skipped.
struct NoBigFrames {
    __device__ void operator()(uint32_t, unsigned long long *, uint64_t) const {}
};

// Frame kernel.  DEC = decode.  Frames whose stream is longer than
// max_stream (with a valid header, for decode) are handed to
// `big(i, list_ctr)` on one lane (the chunked path's head: block 0, records,
// an entry in this call's big-frame list).
// zs: the context's call state (see ZState); decode with rp.lb_flag set
// applies the one-session replay rule in this kernel.
#define ZMQG_FRAMES_PARAMS                                                                                    \
    uint32_t n, const uint32_t *__restrict__ sid, const uint64_t *__restrict__ nonce,                             \
        const uint8_t *__restrict__ flags, const uint64_t *__restrict__ in_off, const uint32_t *__restrict__ len, \
        const uint8_t *__restrict__ in, const uint64_t *__restrict__ out_off, uint8_t *__restrict__ out,          \
        const DevSession *__restrict__ sessions, uint32_t max_sessions, uint32_t max_stream,                      \
        uint8_t *__restrict__ flags_out, int32_t *__restrict__ status_out, ReplayOut rp, BigOp big,               \
        ZState *__restrict__ zs, FrameCtl ctl
#define ZMQG_FRAMES_ARGS                                                                                      \
    n, sid, nonce, flags, in_off, len, in, out_off, out, sessions, max_sessions, max_stream, flags_out,           \
        status_out, rp, big, zs, ctl

// (the body of k_frames<G>; in a k_frames_split launch its workgroups are
// those from ctl.split_wg on and its frames those from ctl.split_n on)
template <bool DEC, int G, class BigOp>
__device__ __forceinline__ void frames_g_impl(ZMQG_FRAMES_PARAMS)
{
    static_assert(G == 1 || G == 2 || G == 4 || G == 8, "lanes per frame");
    const bool lb = DEC && rp.lb_flag != nullptr;
    unsigned long long clk0 = 0, rclk0 = 0;
    if (rp.clk) {
        clk0 = __builtin_amdgcn_s_memtime();
        rclk0 = __builtin_amdgcn_s_memrealtime();
    }
    __shared__ unsigned long long sh_wmax[kFramesWaves];
    const bool use_ticket = lb && !rp.ordered && !(rp.dbg & 2);
    const CallState cs = call_state_begin<DEC>(zs, ctl, use_ticket);
    const uint32_t epoch = cs.epoch;
    const uint32_t wg = use_ticket ? cs.ticket : blockIdx.x;
    const uint64_t nbase = cs.nbase;
    unsigned long long *const list_ctr = zs->list_ctr + (epoch & 1u);
    if (blockIdx.x == 0 && threadIdx.x == 0)
        zs->list_ctr[(epoch & 1u) ^ 1u] = 0; // the next call's list (the previous body has finished with it)
    const uint32_t gl = (wg - ctl.split_wg) * kFramesBS + threadIdx.x;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t i = ctl.split_n + gl / G, q = gl % G;
    const uint32_t gbase = lane - q; // the group's lane 0
    const bool valid = i < n;
    const uint32_t ii = valid ? i : n - 1;
    const bool sid_ok = sid[ii] < max_sessions;
    const uint32_t s = sid_ok ? sid[ii] : 0u; // (a frame of an unknown session is not processed)
    const DevSession &ses = sessions[s];
    uint32_t key[8];
#pragma unroll
    for (int t = 0; t < 8; ++t)
        key[t] = DEC ? ses.dec_key[t] : ses.enc_key[t];
    const uint8_t *src = in + in_off[ii];
    uint8_t *dst = out + out_off[ii];
    const uint32_t L_in = len[ii];
    const bool over = frame_over<DEC>(ctl, L_in, out_off[ii]); // the caller's bounds broken

    uint32_t S = 0, n0 = 0, n1 = 0, hl = 1;
    uint64_t A = 0, B = 0;
    int32_t status = 0;
    uint32_t hw[3] = {0, 0, 0};
    if (!DEC) {
        const uint64_t nc = frame_nonce(nonce, ctl, nbase, ii);
        n0 = bswap32((uint32_t) (nc >> 32));
        n1 = bswap32((uint32_t) nc);
        hl = plaintext_header(flags[ii], ses.downgrade_sub, hw);
        S = sid_ok && !over ? 32u + hl + L_in : 0u;
        A = (uint64_t) (uintptr_t) src - 32u - hl;
        B = (uint64_t) (uintptr_t) dst;
    } else {
        // mechanism_base.cpp:14-25, curve_mechanism_base.cpp:80-97
        uint32_t h16[16];
        load_window(src, L_in < 16u ? (int) L_in : 16, h16);
        const uint32_t b0 = h16[0] & 0xffu;
        if (L_in <= 1u || L_in <= b0)
            status = ZMQG_ERR_MALFORMED_UNSPECIFIED;
        else if (L_in < 8u || h16[0] != 0x53454d07u || h16[1] != 0x45474153u)
            status = ZMQG_ERR_UNEXPECTED_COMMAND;
        else if (L_in < 33u)
            status = ZMQG_ERR_MALFORMED_MESSAGE;
        if (!sid_ok)
            status = ZMQG_ERR_SESSION;
        if (over)
            status = ZMQG_ERR_BOUND;
        n0 = h16[2];
        n1 = h16[3];
        S = status == 0 ? L_in : 0u;
        A = (uint64_t) (uintptr_t) src;
        B = (uint64_t) (uintptr_t) dst - 33u;
    }
    const bool small = valid && S <= max_stream;
    // decode replay bookkeeping: header-valid nonce (0 = not a candidate),
    // its exclusive max-scan inside the workgroup (frame order = thread
    // order), the workgroup aggregate published for the look-back
    unsigned long long vn = 0, wexcl = 0, psn = 0, wagg = 0;
    if (DEC) {
        vn = valid && q == 0 && status == 0 ? (((unsigned long long) bswap32(n0) << 32) | bswap32(n1)) : 0ull;
        psn = rp.peer[s];
        if (valid && q == 0 && !lb) { // (several sessions: the replay tables' input)
            rp.vout[i] = vn;
            rp.psnap[i] = psn;
            if (rp.iota)
                rp.iota[i] = i;
        }
        if (lb) {
            unsigned long long sc = vn;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const unsigned long long o = __shfl_up(sc, d);
                if ((int) lane >= d)
                    sc = o > sc ? o : sc;
            }
            const unsigned long long up = __shfl_up(sc, 1);
            if (lane == 63)
                sh_wmax[threadIdx.x >> 6] = sc;
            __syncthreads();
            const uint32_t wv = threadIdx.x >> 6;
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
        S = 0; // nothing for this lane
    const uint32_t nw = (S + 63u) >> 6;
    const uint32_t L = nw ? nw - 1 : 0;
    const uint32_t kb = nw ? ((S - 64u * L + 15u) >> 4) : 0; // virtual blocks in the last window
    // steps: the wave walks the maximum over its frames
    uint32_t nst = (nw + G - 1 - q) / G; // this lane's windows
    uint32_t mx = nst;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const uint32_t o = __shfl_xor(mx, d);
        mx = o > mx ? o : mx;
    }
    const uint32_t steps = __builtin_amdgcn_readfirstlane(mx);

    const uint32_t vin = (uint32_t) A & 3u;
    fe5 P1, P2, P3, P4, PG; // r^1..r^4, r^(4G)
    uint32_t spad[4] = {0, 0, 0, 0}, wtag[4] = {0, 0, 0, 0}, fl = 0;
    uint64_t H[5] = {0, 0, 0, 0, 0};
    uint32_t tot[5] = {0, 0, 0, 0, 0}; // this lane's share of h
    bool hasH = false;
    uint32_t lastH = 0; // window index of the lane's last window below L
    uint32_t ycarry = 0; // word 15 of window (this lane's window - 1), for q == 0
    uint32_t dn[17]; // raw input words of this lane's next window, loaded a step ahead
    if (nst > 0 && !(q == 0 && !DEC)) // encode's window 0 reads the payload itself
        frame_load_raw(A, q, S, dn);
    call_state_count(zs);

#pragma unroll 1
    for (uint32_t t = 0; t < steps; ++t) {
        // Progress-based issue priority: the two waves on a SIMD share its
        // VALU, which favours the older wave; a wave that is ahead drops its
        // priority so both finish together instead of the younger one
        // running its last third alone (latency-bound).
        if (4 * t < steps)
            __builtin_amdgcn_s_setprio(3);
        else if (2 * t < steps)
            __builtin_amdgcn_s_setprio(2);
        else if (4 * t < 3 * steps)
            __builtin_amdgcn_s_setprio(1);
        else
            __builtin_amdgcn_s_setprio(0);
        const uint32_t w = t * G + q;
        const bool act = w < nw;
        // the keystream first: it needs no input, so the wait for this
        // step's words (and, vmcnt being in order, for the previous step's
        // stores issued after them) comes after ~1000 instructions of Salsa20.
        // (Its counter-free first-round steps are loop-invariant: the
        // compiler hoists them, so they are computed once per lane.)
        uint32_t ks[16];
        salsa20_block(ks, key, n0, n1, w, 0);
        uint32_t dc[17];
#pragma unroll
        for (int k = 0; k < 17; ++k)
            dc[k] = dn[k];
        if (w + G < nw)
            frame_load_raw(A, w + G, S, dn);
        uint32_t x[16];
        if (!DEC && w == 0) {
            // plaintext bytes 0..31 = header || payload[0 .. 32-hl)
            uint32_t pw16[16];
            load_window(src, L_in < 32u ? (int) L_in : 32, pw16);
            uint32_t pt[8];
            switch (hl) {
            case 1: shift_in<1>(pw16, pt); break;
            case 2: shift_in<2>(pw16, pt); break;
            case 8: shift_in<8>(pw16, pt); break;
            default: shift_in<11>(pw16, pt); break;
            }
            pt[0] |= hw[0];
            pt[1] |= hw[1];
            pt[2] |= hw[2];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                x[k] = 0;
                x[8 + k] = pt[k];
            }
            if (S < 64u)
                mask_tail(x, (int) S);
        } else {
            if (ZMQG_FRAMES_ABLATE & 4) {
#pragma unroll
                for (int k = 0; k < 16; ++k)
                    x[k] = dc[k];
            } else {
                frame_words(dc, vin, w, S, x, DEC, act); // encode masks the ciphertext instead
            }
        }
        // r from keystream block 0 (lane 0 of the group) to the group
        if (t == 0) {
            const fe r0 = poly_r_from_key(ks[0], ks[1], ks[2], ks[3]);
            fe r;
#pragma unroll
            for (int k = 0; k < 5; ++k)
                r.l[k] = (uint32_t) __shfl((int) r0.l[k], (int) gbase);
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
#pragma unroll
            for (int k = 1; k < G; k <<= 1)
                fe_mul(tg, tg); // r^(4G) by squaring (G = 1, 2, 4)
            PG = fe5_of(tg);
            if (w == 0) {
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    spad[k] = ks[4 + k];
            }
        }
        // ciphertext words c (the Poly1305 input) and output words y
        uint32_t c[16], y[16];
        if (DEC) {
            // y beyond S is never stored (frame_store and window 0's
            // store_window are byte-exact), so only the MAC input is masked
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                c[k] = x[k];
                y[k] = x[k] ^ ks[k];
            }
        } else {
#pragma unroll
            for (int k = 0; k < 16; ++k)
                c[k] = x[k] ^ ks[k];
            mask_tail_wave(c, w, S, act);
#pragma unroll
            for (int k = 0; k < 16; ++k)
                y[k] = c[k];
        }
        if (w == 0) {
#pragma unroll
            for (int k = 0; k < 8; ++k)
                c[k] = 0; // key area: not ciphertext
        }
        if (act) {
            // Poly1305 contribution of this window
            if (ZMQG_FRAMES_ABLATE & 1) {
                if (w < L) {
                    H[0] ^= c[0] ^ c[7] ^ c[13];
                    hasH = true;
                    lastH = w;
                }
            } else if (w < L) {
                uint64_t a[5];
                if (hasH) {
#pragma unroll
                    for (int k = 0; k < 5; ++k)
                        a[k] = 0;
                    uint32_t hh[5];
                    const fe hf = fe_from_wide(H);
#pragma unroll
                    for (int k = 0; k < 5; ++k)
                        hh[k] = hf.l[k];
                    acc_mul(a, hh, PG);
                } else {
#pragma unroll
                    for (int k = 0; k < 5; ++k)
                        a[k] = 0;
                }
                uint32_t m[5];
                if (w > 0) {
                    block_limbs(c, 16, m);
                    acc_mul(a, m, P4);
                    block_limbs(c + 4, 16, m);
                    acc_mul(a, m, P3);
                }
                block_limbs(c + 8, 16, m);
                acc_mul(a, m, P2);
                block_limbs(c + 12, 16, m);
                acc_mul(a, m, P1);
#pragma unroll
                for (int k = 0; k < 5; ++k)
                    H[k] = a[k];
                hasH = true;
                lastH = w;
            } else {
                // w == L: U'_L = sum_{j<kb} m_j r^(kb-j); window 0's j < 2 are zero
                uint64_t a[5] = {0, 0, 0, 0, 0};
                const int rem = (int) (S - 64u * w); // stream bytes in this window
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    if (j < (int) kb && !(w == 0 && j < 2)) {
                        uint32_t m[5];
                        const int nb = rem - 16 * j >= 16 ? 16 : rem - 16 * j;
                        block_limbs(c + 4 * j, nb, m);
                        const int e = (int) kb - j; // 1..4
                        const fe5 pe = e == 1 ? P1 : e == 2 ? P2 : e == 3 ? P3 : P4;
                        acc_mul(a, m, pe);
                    }
                }
                const fe u = fe_from_wide(a);
#pragma unroll
                for (int k = 0; k < 5; ++k)
                    tot[k] += u.l[k];
            }
        }
        // window 0's extra outputs and state
        if (w == 0 && act) {
            if (DEC) {
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    wtag[k] = x[4 + k];
                fl = y[8] & 3u;
                // payload bytes 0 .. min(31, S-33) = plaintext bytes 1..
                uint32_t pay[16];
#pragma unroll
                for (int k = 0; k < 7; ++k)
                    pay[k] = __builtin_amdgcn_alignbyte(y[9 + k], y[8 + k], 1);
                pay[7] = __builtin_amdgcn_alignbyte(0u, y[15], 1);
#pragma unroll
                for (int k = 8; k < 16; ++k)
                    pay[k] = 0;
                const int np = (int) (S < 64u ? S : 64u) - 33;
                store_window(dst, np, pay);
            } else {
                uint32_t o[16];
                o[0] = 0x53454d07u; // "\x07MESSAGE" || nonce
                o[1] = 0x45474153u;
                o[2] = n0;
                o[3] = n1;
#pragma unroll
                for (int k = 4; k < 16; ++k)
                    o[k] = 0;
                store_bytes_c<16>(dst, o);
                const int nc = (int) (S < 64u ? S : 64u) - 32;
                uint32_t ct[16];
#pragma unroll
                for (int k = 0; k < 16; ++k)
                    ct[k] = k < 8 ? y[8 + k] : 0u;
                store_window(dst + 32, nc, ct);
            }
        }
        // the previous window's last output word: lane q-1 of this step, or
        // (q == 0) lane G-1 of the previous step
        const uint32_t y15 = act ? y[15] : 0u;
        const uint32_t fromleft = (uint32_t) __shfl((int) y15, (int) (lane > 0 ? lane - 1 : 0));
        const uint32_t yprev = q == 0 ? ycarry : fromleft;
        if (act && w > 0) {
            if (!(ZMQG_FRAMES_ABLATE & 2))
                frame_store(B, w, S, y, yprev, w == L);
            else
                *(GU32 *) (uintptr_t) (B + 64ull * w) = y[0] ^ y[5] ^ y[9] ^ y[15] ^ yprev;
        }
        ycarry = (uint32_t) __shfl((int) y15, (int) (gbase + G - 1));
    }
    // H_q * r^(kb + 4(L-1-lastH)), plus U'_L (already in tot)
    if (hasH) {
        fe e;
        const uint32_t m4 = L - 1 - lastH; // 0 .. G-1
        const fe5 pk = kb == 1 ? P1 : kb == 2 ? P2 : kb == 3 ? P3 : P4;
        fe hf = fe_from_wide(H);
        fe_mul_s(hf, pk.e, pk.s1, pk.s2, pk.s3, pk.s4);
        e = hf;
        for (uint32_t k = 0; k < m4; ++k) // at most G-1 times
            fe_mul_s(e, P4.e, P4.s1, P4.s2, P4.s3, P4.s4);
#pragma unroll
        for (int k = 0; k < 5; ++k)
            tot[k] += e.l[k];
    }
#pragma unroll
    for (int d = 1; d < G; d <<= 1)
#pragma unroll
        for (int k = 0; k < 5; ++k)
            tot[k] += (uint32_t) __shfl_xor((int) tot[k], d);
    // replay: this workgroup's exclusive prefix (every earlier frame's
    // header-valid nonce) from the look-back -- at the end, when the earlier
    // workgroups' aggregates (published after their header pass) are long
    // visible and most have published their inclusive values
    unsigned long long excl = 0;
    if (lb) {
        const unsigned long long P =
            (rp.dbg & 1) ? 0ull : lookback_excl(wg, epoch, rp.lb_flag, rp.lb_agg, rp.lb_inc);
        if (threadIdx.x == 0) {
            const unsigned long long inc = P > wagg ? P : wagg;
            // (a grid of at most kFramesBS workgroups looks back over every
            // aggregate in one round and needs no inclusive values: no
            // publish, and no drain of this wave's last stores for it)
            if (gridDim.x > kFramesBS)
                lookback_publish(rp.lb_flag + wg, rp.lb_inc + wg, inc, epoch, 2);
            if (wg + 1 == gridDim.x) { // _cn_peer_nonce after the batch
                *rp.peer = inc > psn ? inc : psn;
                if (rp.smax)
                    *rp.smax = inc;
            }
        }
        excl = P > wexcl ? P : wexcl;
        if (excl < psn)
            excl = psn;
    }
    if (is_big && q == 0 && !ctl.no_body) {
        if (lb) { // the body's finisher applies the rule to this frame
            rp.excl[i] = excl;
            rp.psnap[i] = psn;
        }
        big(i, list_ctr, nbase);
    }
    if (rp.clk && threadIdx.x == 0) {
        unsigned long long *c = rp.clk + 4ull * blockIdx.x;
        c[0] = rclk0;
        c[1] = __builtin_amdgcn_s_memrealtime();
        c[2] = __builtin_amdgcn_s_memtime() - clk0;
        c[3] = ((unsigned long long) __builtin_amdgcn_s_getreg((31 << 11) | 20) << 32) |
               __builtin_amdgcn_s_getreg((31 << 11) | 4); // XCC_ID : HW_ID
    }
    call_state_end<DEC>(zs, ctl, cs, n);
    frame_result_copy<DEC>(big);
    if (!DEC && valid && q == 0 && ctl.enc_status)
        ctl.enc_status[i] = !sid_ok ? ZMQG_ERR_SESSION : over ? ZMQG_ERR_BOUND : 0;
    if (!valid || q != 0 || !small)
        return;
    if (S == 0) { // decode: header failure (encode: a frame not processed)
        if (DEC)
            fail_unprocessed(status, L_in, dst, flags_out + i, status_out + i, zs, ctl);
        return;
    }
    uint64_t wide[5];
#pragma unroll
    for (int k = 0; k < 5; ++k)
        wide[k] = tot[k];
    uint32_t tag[4];
    poly_finish(fe_from_wide(wide), spad, tag);
    if (!DEC) {
        uint32_t o[16] = {tag[0], tag[1], tag[2], tag[3]};
        store_bytes_c<16>(dst + 16, o);
    } else {
        if (lb && !(vn > excl))
            status = ZMQG_ERR_INVALID_SEQUENCE; // src/curve_mechanism_base.cpp:99-104 (before the MAC)
        else if ((tag[0] ^ wtag[0]) | (tag[1] ^ wtag[1]) | (tag[2] ^ wtag[2]) | (tag[3] ^ wtag[3]))
            status = ZMQG_ERR_CRYPTOGRAPHIC; // src/curve_mechanism_base.cpp:277-281
        status_out[i] = status;
        flags_out[i] = status == 0 ? (uint8_t) (fl | frame_zbits<DEC>(big, i)) : 0;
        if (status != 0) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); // the group's plaintext stores first
            zero_bytes(dst, S - 33u);
        }
    }
}

template <bool DEC, int G, class BigOp>
__global__ __launch_bounds__(kFramesBS) void k_frames(ZMQG_FRAMES_PARAMS)
{
    frames_g_impl<DEC, G, BigOp>(ZMQG_FRAMES_ARGS);
}

// Prefetch of words 1..16 of window w of a stream read in order (word 0 is
// the previous window's word 16): dd[k] = the aligned word at A4 + 64w +
// 4(k+1) (kept apart from word 0 so that they are an even register tuple),
// four dwordx4, issued only where all 16 words are readable -- inside the
// frame, or below the end of the wave's furthest frame (the caller's buffer
// covers every frame, so reading up to that end stays inside it).  Returns
// false where it issued nothing: that lane reloads its words exactly
// (frame_load_exact) in the step that uses them.  The prefetch writes dd only
// through these loads, so dd keeps the loads' register tuples from step to
// step (a second writer of dd, e.g. a select, makes the compiler copy the
// tuples and wait for the loads right where they are issued).
__device__ __forceinline__ bool frame_prefetch(uint64_t A4, uint32_t lim, uint64_t wave_end, uint32_t w,
                                               uint32_t dd[16])
{
    const uint64_t a = A4 + 64ull * w;
    const bool ok = 64u * w + 68u <= lim || a + 68ull <= wave_end;
    if (ok) {
        // (ablation 256, timing only: the 64 bytes read from the 64-byte-aligned place below)
        const GCU4a4 *p = (const GCU4a4 *) (uintptr_t) ((ZMQG_FRAMES_ABLATE & 256) ? (a & ~63ull) : a + 4ull);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const u32x4 tt = p[k];
            dd[4 * k] = tt.x;
            dd[4 * k + 1] = tt.y;
            dd[4 * k + 2] = tt.z;
            dd[4 * k + 3] = tt.w;
        }
    }
    return ok;
}

// Words 1..16 of window w read one by one, a word past the stream's last one
// from the last word's address instead (its bytes are >= S: masked or never
// stored), so no word outside the stream is touched.
__device__ __forceinline__ void frame_load_exact(uint64_t A4, uint32_t lim, uint32_t w, uint32_t dd[16])
{
    const uint32_t last = (lim - 1u) & ~3u; // offset of the last word holding a stream byte
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const uint32_t o = 64u * w + 4u * (k + 1);
        dd[k] = *(GCU32 *) (uintptr_t) (A4 + (o <= last ? o : last));
    }
}

// ---------------------------------------------------------------- one lane per frame
// Wave-wide reductions and scans of the frame kernels' prologue on DPP
// moves instead of LDS permutes (row_shr 1, 2, 4, 8 within rows of 16, then
// row_bcast 15 and 31, or readlanes of the row results): a level costs a
// couple of VALU cycles instead of an LDS round trip.  Lanes without a
// source read 0, the identity of an unsigned maximum.
template <int CTRL, int ROWS>
__device__ __forceinline__ unsigned long long dpp_u64(unsigned long long v)
{
    const uint32_t lo = (uint32_t) __builtin_amdgcn_update_dpp(0, (int) (uint32_t) v, CTRL, ROWS, 0xf, true);
    const uint32_t hi = (uint32_t) __builtin_amdgcn_update_dpp(0, (int) (uint32_t) (v >> 32), CTRL, ROWS, 0xf, true);
    return ((unsigned long long) hi << 32) | lo;
}
__device__ __forceinline__ unsigned long long max_u64(unsigned long long a, unsigned long long b)
{
    return a > b ? a : b;
}
// inclusive prefix maximum over the wave's lanes
__device__ __forceinline__ unsigned long long wave_scan_max_u64(unsigned long long v)
{
    v = max_u64(v, dpp_u64<0x111, 0xf>(v)); // row_shr:1
    v = max_u64(v, dpp_u64<0x112, 0xf>(v)); // row_shr:2
    v = max_u64(v, dpp_u64<0x114, 0xf>(v)); // row_shr:4
    v = max_u64(v, dpp_u64<0x118, 0xf>(v)); // row_shr:8
    v = max_u64(v, dpp_u64<0x142, 0xa>(v)); // row_bcast:15
    v = max_u64(v, dpp_u64<0x143, 0xc>(v)); // row_bcast:31
    return v;
}
// the previous lane's value (lane 0: 0)
__device__ __forceinline__ unsigned long long wave_prev_u64(unsigned long long v)
{
    return dpp_u64<0x138, 0xf>(v); // wave_shr:1
}
// the wave's maximum, on every lane
__device__ __forceinline__ unsigned long long wave_max_u64(unsigned long long v)
{
    v = max_u64(v, dpp_u64<0x111, 0xf>(v));
    v = max_u64(v, dpp_u64<0x112, 0xf>(v));
    v = max_u64(v, dpp_u64<0x114, 0xf>(v));
    v = max_u64(v, dpp_u64<0x118, 0xf>(v));
    unsigned long long m = 0;
#pragma unroll
    for (int r = 15; r < 64; r += 16) {
        const unsigned long long x = ((unsigned long long) (uint32_t) __builtin_amdgcn_readlane((int) (uint32_t) (v >> 32), r) << 32) |
                                     (uint32_t) __builtin_amdgcn_readlane((int) (uint32_t) v, r);
        m = max_u64(m, x);
    }
    return m;
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v)
{
    auto mx = [](uint32_t a, uint32_t b) { return a > b ? a : b; };
    v = mx(v, (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x111, 0xf, 0xf, true));
    v = mx(v, (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x112, 0xf, 0xf, true));
    v = mx(v, (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x114, 0xf, 0xf, true));
    v = mx(v, (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x118, 0xf, 0xf, true));
    return mx(mx((uint32_t) __builtin_amdgcn_readlane((int) v, 15), (uint32_t) __builtin_amdgcn_readlane((int) v, 31)),
              mx((uint32_t) __builtin_amdgcn_readlane((int) v, 47), (uint32_t) __builtin_amdgcn_readlane((int) v, 63)));
}

// Sequential frame kernel: one lane owns one frame and walks its keystream
// windows in order (64 frames per wave), with Poly1305 in the sequential
// radix-2^32 form (curve_device.hpp poly32_*): no powers of r, no
// cross-lane traffic, and a window's last output word carried in a
// register to the next window's store.  Measured against the G-lanes kernel
// (k_frames) and its cost model in tools/frames_proto.hip, DESIGN.md
// section 3:
//   * The MAC of window w is absorbed in step w+1, unconditionally in the
//     keystream's basic block, so the scheduler interleaves its multiply and
//     carry chains with the Salsa20 rounds (at the batch sizes this kernel
//     is chosen for, a wave is alone on its SIMD).
//   * Each step issues the next window's loads and this window's stores
//     together after the input has been consumed: the wait for them comes a
//     whole Salsa20 block later (vmcnt counts loads and stores together, so
//     an earlier wait would drain the stores too).  Issuing them before the
//     keystream instead (stores one step late) measured no faster in this
//     kernel, with the loads branch-free or not.
//   * Decode reads window 0 (header, nonce, tag, first ciphertext) in one
//     load with the header checks taken from it; encode fetches the payload's
//     first bytes with the descriptors.
// ---- LDS-DMA staging, shared by k_frames_lds and k_frames_seq's staged input
constexpr uint32_t kStIn = 80; // input slot: a 64-byte window's 16-byte-aligned cover (5 granules)
typedef u32x4 u32x4_u1 __attribute__((aligned(1)));
typedef __attribute__((address_space(3))) void StLdsVoid;

// One LDS-DMA granule per lane: global [gaddr, +16) -> LDS lds_base + 16 * lane
// (global_load_lds_dwordx4).  Issued from inline asm so that the compiler
// does not treat it as an LDS write of unknown extent: it would then wait for
// it (vmcnt(0)) before every later LDS access of the wave.  The kernel orders
// it itself: one explicit vmcnt(0) at the top of the step that reads the
// buffer, and a buffer is only refilled a step after it was last read.
__device__ __forceinline__ void lds_dma16(uint64_t gaddr, uint32_t lds_base)
{
    // M0 is the compiler's: saved and restored in the same statement
    // (cdna_hip_programming.md section 5.7)
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(gaddr), "s"(lds_base)
                 : "memory");
}

__device__ __forceinline__ uint64_t shfl_u64(uint64_t v, uint32_t src)
{
    const uint32_t lo = (uint32_t) __shfl((int) (uint32_t) v, (int) src);
    const uint32_t hi = (uint32_t) __shfl((int) (uint32_t) (v >> 32), (int) src);
    return ((uint64_t) hi << 32) | lo;
}

// Same frame semantics, replay rule, big-frame hand-off and call state as
// k_frames with G = 1.
template <bool DEC, class BigOp, bool SO = false>
#ifndef ZMQG_SEQ_WPE
#define ZMQG_SEQ_WPE 0 // k_frames_seq: minimum waves per SIMD the register allocation must allow (0: no bound)
#endif
#if ZMQG_SEQ_WPE
#define ZMQG_SEQ_ATTR __attribute__((amdgpu_waves_per_eu(ZMQG_SEQ_WPE)))
#else
#define ZMQG_SEQ_ATTR
#endif
__device__ __forceinline__ void frames_seq_impl(ZMQG_FRAMES_PARAMS)
{
    const bool lb = DEC && rp.lb_flag != nullptr;
    // frames this body covers: all, or (k_frames_split) the first split_n
    const uint32_t nlim = ctl.split_wg ? ctl.split_n : n;
    SEQ_STAMP(0u);
    __shared__ unsigned long long sh_wmax[kFramesWaves];
    __shared__ CallState sh_cs;
    const bool use_ticket = lb && !rp.ordered; // (kernel-uniform)
    const uint32_t lane = threadIdx.x & 63u;

    // The frame's descriptors, session key and first window.  Without a
    // look-back ticket to take, the workgroup's frames are known at entry, so
    // these loads go out before the call state's round trip (thread 0's
    // reads, joined by the barrier below) instead of after it.
    uint32_t i = 0, ii = 0, s = 0, L_in = 0;
    bool valid = false, sid_ok = false, over = false;
    const uint8_t *src = nullptr;
    uint8_t *dst = nullptr;
    uint32_t key[8];
    uint32_t S = 0, n0 = 0, n1 = 0, hl = 1;
    uint64_t A = 0, B = 0;
    int32_t status = 0;
    uint32_t hw[3] = {0, 0, 0};
    uint32_t x0[16], d0 = 0; // window 0's stream words (decode: the wire; encode: payload bytes 0..), word 16
    auto fetch = [&](uint32_t wgv) {
        i = wgv * kFramesBS + threadIdx.x;
        valid = i < nlim;
        ii = valid ? i : nlim - 1;
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
            if (S > 64u)                                     // word 16: stream bytes 64-v.. (payload)
                d0 = *(GCU32 *) (uintptr_t) ((A & ~3ull) + 64ull);
        } else {
            // the wire frame's first window: header, nonce, tag, 32 ciphertext bytes
            A = (uint64_t) (uintptr_t) src;
            uint32_t d[17];
            frame_load_raw(A, 0, L_in, d);
#pragma unroll
            for (int k = 0; k < 16; ++k)
                x0[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], (uint32_t) A & 3u);
            d0 = d[16];
            B = (uint64_t) (uintptr_t) dst - 33u;
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
    const bool small = valid && S <= max_stream;
    unsigned long long vn = 0, wexcl = 0, psn = 0, wagg = 0;
    if (DEC) {
        vn = valid && status == 0 ? (((unsigned long long) bswap32(n0) << 32) | bswap32(n1)) : 0ull;
        psn = rp.peer[s];
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
                sh_wmax[threadIdx.x >> 6] = sc;
            __syncthreads();
            const uint32_t wv = threadIdx.x >> 6;
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
    const uint32_t v = (uint32_t) A & 3u;
    const uint64_t A4 = A & ~3ull;
    const uint32_t lim = S + v; // stream words whose first byte is below lim hold a stream byte
    const uint64_t wave_end = wave_max_u64(nw ? A + S : 0); // end of the wave's furthest frame: reads below it stay in the buffer
    // window 1's words (word 0 is window 0's word 16, d0); windows t and t+1
    // alternate between the two buffers -- or, ZMQG_SEQ_PF 2, windows 1 and
    // 2 are requested here and windows rotate over three buffers, each
    // requested two steps before it is used (inputs from HBM rather than the
    // Infinity Cache take longer than one keystream to arrive)
    uint32_t ddA[16], ddB[16];
    bool fastA = !ZMQG_SEQ_LDSIN && nw > 1u ? frame_prefetch(A4, lim, wave_end, 1u, ddA) : true, fastB = true;
    // ZMQG_SEQ_LDSIN: the wave moves its 64 frames' window covers (five
    // 16-byte granules each, the k_frames_lds input path) into one of two
    // LDS buffers by LDS-DMA, a window ahead; pair j of lane l moves granule
    // (64j + l) % 5 of frame (64j + l) / 5, so each instruction covers runs of
    // whole 80-byte covers instead of 64 lanes' scattered 16-byte pieces, and
    // the owning lane reads its window at its byte offset (unaligned
    // ds_read_b128): no alignbyte shifts, no register buffers held across a
    // keystream
    __shared__ __attribute__((aligned(16))) uint8_t sq_lds[ZMQG_SEQ_LDSIN ? kFramesWaves * 2 * 64 * kStIn : 16];
    uint8_t *const sq_w = sq_lds + (ZMQG_SEQ_LDSIN ? (threadIdx.x >> 6) * 2 * 64 * kStIn : 0u);
    const uint32_t sq_off = __builtin_amdgcn_readfirstlane((uint32_t) (uintptr_t) (StLdsVoid *) sq_w);
    const uint32_t sq_va = (uint32_t) A & 15u;
    uint64_t sq_la[5];
    uint32_t sq_rel[5], sq_lim[5];
    if (ZMQG_SEQ_LDSIN) {
        const uint64_t Ab = A - sq_va;
        const uint32_t lm = S ? sq_va + S : 0u;
#pragma unroll
        for (uint32_t j = 0; j < 5; ++j) {
            const uint32_t idx = 64u * j + lane, f = idx / 5u, k = idx - 5u * f;
            sq_rel[j] = 16u * k;
            sq_la[j] = shfl_u64(Ab, f) + sq_rel[j];
            sq_lim[j] = (uint32_t) __shfl((int) lm, (int) f);
            // (a 16-byte-aligned frame's windows are granules 0..3: its fifth
            // would be the next window's first, moved twice)
            // (the shuffle outside the condition: from an inactive lane it reads 0)
            const int fva = __shfl((int) sq_va, (int) f);
            if (ZMQG_SEQ_SKIP5 && k == 4u && fva == 0)
                sq_lim[j] = 0;
        }
    }
    auto sq_dma = [&](uint32_t t) { // window t's covers -> buffer t & 1 (granules holding a stream byte)
        const uint32_t b = sq_off + (t & 1u) * 64u * kStIn;
#pragma unroll
        for (uint32_t j = 0; j < 5; ++j)
            if (64u * t + sq_rel[j] < sq_lim[j])
                lds_dma16(sq_la[j] + 64ull * t, b + 1024u * j);
    };
    if (ZMQG_SEQ_LDSIN && steps > 1u)
        sq_dma(1u);
#if ZMQG_SEQ_PF == 2
    uint32_t ddC[16];
    bool fastC = true;
    if (nw > 2u)
        fastB = frame_prefetch(A4, lim, wave_end, 2u, ddB);
#endif

    // Decode output in 64-byte payload chunks when every lane's payload
    // starts on a 64-byte boundary (wave-uniform; e.g. packed 1 KiB
    // payloads): chunk c, payload bytes [64c, 64c+64) = stream bytes
    // [64c+33, 64c+97), leaves in step c+1 from windows c (yp) and c+1 as
    // four dwordx4 on one aligned 64-byte piece, so a frame's consecutive
    // steps fill whole 128-byte lines.  Otherwise each window's 64 output
    // bytes go out at their own alignment (frame_store), two partial lines
    // per window.
    const bool al64 = ZMQG_SEQ_AL64 && DEC && __builtin_amdgcn_ballot_w64(((uint32_t) (uintptr_t) dst & 63u) != 0u) == 0;
    uint32_t yp[16]; // al64: the previous window's output words
    // ZMQG_SEQ_COOPST (al64 decode): each lane puts its 64-byte chunk into the
    // wave's LDS staging area, and store j of lane l writes 16 bytes (l % 4)
    // of frame 16j + l / 4's chunk -- each instruction whole 64-byte segments
    // of 16 frames instead of 16-byte pieces of 64 frames' segments, which
    // the L2 wrote back as partial segments (WRITE_SIZE 1.41x the payload,
    // TCC_EA0_WRREQ_64B 1.49 M requests per launch for 1.05 M segments;
    // profiles/pmc_traffic_config2.json)
    // ZMQG_SEQ_COOPST 2: a step's chunks go into the staging area at its end
    // and leave in the next step -- read back at its top, stored after its
    // keystream -- so the single wave on the SIMD never waits on the LDS
    // round trip (form 1, read back and stored at once, costs the resident
    // decode ~8 us per launch)
    bool cs_pend = false; // the staging area holds the previous step's chunks
    // Layout granule-major (granule k of lane l's chunk at kStgPlane k + 16 l,
    // each plane padded by 16 bytes): a lane's four writes are four
    // conflict-free instructions (consecutive lanes, consecutive 16 bytes)
    // instead of 64-byte strides that put every lane on the same eight banks
    constexpr uint32_t kStgPlane = 64u * 16u + 16u;
    __shared__ __attribute__((aligned(16))) uint8_t sq_stg[ZMQG_SEQ_COOPST && SO ? kFramesWaves * 4 * kStgPlane : 16];
    uint8_t *const stg = sq_stg + (ZMQG_SEQ_COOPST && SO ? (threadIdx.x >> 6) * 4u * kStgPlane : 0u);
    auto stg_put = [&](uint32_t k) { return stg + kStgPlane * k + 16u * lane; };
    // store j of this lane: granule lane % 4 of frame 16 j + lane / 4
    auto stg_get = [&](uint32_t j) { return stg + kStgPlane * (lane & 3u) + 16u * (16u * j + (lane >> 2)); };
    uint64_t cs_dst[4];
    uint32_t cs_nw[4];
    // (SO: the ZMQG_OPT_STREAM_OUT instantiation; al64 is wave-uniform)
    // (encode, form 2 only: each window's 64 bytes at frame_store's 4-byte-
    // aligned place, B - up + 64 t; the frame's last window stays per lane)
    const bool coop = ZMQG_SEQ_COOPST && SO && (DEC ? al64 : ZMQG_SEQ_COOPST == 2);
    if (coop) {
        const uint64_t cbase = DEC ? (uint64_t) (uintptr_t) dst : B - (((uint32_t) B & 3u) ? ((uint32_t) B & 3u) : 4u);
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
            const uint32_t f = 16u * j + (lane >> 2);
            cs_dst[j] = shfl_u64(cbase, f) + 16u * (lane & 3u);
            cs_nw[j] = (uint32_t) __shfl((int) nw, (int) f);
        }
    }
    uint32_t ct0[8]; // encode: window 0's ciphertext words (stored with the tag)

    SEQ_STAMP(1u);
    // ---- step 0: window 0 (Poly1305 key, first 32 ciphertext bytes, header)
    PolyKey32 pk;
    Poly32 h = {0, 0, 0, 0, 0};
    uint32_t spad[4], wtag[4] = {0, 0, 0, 0}, fl = 0;
    uint32_t cp[16];  // ciphertext of the window whose MAC is absorbed next step
    uint32_t cp_j0 = 2, cp_len = 0; // its first block slot and ciphertext bytes
    uint32_t ycarry;  // last output word of the previous window
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
        ycarry = y[15];
#pragma unroll
        for (int k = 0; k < 16; ++k)
            yp[k] = y[k];
        if (nw > 0) {
            if (DEC) {
                fl = y[8] & 3u;
                // payload bytes 0 .. min(31, S-33) = plaintext bytes 1..
                uint32_t pay[16];
#pragma unroll
                for (int k = 0; k < 7; ++k)
                    pay[k] = __builtin_amdgcn_alignbyte(y[9 + k], y[8 + k], 1);
                pay[7] = __builtin_amdgcn_alignbyte(0u, y[15], 1);
#pragma unroll
                for (int k = 8; k < 16; ++k)
                    pay[k] = 0;
                if (!al64 || nw == 1u) // (al64: chunk 0 goes out with window 1)
                    store_window(dst, (int) (S < 64u ? S : 64u) - 33, pay);
            } else {
#pragma unroll
                for (int k = 0; k < 8; ++k)
                    ct0[k] = y[8 + k];
                if (S < 64u) { // (a whole first window leaves at the end, with the tag)
                    uint32_t o[16];
                    o[0] = 0x53454d07u; // "\x07MESSAGE" || nonce
                    o[1] = 0x45474153u;
                    o[2] = n0;
                    o[3] = n1;
#pragma unroll
                    for (int k = 4; k < 16; ++k)
                        o[k] = 0;
                    store_bytes_c<16>(dst, o);
                    uint32_t ct[16];
#pragma unroll
                    for (int k = 0; k < 16; ++k)
                        ct[k] = k < 8 ? y[8 + k] : 0u;
                    store_window(dst + 32, (int) S - 32, ct);
                }
            }
        }
    }
    SEQ_STAMP(2u);
    call_state_count(zs);

    // ---- steps 1 ..: window t (words in dd, prefetched by the previous
    // step; the two buffers alternate so that the loads keep their register
    // tuples)
    auto step = [&](uint32_t t, uint32_t (&dd)[16], bool &fast, uint32_t (&dn)[16], bool &fastn) {
        SEQ_STAMP(3u + t);
        const bool act = t < nw;
        // (COOPST 2) the previous step's staged chunks, read now, stored
        // after the keystream
        const bool had = ZMQG_SEQ_COOPST >= 2 && coop && cs_pend;
        u32x4 cg[4];
        if (had) {
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
#pragma unroll
            for (uint32_t j = 0; j < 4; ++j)
                cg[j] = *(const u32x4 *) stg_get(j);
            if (ZMQG_SEQ_COOPST == 3) { // stored here, a whole keystream ahead of the next step's wait
#pragma unroll
                for (uint32_t j = 0; j < 4; ++j)
                    if (t - 1u < cs_nw[j])
                        seq_store4(cs_dst[j] + 64ull * (t - 2u), cg[j].x, cg[j].y, cg[j].z, cg[j].w);
                cs_pend = false;
            }
        }
#if ZMQG_SEQ_PF == 2
        // window t+2 into the buffer window t-1 has left
        if (t + 2u < nw)
            fastn = frame_prefetch(A4, lim, wave_end, t + 2u, dn);
#endif
        uint32_t ks[16];
        if (ZMQG_FRAMES_ABLATE & 32) {
#pragma unroll
            for (int k = 0; k < 16; ++k)
                ks[k] = key[k & 7] ^ (t * 0x9e3779b9u + k);
        } else {
            salsa20_block(ks, key, n0, n1, t, 0);
        }
        // The previous window's MAC (its ciphertext is in cp).  The
        // four-block form runs for every lane, unconditionally, so that it
        // shares a basic block with the keystream and the scheduler
        // interleaves the two; lanes whose window was not four full blocks
        // keep h and take the general form below.
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
        // (keystream and MAC are pinned here, ahead of the next branch:
        // left to itself the compiler sinks them into later blocks -- the
        // keystream below the wait for this window's words)
#pragma unroll
        for (int k = 0; k < 16; ++k)
            asm volatile("" : "+v"(ks[k]));
        asm volatile("" : "+v"(h.h0), "+v"(h.h1), "+v"(h.h2), "+v"(h.h3), "+v"(h.h4));
        if (!(ZMQG_FRAMES_ABLATE & 64) && __builtin_amdgcn_ballot_w64(pv && !full) != 0) {
            if (pv && !full)
                poly32_window(h, pk, cp, cp_j0, cp_len);
        }
        SEQ_STAMP(24u + t);
        uint32_t x[16], w16; // w16: this window's word 16 = the next window's word 0
        if (ZMQG_SEQ_LDSIN) {
            // window t's covers have landed (and the stores of a step ago
            // are out of the way)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            const uint8_t *const p = sq_w + (t & 1u) * 64u * kStIn + kStIn * lane + sq_va;
#pragma unroll
            for (uint32_t q = 0; q < 4; ++q) {
                const u32x4 u = *(const u32x4_u1 *) (p + 16u * q);
                x[4 * q] = u.x;
                x[4 * q + 1] = u.y;
                x[4 * q + 2] = u.z;
                x[4 * q + 3] = u.w;
            }
            w16 = 0;
        } else if (__builtin_amdgcn_ballot_w64(act && !fast) != 0) {
            // a lane whose words were not prefetched (the end of the wave's
            // furthest frame) reads them exactly
            uint32_t ee[16];
            if (act && !fast)
                frame_load_exact(A4, lim, t, ee);
            const bool ex = act && !fast;
            uint32_t e0 = ex ? ee[0] : dd[0];
            x[0] = __builtin_amdgcn_alignbyte(e0, d0, v);
#pragma unroll
            for (int k = 1; k < 16; ++k) {
                const uint32_t ek = ex ? ee[k] : dd[k];
                x[k] = __builtin_amdgcn_alignbyte(ek, e0, v);
                e0 = ek;
            }
            w16 = e0;
        } else {
            x[0] = __builtin_amdgcn_alignbyte(dd[0], d0, v);
#pragma unroll
            for (int k = 1; k < 16; ++k)
                x[k] = __builtin_amdgcn_alignbyte(dd[k], dd[k - 1], v);
            w16 = dd[15];
        }
        d0 = w16;
        if (t < 8u)
            SEQ_STAMP(44u + t);
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
        // window t+1's loads and window t's stores, issued together after
        // the input has been consumed: the wait for the loads comes a whole
        // keystream later
        if (ZMQG_FRAMES_ABLATE & 16) {
#pragma unroll
            for (int k = 0; k < 16; ++k)
                dn[k] = y[k] + k;
            fastn = true;
        } else if (ZMQG_SEQ_LDSIN) {
            if (t + 1u < steps)
                sq_dma(t + 1u);
        } else if (ZMQG_SEQ_PF == 1 && t + 1u < nw) {
            fastn = frame_prefetch(A4, lim, wave_end, t + 1u, dn);
        }
        if (t < 8u)
            SEQ_STAMP(52u + t);
        if (ZMQG_FRAMES_ABLATE & 8) {
            if (act && y[3] == 0x12345678u && y[7] == ycarry)
                *(GU32 *) (uintptr_t) B = y[0];
        } else if (DEC && al64) {
            // payload chunk t-1 (windows t-1 and t); on a lane's last window
            // also what is left of the payload (chunk t, window t alone)
            uint32_t o[16];
#pragma unroll
            for (int k = 0; k < 7; ++k)
                o[k] = __builtin_amdgcn_alignbyte(yp[9 + k], yp[8 + k], 1);
            o[7] = __builtin_amdgcn_alignbyte(y[0], yp[15], 1);
#pragma unroll
            for (int k = 8; k < 16; ++k)
                o[k] = __builtin_amdgcn_alignbyte(y[k - 7], y[k - 8], 1);
            uint8_t *const cdst = dst + 64u * (t - 1u);
            const bool lastw = act && t + 1u == nw;
            if (ZMQG_SEQ_COOPST == 2 && had) { // chunk t-2 of every frame that was active a step ago
#pragma unroll
                for (uint32_t j = 0; j < 4; ++j)
                    if (t - 1u < cs_nw[j])
                        seq_store4(cs_dst[j] + 64ull * (t - 2u), cg[j].x, cg[j].y, cg[j].z, cg[j].w);
                cs_pend = false;
            }
            if (ZMQG_SEQ_COOPST >= 2 && coop && __builtin_amdgcn_ballot_w64(lastw) == 0) {
                // (no lane on its last window: every active frame's chunk is
                // whole; a later step is certain -- the wave's longest frame
                // has not reached its last window -- and stores them)
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); // (after this step's reads)
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    *(u32x4 *) stg_put(k) = (u32x4){o[4 * k], o[4 * k + 1], o[4 * k + 2], o[4 * k + 3]};
                cs_pend = true;
            } else if (ZMQG_SEQ_COOPST == 1 && coop && __builtin_amdgcn_ballot_w64(lastw) == 0) {
                // (no lane on its last window: every active frame's chunk is whole)
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    *(u32x4 *) stg_put(k) = (u32x4){o[4 * k], o[4 * k + 1], o[4 * k + 2], o[4 * k + 3]};
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                u32x4 g[4];
#pragma unroll
                for (uint32_t j = 0; j < 4; ++j)
                    g[j] = *(const u32x4 *) stg_get(j);
#pragma unroll
                for (uint32_t j = 0; j < 4; ++j)
                    if (t < cs_nw[j])
                        seq_store4(cs_dst[j] + 64ull * (t - 1u), g[j].x, g[j].y, g[j].z, g[j].w);
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); // (the reads before the next step's writes)
            } else if (__builtin_amdgcn_ballot_w64(lastw) == 0) {
                if (act) {
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                        seq_store4((uint64_t) (uintptr_t) cdst + 16u * k, o[4 * k], o[4 * k + 1], o[4 * k + 2],
                                   o[4 * k + 3]);
                }
            } else {
                const uint32_t P = S - 33u; // (act: S >= 64t + 1 > 33)
                if (act) {
                    const uint32_t r = P - 64u * (t - 1u);
                    const uint32_t o17[17] = {o[0], o[1], o[2],  o[3],  o[4],  o[5],  o[6],  o[7], o[8],
                                              o[9], o[10], o[11], o[12], o[13], o[14], o[15], 0u};
                    store_tail((uint64_t) (uintptr_t) cdst, r < 64u ? r : 64u, o17);
                }
                if (lastw && P > 64u * t) {
                    uint32_t o2[17];
#pragma unroll
                    for (int k = 0; k < 7; ++k)
                        o2[k] = __builtin_amdgcn_alignbyte(y[9 + k], y[8 + k], 1);
                    o2[7] = __builtin_amdgcn_alignbyte(0u, y[15], 1);
#pragma unroll
                    for (int k = 8; k < 17; ++k)
                        o2[k] = 0;
                    store_tail((uint64_t) (uintptr_t) (cdst + 64), P - 64u * t, o2);
                }
            }
#pragma unroll
            for (int k = 0; k < 16; ++k)
                yp[k] = y[k];
        } else {
            const bool lastw = act && t + 1u == nw;
            if constexpr (!DEC) {
                if (ZMQG_SEQ_COOPST == 2 && had) { // window t-1 of every frame that was active a step ago
#pragma unroll
                    for (uint32_t j = 0; j < 4; ++j)
                        if (t - 1u < cs_nw[j])
                            seq_store4(cs_dst[j] + 64ull * (t - 1u), cg[j].x, cg[j].y, cg[j].z, cg[j].w);
                    cs_pend = false;
                }
            }
            if (!DEC && ZMQG_SEQ_COOPST == 2 && coop && __builtin_amdgcn_ballot_w64(lastw) == 0) {
                // (no lane on its last window: each active frame's window is
                // frame_store's whole 64 bytes; a later step stores them)
                const uint32_t u = (uint32_t) B & 3u, sh = u ? 4u - u : 0u;
                uint32_t o[16];
                o[0] = __builtin_amdgcn_alignbyte(y[0], ycarry, sh);
#pragma unroll
                for (int k = 1; k < 16; ++k)
                    o[k] = __builtin_amdgcn_alignbyte(y[k], y[k - 1], sh);
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); // (after this step's reads)
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    *(u32x4 *) stg_put(k) = (u32x4){o[4 * k], o[4 * k + 1], o[4 * k + 2], o[4 * k + 3]};
                cs_pend = true;
            } else if (act) {
                frame_store(B, t, S, y, ycarry, lastw);
            }
        }
        ycarry = y[15];
        if (t < 8u)
            SEQ_STAMP(36u + t);
    };
    // (both exits leave the loop: a skipped second step reaching the back
    // edge would leave buffer B's loads outstanding at the loop head as far
    // as the compiler's wait analysis knows, and every step would then wait
    // for all loads before its first write of a buffer register)
    if (steps > 1u) {
#if ZMQG_SEQ_PF == 2
#pragma unroll 1
        for (uint32_t t = 1;; t += 3) {
            step(t, ddA, fastA, ddC, fastC);
            if (t + 1u >= steps)
                break;
            step(t + 1u, ddB, fastB, ddA, fastA);
            if (t + 2u >= steps)
                break;
            step(t + 2u, ddC, fastC, ddB, fastB);
            if (t + 3u >= steps)
                break;
        }
#else
#pragma unroll 1
        for (uint32_t t = 1;; t += 2) {
            step(t, ddA, fastA, ddB, fastB);
            if (t + 1u >= steps)
                break;
            step(t + 1u, ddB, fastB, ddA, fastA);
            if (t + 2u >= steps)
                break;
        }
#endif
    }
    SEQ_STAMP(60u);
    // the last window's MAC
    if (steps > 0 && nw == steps)
        poly32_window(h, pk, cp, cp_j0, cp_len);

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
#if ZMQG_SEQ_STAMPS
    // (diagnostic: where the wave ran -- XCC_ID : HW_ID, whose CU, SH, SE and
    // SIMD fields tell which waves shared a CU or a SIMD)
    if (rp.clk && (threadIdx.x & 63u) == 0)
        rp.clk[64ull * (blockIdx.x * kFramesWaves + (threadIdx.x >> 6)) + 62u] =
            ((unsigned long long) __builtin_amdgcn_s_getreg((31 << 11) | 20) << 32) |
            __builtin_amdgcn_s_getreg((31 << 11) | 4);
#endif
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
        if (S >= 64u) {
            // wire bytes 0..63: "\x07MESSAGE", nonce, tag, the first 32
            // ciphertext bytes -- one fixed store sequence at the frame's
            // alignment instead of three byte-exact ones
            const uint32_t o[16] = {0x53454d07u, 0x45474153u, n0,     n1,     tag[0], tag[1], tag[2], tag[3],
                                    ct0[0],      ct0[1],      ct0[2], ct0[3], ct0[4], ct0[5], ct0[6], ct0[7]};
            store_bytes_c<64>(dst, o);
        } else {
            const uint32_t o[16] = {tag[0], tag[1], tag[2], tag[3]};
            store_bytes_c<16>(dst + 16, o);
        }
    } else {
        if (lb && !(vn > excl))
            status = ZMQG_ERR_INVALID_SEQUENCE; // src/curve_mechanism_base.cpp:99-104 (before the MAC)
        else if ((tag[0] ^ wtag[0]) | (tag[1] ^ wtag[1]) | (tag[2] ^ wtag[2]) | (tag[3] ^ wtag[3]))
            status = ZMQG_ERR_CRYPTOGRAPHIC; // src/curve_mechanism_base.cpp:277-281
        status_out[i] = status;
        flags_out[i] = status == 0 ? (uint8_t) (fl | frame_zbits<DEC>(big, i)) : 0;
        if (status != 0) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); // this lane's plaintext stores first
            zero_bytes(dst, S - 33u);
        }
    }
}

template <bool DEC, class BigOp, bool SO = false>
__global__ __launch_bounds__(kFramesBS) ZMQG_SEQ_ATTR void k_frames_seq(ZMQG_FRAMES_PARAMS)
{
    frames_seq_impl<DEC, BigOp, SO>(ZMQG_FRAMES_ARGS);
}

// Batches just above one wave per SIMD (slots < n <= 3 slots / 2): the
// first split_n = slots frames one lane each (one wave on every SIMD), the
// remainder GT lanes per frame, in the same launch.  A SIMD that also holds
// a remainder wave then runs about ceil(17 / GT) windows more instead of a
// whole second frame (k_frames_seq alone: +50 % at 70,000 x 1 KiB,
// DESIGN.md section 3.1).  Workgroup order is frame order, so the
// one-session replay look-back runs across the two bodies unchanged; the
// host launches this only when the grid is co-resident (no tickets).
template <bool DEC, int GT, class BigOp>
__global__ __launch_bounds__(kFramesBS) ZMQG_SEQ_ATTR void k_frames_split(ZMQG_FRAMES_PARAMS)
{
    if (blockIdx.x < ctl.split_wg)
        frames_seq_impl<DEC, BigOp>(ZMQG_FRAMES_ARGS);
    else
        frames_g_impl<DEC, GT, BigOp>(ZMQG_FRAMES_ARGS);
}

} // namespace zmqg
