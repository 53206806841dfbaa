// zmqg_curve.hip -- batched CurveZMQ MESSAGE encode/decode for MI355X (gfx950).
//
// Replaces, for a batch of frames at once, reference
// src/curve_mechanism_base.cpp:80-284 (curve_encoding_t::encode / decode /
// check_validity, which call libsodium crypto_box_easy_afternm and
// crypto_box_open_easy_afternm) and src/mechanism_base.cpp:14-25.
// The C ABI is include/zmqg_curve.h.
//
// Work decomposition:
//   frame kernel  G lanes per frame (curve_frames.hpp): every frame whose
//                 stream fits kMaxFrameStream bytes is encoded/decoded whole
//                 (keystream, Poly1305, tag) in one pass.  Decode also
//                 records each frame's header-valid nonce for the replay rule.
//   head kernel   one lane per larger frame: keystream block 0 (Poly1305
//                 key r,s + first 32 ciphertext bytes), the powers of r the
//                 body needs, and the frame's body chunks; the frame is
//                 appended to the big-frame list (one packed atomic gives
//                 its list position and chunk range together).
//   body kernel   big frames: one lane per chunk = 2 Salsa20 blocks = 128
//                 ciphertext bytes = 8 Poly1305 blocks; lanes of a frame are
//                 adjacent, so the per-chunk Poly1305 partials (each
//                 multiplied by its power of r) are summed by a segmented
//                 wave reduction and the segment leader finishes the tag;
//                 frames spanning several waves combine through 64-bit
//                 atomics and an arrival counter (last arriver finishes).
//   replay fixup  decode only: the reference's sequential _cn_peer_nonce
//                 rule (src/curve_mechanism_base.cpp:98-106) in batch order
//                 -- per-session exclusive prefix max of header-valid nonces
//                 (one session: workgroup maxima + in-tile scan; several:
//                 hipCUB sort-by-session + segmented scan) -- sets
//                 INVALID_SEQUENCE and each session's new peer nonce.
#include <errno.h>
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <sched.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <mutex>
#include <vector>

#include "../../include/zmqg_curve.h"
#include "curve_box.hpp"
#include "curve_device.hpp"
#include "curve_frames.hpp"
#include "curve_frames_lds.hpp"
#include "curve_msg.hpp"
#include "curve_z85.hpp"
#include "curve_x25519.hpp"
#include "curve_zmtp.hpp"

#ifndef ZMQG_ABLATE
#define ZMQG_ABLATE 0
#endif
#ifndef ZMQG_STAMPS
#define ZMQG_STAMPS 0
#endif
#if ZMQG_STAMPS // diagnostic build only: per-wave phase timestamps (tools/stamps.py)
__device__ unsigned long long zmqg_stamp_buf[1 << 17];
__device__ unsigned int zmqg_stamp_ctr;
#define ZSTAMP(k)                                                                   \
    do {                                                                            \
        __builtin_amdgcn_sched_barrier(0);                                          \
        unsigned long long t_;                                                      \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory"); \
        __builtin_amdgcn_sched_barrier(0);                                          \
        st_[k] = t_;                                                                \
    } while (0)
#else
#define ZSTAMP(k) do { } while (0)
#endif

using namespace zmqg;

namespace {

constexpr uint32_t kChunk = 128;      // body chunk: 2 Salsa20 blocks = 8 Poly1305 blocks per lane
constexpr int kMaxPow = 25;           // r^(8*2^k), k < 25: frames up to 2^32 bytes
constexpr uint32_t kIdle = 0xffffffffu;
constexpr int kBodyThreads = 256; // 4 waves x 2 tile buffers of 9 KiB: 2 workgroups (8 waves) per CU
constexpr int kHeadThreads = 256;
constexpr uint32_t kMaxFrameStream = 64 * 72; // frames up to 4.5 KiB of stream: frame kernel
constexpr int kFixupThreads = 256;

// Per-frame records written by the head kernel and read by the body kernel,
// grouped by when a body lane needs them so each group is one batch of
// independent dwordx4 loads (no dependent-load chains in the body).
struct __attribute__((aligned(16))) FrameHot { // needed to start a chunk (96 B)
    uint32_t key[8];  // XSalsa20 subkey of the frame's session/direction
    uint32_t r[5];    // Poly1305 r (clamped), 26-bit limbs
    uint32_t nch;     // body chunks (>= 1; a frame with no body bytes gets one empty chunk)
    uint32_t mlen;    // boxed plaintext length (flags + sub/cancel + payload)
    uint32_t hl;      // encode: plaintext header length (1, 2, 8 or 11)
    uint32_t n0, n1;  // Salsa20 nonce words (the 8 wire nonce bytes, little-endian)
    int32_t status;   // decode: header status (0 = header ok)
    uint32_t flags;   // decode: plaintext flags & 3, | kHotMove
    uint64_t in_base;  // encode: payload byte 0; decode: wire byte 0
    uint64_t out_base; // encode: wire byte 0; decode: payload byte 0
};
static_assert(sizeof(FrameHot) == 96, "FrameHot layout");
constexpr uint32_t kHotMove = 0x80; // decode in place: payload moved from wire offset 33 to 0 by k_post

constexpr int kPowInline = 6; // r^(8*2^k) for k < 6 kept in the record: a tile's in-segment powers (< 64 chunks)
struct __attribute__((aligned(16))) FramePow { // chunk factor inputs (144 B)
    uint32_t rb[5];                // r^(Poly1305 blocks in the last chunk)
    uint32_t t[kPowInline][5];     // r^(8*2^k)
    uint32_t pad[1];
};
static_assert(sizeof(FramePow) == 144, "FramePow layout");

struct __attribute__((aligned(16))) FrameFin { // tag / status inputs (64 B)
    uint32_t hh[5];     // head blocks' Horner value times r^(body blocks)
    uint32_t s[4];      // Poly1305 pad
    uint32_t tag[4];    // decode: tag carried on the wire
    uint32_t wire_len;  // decode: frame bytes on the wire
    uint32_t frame;     // the frame's index in the batch
    uint32_t pad;
};
static_assert(sizeof(FrameFin) == 64, "FrameFin layout");

struct Workspace {
    uint64_t cap = 0; // frames
    FrameHot *hot = nullptr;
    FramePow *pw = nullptr;
    FrameFin *fin = nullptr;
    uint32_t *powtab = nullptr;   // [cap][kMaxPow][5], entries k >= kPowInline
    unsigned long long *acc = nullptr; // [cap][5]
    uint32_t *cnt = nullptr;      // [cap]
    uint32_t *nch = nullptr;      // [cap]
    uint32_t *chunk_end = nullptr; // [cap]
    unsigned long long *v = nullptr;     // [cap] accepted nonce or 0
    unsigned long long *excl = nullptr;  // [cap]
    unsigned long long *v_s = nullptr;   // [cap] sorted
    unsigned long long *excl_s = nullptr; // [cap]
    uint32_t *iota = nullptr;     // [cap]
    uint32_t *perm = nullptr;     // [cap]
    uint32_t *keys_s = nullptr;   // [cap]
    uint8_t *last = nullptr;      // [cap] last frame of its session in the batch
    uint32_t *list_frame = nullptr;      // [cap] big-frame list: frame index at each position
    PostOp *post = nullptr;              // [cap] decode: k_post's zero fills and in-place moves
    unsigned long long *psnap = nullptr; // [cap] session peer nonce before the batch, per frame
    unsigned long long *blockmax = nullptr; // [cap] frame-kernel workgroup maxima of vout
    ZState *zs = nullptr;                   // call state carried from call to call (on the device)
    unsigned long long *lb_flag = nullptr;  // [cap] look-back state per workgroup ticket
    unsigned long long *lb_agg = nullptr;   // [cap]
    unsigned long long *lb_inc = nullptr;   // [cap]
    void *temp = nullptr;
    size_t temp_bytes = 0;
    unsigned long long *rt = nullptr; // replay tables: [tiles][S] then [row blocks][S] (also the nonce tables)
    uint64_t *nonce = nullptr;        // [cap] ZMQG_OPT_NONCE_AUTO over several sessions: each frame's nonce
    size_t rt_cap = 0;
    uint8_t *stage = nullptr;         // ZMQG_OPT_VERIFY_FIRST: decoded payloads before the verdict copy
    size_t stage_cap = 0;
    bool use_last = false; // the last replay ran the sort fallback (k_fixup writes the peer nonces)
};

} // namespace

namespace {
// The synchronous zmqg_decode_zmtp's result, written by the decode into
// mapped host memory.
struct ZmtpResHost {
    zmqg_zmtp_result r;
};

// device buffers of the ZMTP framing calls
struct ZmtpWs {
    uint64_t n_cap = 0;                   // send side: frames
    uint64_t *F = nullptr;                // [n_cap + 1] frame bytes
    uint64_t *wire_off = nullptr;         // [n_cap] body offsets
    uint64_t g_cap = 0;                   // receive side: 16 KiB workgroups of the stream
    uint64_t c_cap = 0;                   // receive side: candidates
    uint64_t f_cap = 0;                   // receive side: frames (max_frames)
    uint64_t *cand_wg = nullptr;          // [g_cap * kZmtpWgCap] each workgroup's candidates, in order
    uint64_t *count_wg = nullptr;         // [g_cap + 1]
    uint64_t *off_wg = nullptr;           // [g_cap + 1] exclusive sum of count_wg
    uint16_t *count16 = nullptr;          // [g_cap + 8] count_wg as 16-bit fields (k_zmtp_compact sums them)
    uint64_t *cand = nullptr;             // [c_cap] sorted candidates
    uint64_t *cdesc = nullptr;            // [c_cap] their frames: body offset | body length << 32
    uint8_t *cflag = nullptr;             // [c_cap] their flags bytes
    uint64_t *nb = nullptr;               // [c_cap] next unlinked candidate in the 256-candidate segment
    uint64_t *first_w = nullptr;          // [g_cap + 1] first unlinked candidate in workgroup lists >= w
    uint32_t *wid = nullptr;              // [c_cap] each candidate's workgroup list
    uint64_t *run = nullptr;              // [2 (f_cap + 1)]
    uint64_t *runpre = nullptr;           // [f_cap + 1]
    uint32_t *sid_fill = nullptr;         // [f_cap]
    uint8_t *fflags = nullptr;            // [f_cap]
    ZmtpWalk *walk = nullptr;
    ZmtpResHost *res = nullptr;           // the synchronous call's result, mapped host memory
    ZmtpResHost *res_dev = nullptr;       // (its device address)
    void *temp = nullptr;
    size_t temp_bytes = 0;
};
} // namespace

struct zmqg_ctx {
    int device = 0;
    int cus = 256; // compute units of the device (one persistent body workgroup each)
    uint32_t max_sessions = 0;
    int sort_bits = 0;
    DevSession *sessions = nullptr;
    unsigned long long *peer = nullptr; // [max_sessions]
    unsigned long long *send = nullptr; // [max_sessions] send nonces (_cn_nonce) for ZMQG_OPT_NONCE_AUTO
    unsigned long long *zero_peer = nullptr; // [max_sessions] zeros: ZMQG_OPT_REPLAY_HOST's peer snapshot
    Workspace ws;
    ZmtpWs zw;
    // host staging for the *_host entry points
    uint8_t *pin = nullptr;
    size_t pin_bytes = 0;
    uint8_t *mpin = nullptr, *mpin_dev = nullptr; // the per-message buffer (zmqg_*_msg), device-mapped
    size_t mpin_bytes = 0;
    // zmqg_session_set_batch: device-mapped descriptors of the last install,
    // free again once `sinst_done` is reached
    uint8_t *sinst = nullptr, *sinst_dev = nullptr;
    size_t sinst_bytes = 0;
    hipEvent_t sinst_done = nullptr;
    hipEvent_t order_ev = nullptr; // zmqg_*_msg: own_stream waits for the last batch stream's work
    uint8_t *dbuf = nullptr;
    size_t dbuf_bytes = 0;
    hipStream_t own_stream = nullptr;
    // the stream of the last batch call (the session accessors and the
    // per-message calls order after it); has_last tells "none yet" from the
    // null stream, which is a stream like any other here
    hipStream_t last_stream = nullptr;
    bool has_last = false;
    std::vector<uint8_t> h_downgrade; // host copy of each session's downgrade_sub
    // profiling: event pairs per kind, recycled through a pool
    bool profiling = false;
    int frames_cap[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}; // decode frame-kernel workgroups resident at once, G = 1,
                                                     // 2, 4, seq, lds, split 2, 4, 8, seq under STREAM_OUT
    int force_g = -1;                 // ZMQG_FRAMES_G: frame-kernel variant override (experiments)
    std::vector<std::pair<hipEvent_t, hipEvent_t>> prof[6];
    std::vector<hipEvent_t> event_pool;
    // completion fences of the asynchronous host path: (id, event) pending,
    // events recycled through fence_pool
    std::vector<std::pair<uint64_t, hipEvent_t>> fences;
    std::vector<hipEvent_t> fence_pool;
    // zmqg_fence_record_notify: ids whose host function has run (a fence
    // found there is reached whatever its event says), and the host
    // functions enqueued and not yet finished
    std::mutex notify_mu;
    std::vector<uint64_t> notified;
    std::atomic<int> notify_pending{0};
    uint64_t fence_ctr = 0;
    std::mutex fence_mu;
    char last_error[256] = {0};
    std::mutex mu;
};

#define ZCHECK(ctx, expr)                                                                      \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess) {                                                                \
            snprintf((ctx)->last_error, sizeof((ctx)->last_error), "%s:%d %s: %s", __FILE__,   \
                     __LINE__, #expr, hipGetErrorString(e_));                                  \
            return -EIO;                                                               \
        }                                                                                      \
    } while (0)

// The ctx's work is ordered by stream: a batch call runs on the caller's
// stream (which then becomes the ctx's last stream); every call that uses
// the ctx's workspace or sessions on another stream than the last one --
// the batch calls, the session installs and accessors, the per-message
// calls -- first makes it wait for everything queued on the last one (an
// event recorded there, order_after_last; nothing when the stream is the
// same).  The null stream is a stream like any other: with own_stream
// non-blocking it is not ordered implicitly.
static int notify_wait(zmqg_ctx *ctx);

static void set_last(zmqg_ctx *ctx, hipStream_t st)
{
    ctx->last_stream = st;
    ctx->has_last = true;
}

static int order_after_last(zmqg_ctx *ctx, hipStream_t st)
{
    if (ctx->has_last && ctx->last_stream != st) {
        if (!ctx->order_ev)
            ZCHECK(ctx, hipEventCreateWithFlags(&ctx->order_ev, hipEventDisableTiming));
        ZCHECK(ctx, hipEventRecord(ctx->order_ev, ctx->last_stream));
        ZCHECK(ctx, hipStreamWaitEvent(st, ctx->order_ev, 0));
    }
    set_last(ctx, st);
    return 0;
}

// =====================================================================
// device helpers
// =====================================================================
namespace {

__device__ __forceinline__ fe load_fe(const uint32_t *p)
{
    fe x;
#pragma unroll
    for (int i = 0; i < 5; ++i)
        x.l[i] = p[i];
    return x;
}

__device__ __forceinline__ void store_fe(uint32_t *p, const fe &x)
{
#pragma unroll
    for (int i = 0; i < 5; ++i)
        p[i] = x.l[i];
}

// Number of Poly1305 blocks in the last body chunk, and body chunk count.
__device__ __forceinline__ void body_geometry(uint32_t mlen, uint32_t &nch, uint32_t &blast)
{
    if (mlen <= 32) {
        nch = 1;
        blast = 0;
        return;
    }
    const uint32_t body = mlen - 32;
    nch = (body + kChunk - 1) / kChunk;
    const uint32_t lastb = body - kChunk * (nch - 1);
    blast = (lastb + 15) / 16;
}

// Computes r^blast and r^(8*2^k) for k < bits(nch-1) (the first kPowInline
// into the frame record, the rest into powtab), and returns the head factor
// r^(body blocks) = r^blast * (r^8)^(nch-1).
static_assert(kChunk == 128, "head_powers assumes 8 Poly1305 blocks per chunk");
__device__ void head_powers(const fe &r, uint32_t nch, uint32_t blast, FramePow *P, uint32_t *powtab, fe &head_factor)
{
    fe r2 = r;
    fe_mul(r2, r);
    fe r4 = r2;
    fe_mul(r4, r2);
    fe r8 = r4;
    fe_mul(r8, r4);
    fe rb = fe_one();
    if (blast == 8) {
        rb = r8;
    } else {
        if (blast & 1)
            fe_mul(rb, r);
        if (blast & 2)
            fe_mul(rb, r2);
        if (blast & 4)
            fe_mul(rb, r4);
    }
    store_fe(P->rb, rb);
#pragma unroll
    for (int k = 0; k < kPowInline; ++k)
        store_fe(P->t[k], fe_zero());
    head_factor = rb;
    const uint32_t m = nch - 1; // head multiplies by (r^8)^(nch-1)
    fe t = r8;
    for (int k = 0; (m >> k) != 0; ++k) {
        if (k < kPowInline)
            store_fe(P->t[k], t); // global record: a runtime index is fine here
        else
            store_fe(powtab + 5 * k, t);
        if ((m >> k) & 1)
            fe_mul(head_factor, t);
        fe t2 = t;
        fe_mul(t2, t);
        t = t2;
    }
}

// =====================================================================
// session setup
// =====================================================================
__global__ void k_session_setup(DevSession *tab, unsigned long long *peer, unsigned long long *send, uint32_t sid,
                                const uint32_t *in)
{
    // in: precom[8] enc_prefix[4] dec_prefix[4] downgrade peer_lo peer_hi
    if (threadIdx.x != 0)
        return;
    uint32_t k[8];
    for (int i = 0; i < 8; ++i)
        k[i] = in[i];
    DevSession s;
    hsalsa20(s.enc_key, k, in + 8);
    hsalsa20(s.dec_key, k, in + 12);
    s.downgrade_sub = in[16];
    for (int i = 0; i < 7; ++i)
        s.pad[i] = 0;
    tab[sid] = s;
    peer[sid] = ((unsigned long long) in[18] << 32) | in[17];
    send[sid] = 1; // _cn_nonce (1), src/curve_mechanism_base.cpp:59
}

// zmqg_session_set_batch: one thread per session, the two HSalsa20 subkeys
// of k_session_setup.  `d` (device-mapped host memory): sid[n], then
// peer_nonce[n] (u64), then send_nonce[n] (u64), then downgrade[n] (u8);
// precom n x 32 bytes
// (device-accessible, 4-byte aligned); pfx = enc_prefix[4] dec_prefix[4].
struct Prefixes {
    uint32_t w[8];
};
__global__ __launch_bounds__(256) void k_session_setup_batch(uint32_t n, const uint8_t *__restrict__ d,
                                                             const uint32_t *__restrict__ precom, Prefixes pfx,
                                                             DevSession *tab, unsigned long long *peer,
                                                             unsigned long long *send)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    const uint32_t *sid = (const uint32_t *) d;
    const unsigned long long *pn = (const unsigned long long *) (d + ((4ull * n + 7) & ~7ull));
    const unsigned long long *sn = pn + n;
    const uint8_t *down = d + ((4ull * n + 7) & ~7ull) + 16ull * n;
    const uint32_t s = sid[i];
    uint32_t k[8];
#pragma unroll
    for (int t = 0; t < 8; ++t)
        k[t] = precom[8ull * i + t];
    DevSession x;
    hsalsa20(x.enc_key, k, pfx.w);
    hsalsa20(x.dec_key, k, pfx.w + 4);
    x.downgrade_sub = down[i] ? 1u : 0u;
#pragma unroll
    for (int t = 0; t < 7; ++t)
        x.pad[t] = 0;
    tab[s] = x;
    peer[s] = pn[i];
    send[s] = sn[i]; // (1 unless given: _cn_nonce (1), src/curve_mechanism_base.cpp:59)
}

__global__ void k_fill_u64(unsigned long long *p, uint32_t n, unsigned long long v)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n)
        p[i] = v;
}

__global__ void k_set_peer(unsigned long long *arr, uint32_t sid, unsigned long long v)
{
    if (threadIdx.x == 0)
        arr[sid] = v;
}

// =====================================================================
// encode
// =====================================================================
// Big-frame list: one packed atomic gives a frame its list position (high
// 24 bits) and its body chunk range (low 40 bits) together, so chunk_end is
// increasing in list position whatever order the frames arrive in.
__device__ __forceinline__ uint32_t list_append(unsigned long long *list_ctr, uint32_t *chunk_end,
                                                uint32_t *list_frame, uint32_t i, uint32_t nch)
{
    const unsigned long long old = atomicAdd(list_ctr, (1ull << 40) | nch);
    const uint32_t pos = (uint32_t) (old >> 40);
    chunk_end[pos] = (uint32_t) (old & ((1ull << 40) - 1)) + nch;
    list_frame[pos] = i;
    return pos;
}

// Where the chunked path keeps a big frame's records (indexed by list position).
struct BigRecords {
    FrameHot *hot;
    FramePow *pw;
    FrameFin *fin;
    uint32_t *powtab;
    unsigned long long *acc;
    uint32_t *cnt;
    uint32_t *chunk_end;
    uint32_t *list_frame;
};

// The chunked path's head for one encode frame whose stream exceeds the
// frame kernel's limit (called by the frame kernel on one lane): keystream
// block 0, records for the body, list entry.
struct EncodeHead {
    const uint32_t *sid;
    const uint64_t *nonce;
    const uint8_t *flags;
    const uint64_t *in_off;
    const uint32_t *len;
    const uint8_t *in;
    const uint64_t *out_off;
    uint8_t *out;
    const DevSession *sessions;
    uint32_t max_sessions;
    BigRecords R;
    const unsigned long long *nonce_ctr; // ZMQG_OPT_NONCE_AUTO, one session (FrameCtl::nonce_ctr)
    __device__ void operator()(uint32_t i, unsigned long long *list_ctr, uint64_t nbase) const;
};

__device__ void EncodeHead::operator()(uint32_t i, unsigned long long *list_ctr, uint64_t nbase) const
{
    FrameHot *hot = R.hot;
    FramePow *pw = R.pw;
    FrameFin *fin = R.fin;
    uint32_t *powtab = R.powtab;
    unsigned long long *acc = R.acc;
    uint32_t *cnt = R.cnt;
    const uint32_t s = sid[i] < max_sessions ? sid[i] : 0;
    const DevSession &ses = sessions[s];
    const uint32_t P = len[i];
    uint32_t hw[3];
    const uint32_t hl = plaintext_header(flags[i], ses.downgrade_sub, hw);
    const uint32_t mlen = hl + P;
    uint32_t nch, blast;
    body_geometry(mlen, nch, blast);
    const uint32_t p = list_append(list_ctr, R.chunk_end, R.list_frame, i, nch);
    FrameHot H;
#pragma unroll
    for (int t = 0; t < 8; ++t)
        H.key[t] = ses.enc_key[t];
    // (the counter as the frame kernel read it at its start: the workgroup
    // completing the call count advances it for the next call)
    const uint64_t nc = nonce_ctr ? nbase + i : nonce[i];
    const uint32_t n0 = bswap32((uint32_t) (nc >> 32)), n1 = bswap32((uint32_t) nc);

    uint32_t ks[16];
    salsa20_block(ks, H.key, n0, n1, 0, 0);
    const fe r = poly_r_from_key(ks[0], ks[1], ks[2], ks[3]);

    // plaintext bytes 0..31 = header || payload[0 .. 32-hl)
    const uint8_t *src = in + in_off[i];
    uint32_t pw16[16];
    load_window(src, P < 32 ? (int) P : 32, pw16);
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
    const int nv0 = mlen < 32 ? (int) mlen : 32;
    uint32_t ct[16];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        ct[t] = pt[t] ^ ks[8 + t];
        ct[8 + t] = 0;
    }
    mask_tail(ct, nv0);

    uint8_t *o = out + out_off[i];
    uint32_t hdr[16] = {0x53454d07u, 0x45474153u, n0, n1};
    store_window(o, 16, hdr);
    store_window(o + 32, nv0, ct);

    fe h = fe_zero();
    const uint32_t s1 = r.l[1] * 5, s2 = r.l[2] * 5, s3 = r.l[3] * 5, s4 = r.l[4] * 5;
    poly_absorb64(h, r, s1, s2, s3, s4, ct, nv0);

    fe hf;
    head_powers(r, nch, blast, pw + p, powtab + (size_t) p * kMaxPow * 5, hf);
    if (mlen > 32)
        fe_mul(h, hf);

    store_fe(H.r, r);
    H.nch = nch;
    H.mlen = mlen;
    H.hl = hl;
    H.n0 = n0;
    H.n1 = n1;
    H.status = 0;
    H.flags = 0;
    H.in_base = (uint64_t) (uintptr_t) src;
    H.out_base = (uint64_t) (uintptr_t) o;
    hot[p] = H;
    FrameFin F;
    store_fe(F.hh, h);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        F.s[t] = ks[4 + t];
        F.tag[t] = 0;
    }
    F.wire_len = mlen + 32;
    F.frame = i;
    F.pad = 0;
    fin[p] = F;
#pragma unroll
    for (int t = 0; t < 5; ++t)
        acc[(size_t) p * 5 + t] = 0;
    cnt[p] = 0;
}

// Segmented (by frame) sum of the lanes' Poly1305 contributions over one
// wave; returns true on the first lane of each segment, which then holds
// the segment total.
__device__ __forceinline__ bool wave_segment_sum(uint32_t key, uint64_t v[5])
{
    const int lane = threadIdx.x & 63;
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t kd = __shfl_down(key, d);
        const bool take = (lane + d < 64) && kd == key && key != kIdle;
        if (!__any(take))
            break;
        uint64_t t[5];
#pragma unroll
        for (int q = 0; q < 5; ++q)
            t[q] = __shfl_down(v[q], d);
        if (take) {
#pragma unroll
            for (int q = 0; q < 5; ++q)
                v[q] += t[q];
        }
    }
    const uint32_t kp = __shfl_up(key, 1);
    return key != kIdle && (lane == 0 || kp != key);
}

// Sum of the lanes' contributions when the whole wave is one segment: 32-bit
// row sums by DPP (each lane's limbs are below 2^26 + 64 -- fe_mul's output
// -- so a row of 16 stays below 2^31), the four rows added in 64 bits.
// Every lane gets the total.
__device__ __forceinline__ void wave_sum_all(uint64_t v[5])
{
#pragma unroll
    for (int q = 0; q < 5; ++q) {
        int x = (int) (uint32_t) v[q];
        x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, true); // row_shr:1
        x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, true); // row_shr:2
        x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, true); // row_shr:4
        x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, true); // row_shr:8
        v[q] = (uint64_t) (uint32_t) __builtin_amdgcn_readlane(x, 15) + (uint32_t) __builtin_amdgcn_readlane(x, 31) +
               (uint32_t) __builtin_amdgcn_readlane(x, 47) + (uint32_t) __builtin_amdgcn_readlane(x, 63);
    }
}

// Combine one wave's share of a frame (`mine` of its nch body chunks, worth
// `sum` at the frame's end) into the frame's accumulator.  Returns true when
// this call completes the frame; `sum` then holds the frame total.
__device__ __forceinline__ bool frame_combine(uint32_t nch, uint32_t mine, unsigned long long *acc, uint32_t *cnt,
                                              uint64_t sum[5])
{
    if (mine == nch)
        return true; // the whole frame went through this wave
    // No fences: the partial sums and the chunk counter are agent-scope
    // atomics, performed at the one coherence point every XCD's atomics to
    // an address go through.  Each wave's adds have returned before its
    // counter add issues, so the wave whose counter add completes the count
    // finds every partial in acc, and reads them back with atomic adds of
    // zero.  (An acq_rel counter add here -- buffer_wbl2 of the XCD's L2 --
    // made frames spanning tiles 5x slower in round 1.)
    unsigned long long ret[5];
#pragma unroll
    for (int q = 0; q < 5; ++q)
        ret[q] = __hip_atomic_fetch_add(acc + q, (unsigned long long) sum[q], __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::"v"(ret[0]), "v"(ret[1]), "v"(ret[2]), "v"(ret[3]), "v"(ret[4]) : "memory");
    const uint32_t old = __hip_atomic_fetch_add(cnt, mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old + mine != nch)
        return false;
#pragma unroll
    for (int q = 0; q < 5; ++q)
        sum[q] = __hip_atomic_fetch_add(acc + q, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return true;
}

// =====================================================================
// decode
// =====================================================================
// The chunked path's head for one decode frame with a valid header whose
// stream exceeds the frame kernel's limit (called by the frame kernel on one
// lane; header failures never get here).
struct DecodeHead {
    const uint32_t *sid;
    const uint64_t *in_off;
    const uint32_t *wire_len;
    const uint8_t *in;
    const uint64_t *out_off;
    uint8_t *out;
    const DevSession *sessions;
    uint32_t max_sessions;
    BigRecords R;
    const uint8_t *zflags = nullptr;             // zmqg_decode_zmtp (frame_zbits)
    const unsigned long long *res_src = nullptr; // zmqg_decode_zmtp (frame_result_copy)
    unsigned long long *res_dst = nullptr;
    __device__ void operator()(uint32_t i, unsigned long long *list_ctr, uint64_t nbase) const;
};

__device__ void DecodeHead::operator()(uint32_t i, unsigned long long *list_ctr, uint64_t) const
{
    FrameHot *hot = R.hot;
    FramePow *pw = R.pw;
    FrameFin *fin = R.fin;
    uint32_t *powtab = R.powtab;
    unsigned long long *acc = R.acc;
    uint32_t *cnt = R.cnt;
    const uint32_t wl = wire_len[i];
    const uint32_t s = sid[i]; // (the frame kernel hands over known sessions only)
    const uint8_t *src = in + in_off[i];
    uint8_t *dst = out + out_off[i];
    // In-place decode with the payload at the frame's start (the reference's
    // memmove layout): the body's chunks run in parallel, and a chunk's output
    // 33 bytes below its input would overwrite ciphertext a neighbouring chunk
    // may not have read yet.  The body decodes to the wire position instead
    // (output byte = its own input byte) and k_post moves the payload down.
    const bool move = dst == src;
    if (move)
        dst += 33;
    uint32_t w[16];
    load_window(src, 64, w); // wl > kMaxFrameStream >= 64
    const uint32_t mlen = wl - 32;
    uint32_t nch, blast;
    body_geometry(mlen, nch, blast);
    const uint32_t p = list_append(list_ctr, R.chunk_end, R.list_frame, i, nch);
#pragma unroll
    for (int t = 0; t < 5; ++t)
        acc[(size_t) p * 5 + t] = 0;
    cnt[p] = 0;

    FrameHot H;
    FrameFin F;
    F.wire_len = wl;
    F.frame = i;
    F.pad = 0;
    H.status = 0;
    H.hl = 0;
    H.in_base = (uint64_t) (uintptr_t) src;
    H.out_base = (uint64_t) (uintptr_t) dst;
#pragma unroll
    for (int t = 0; t < 8; ++t)
        H.key[t] = sessions[s].dec_key[t];
    uint32_t ks[16];
    salsa20_block(ks, H.key, w[2], w[3], 0, 0);
    const fe r = poly_r_from_key(ks[0], ks[1], ks[2], ks[3]);
    uint32_t ct[16];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        ct[t] = w[8 + t];
        ct[8 + t] = 0;
    }
    fe h = fe_zero();
    const uint32_t s1 = r.l[1] * 5, s2 = r.l[2] * 5, s3 = r.l[3] * 5, s4 = r.l[4] * 5;
    poly_absorb64(h, r, s1, s2, s3, s4, ct, 32);
    uint32_t pt[16];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        pt[t] = ct[t] ^ ks[8 + t];
        pt[8 + t] = 0;
    }
    // payload bytes 0 .. 30 = plaintext bytes 1 .. 31 (speculative: zeroed
    // by the finisher or the replay fixup if the frame fails)
    uint32_t pay[16];
#pragma unroll
    for (int t = 0; t < 15; ++t)
        pay[t] = __builtin_amdgcn_alignbyte(pt[t + 1], pt[t], 1);
    pay[15] = 0;
    store_window(dst, 31, pay);

    fe hf;
    head_powers(r, nch, blast, pw + p, powtab + (size_t) p * kMaxPow * 5, hf);
    fe_mul(h, hf);
    store_fe(H.r, r);
    H.nch = nch;
    H.mlen = mlen;
    H.n0 = w[2];
    H.n1 = w[3];
    H.flags = (pt[0] & (ZMQG_MSG_MORE | ZMQG_MSG_COMMAND)) | (move ? kHotMove : 0u);
    store_fe(F.hh, h);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        F.s[t] = ks[4 + t];
        F.tag[t] = w[4 + t];
    }
    hot[p] = H;
    fin[p] = F;
}

__global__ void k_gather_u64(uint32_t n, const uint32_t *__restrict__ perm, const unsigned long long *__restrict__ src,
                             unsigned long long *__restrict__ dst)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n)
        dst[i] = src[perm[i]];
}

__global__ void k_scatter_replay(uint32_t n, const uint32_t *__restrict__ perm, const uint32_t *__restrict__ keys_s,
                                 const unsigned long long *__restrict__ excl_s, unsigned long long *__restrict__ excl,
                                 uint8_t *__restrict__ last)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    const uint32_t m = perm[i];
    excl[m] = excl_s[i];
    last[m] = (i + 1 == n || keys_s[i + 1] != keys_s[i]) ? 1 : 0;
}

// Replay rule of src/curve_mechanism_base.cpp:98-106 for a batch over
// several sessions, as if the frames were decoded one by one in batch
// order: a header-valid frame passes iff its nonce exceeds max(its session's
// peer nonce before the batch, every earlier header-valid nonce of that
// session in the batch) -- excl[i], computed by the replay tables below
// (k_replay_*); the peer nonce is set before the MAC check, so a MAC failure
// still advances it.  Small frames get INVALID_SEQUENCE, flags 0 and a
// zero-filled payload here (big frames in the body finisher, which runs
// before).  With `last` (the sort fallback), the last frame of each session
// also writes the session's new peer nonce; the tables write it themselves.
// (One session: the frame kernel does all of this.)
__global__ __launch_bounds__(kFixupThreads) void k_fixup(
    uint32_t n, uint32_t max_stream, const unsigned long long *__restrict__ vout,
    const unsigned long long *__restrict__ psnap, const unsigned long long *__restrict__ excl,
    const uint8_t *__restrict__ last, const uint32_t *__restrict__ sid, uint32_t max_sessions,
    const uint32_t *__restrict__ wire_len, const uint64_t *__restrict__ out_off, uint8_t *__restrict__ out,
    int32_t *__restrict__ status_out, uint8_t *__restrict__ flags_out, unsigned long long *__restrict__ peer,
    unsigned long long *__restrict__ smax)
{
    const uint32_t i = blockIdx.x * kFixupThreads + threadIdx.x;
    if (i >= n)
        return;
    const unsigned long long v = vout[i], ex = excl[i], ps = psnap[i];
    const unsigned long long prev = ex > ps ? ex : ps;
    const uint32_t wl = wire_len[i];
    const int32_t st = status_out[i];
    const bool header_ok = st == 0 || st == ZMQG_ERR_CRYPTOGRAPHIC || st == ZMQG_ERR_INVALID_SEQUENCE;
    if (header_ok && wl <= max_stream && !(v > prev) && st != ZMQG_ERR_INVALID_SEQUENCE) {
        status_out[i] = ZMQG_ERR_INVALID_SEQUENCE;
        flags_out[i] = 0;
        if (st == 0) // (a MAC failure is already zero-filled)
            zero_bytes(out + out_off[i], wl - 33u);
    }
    if (last && last[i] && sid[i] < max_sessions) {
        unsigned long long pn = prev, bm = ex;
        if (header_ok && v > pn)
            pn = v;
        if (header_ok && v > bm)
            bm = v;
        peer[sid[i]] = pn;
        if (smax)
            smax[sid[i]] = bm;
    }
}

// Header pass for sharded decode: per session, the
// largest header-valid nonce among n wire frames -- what a rank contributes to
// the exclusive max-scan over ranks (libzmq_amd/shard.py peer_prefix) before
// any rank decodes.  Header rule as the frame kernel's
// (src/mechanism_base.cpp:14-25, src/curve_mechanism_base.cpp:80-97).
__global__ __launch_bounds__(256) void k_session_max(uint32_t n, const uint32_t *__restrict__ sid,
                                                    const uint64_t *__restrict__ in_off,
                                                    const uint32_t *__restrict__ wire_len,
                                                    const uint8_t *__restrict__ in, uint32_t max_sessions,
                                                    unsigned long long *__restrict__ smax)
{
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n)
        return;
    const uint32_t L = wire_len[i], s = sid[i];
    if (s >= max_sessions || L < 33u)
        return;
    uint32_t h[16];
    load_window(in + in_off[i], 16, h);
    if (L <= (h[0] & 0xffu) || h[0] != 0x53454d07u || h[1] != 0x45474153u)
        return;
    const unsigned long long v = ((unsigned long long) bswap32(h[2]) << 32) | bswap32(h[3]);
    if (v)
        atomicMax(smax + s, v);
}

// ---------------------------------------------------------------- replay tables
// The exclusive max of header-valid nonces per session in batch order (the
// excl[] k_fixup and the body finisher read), for up to kReplayMaxSessions
// sessions, without sorting the batch (a 16 Mi-frame radix sort + segmented
// scan cost 1.1 ms):
//   k_replay_tiles    tile t of the batch (T frames): per-session maxima in an
//                     LDS table (ds_max_u64), written as row t of tab[tiles][S]
//   k_replay_colblk   per session and block of kReplayRB rows: the block max
//   k_replay_colscan  per session and row block: tab[t][s] := the exclusive
//                     max over rows < t (the prefix of the block maxima, then
//                     down the block); the last block also writes the
//                     session's new peer nonce and session max
//   k_replay_frames   one wave per tile walks its frames 64 at a time with the
//                     tile's prefix row in LDS: excl = table[sid] (plus, when
//                     a session repeats within the 64, the max of its earlier
//                     lanes), then table[sid] = max(table[sid], v)
constexpr uint32_t kReplayMaxSessions = 8192, kReplayRB = 64, kReplayMaxTiles = 4096;

__global__ __launch_bounds__(256) void k_replay_tiles(uint32_t n, uint32_t T, uint32_t S,
                                                     const uint32_t *__restrict__ sid,
                                                     const unsigned long long *__restrict__ vout,
                                                     unsigned long long *__restrict__ tab)
{
    extern __shared__ unsigned long long sh_tab[];
    for (uint32_t k = threadIdx.x; k < S; k += 256)
        sh_tab[k] = 0;
    __syncthreads();
    const uint64_t b = (uint64_t) blockIdx.x * T, e = b + T < n ? b + T : n;
    for (uint64_t i = b + threadIdx.x; i < e; i += 256) {
        const unsigned long long v = vout[i];
        const uint32_t s = sid[i];
        if (v && s < S)
            atomicMax(sh_tab + s, v);
    }
    __syncthreads();
    unsigned long long *row = tab + (size_t) blockIdx.x * S;
    for (uint32_t k = threadIdx.x; k < S; k += 256)
        row[k] = sh_tab[k];
}

__global__ __launch_bounds__(256) void k_replay_colblk(uint32_t tiles, uint32_t S,
                                                      const unsigned long long *__restrict__ tab,
                                                      unsigned long long *__restrict__ blk)
{
    const uint32_t s = blockIdx.x * 256 + threadIdx.x, rb = blockIdx.y;
    if (s >= S)
        return;
    const uint32_t r0 = rb * kReplayRB, r1 = r0 + kReplayRB < tiles ? r0 + kReplayRB : tiles;
    unsigned long long m = 0;
    for (uint32_t r = r0; r < r1; ++r) {
        const unsigned long long x = tab[(size_t) r * S + s];
        m = x > m ? x : m;
    }
    blk[(size_t) rb * S + s] = m;
}

__global__ __launch_bounds__(256) void k_replay_colscan(uint32_t tiles, uint32_t S,
                                                       unsigned long long *__restrict__ tab,
                                                       const unsigned long long *__restrict__ blk,
                                                       unsigned long long *__restrict__ peer,
                                                       unsigned long long *__restrict__ smax)
{
    const uint32_t s = blockIdx.x * 256 + threadIdx.x, rb = blockIdx.y;
    if (s >= S)
        return;
    unsigned long long m = 0;
    for (uint32_t k = 0; k < rb; ++k) {
        const unsigned long long x = blk[(size_t) k * S + s];
        m = x > m ? x : m;
    }
    const uint32_t r0 = rb * kReplayRB, r1 = r0 + kReplayRB < tiles ? r0 + kReplayRB : tiles;
    for (uint32_t r = r0; r < r1; ++r) {
        unsigned long long *p = tab + (size_t) r * S + s;
        const unsigned long long x = *p;
        *p = m;
        m = x > m ? x : m;
    }
    if (r1 == tiles) { // the session's batch total
        if (m > peer[s])
            peer[s] = m;
        if (smax)
            smax[s] = m;
    }
}

__global__ __launch_bounds__(64) void k_replay_frames(uint32_t n, uint32_t T, uint32_t S,
                                                     const uint32_t *__restrict__ sid,
                                                     const unsigned long long *__restrict__ vout,
                                                     const unsigned long long *__restrict__ tab,
                                                     unsigned long long *__restrict__ excl)
{
    extern __shared__ unsigned long long sh_tab[]; // [S] running maxima, then [S] u32 lane tags
    uint32_t *const tag = (uint32_t *) (sh_tab + S);
    const uint32_t lane = threadIdx.x;
    const unsigned long long *row = tab + (size_t) blockIdx.x * S;
    for (uint32_t k = lane; k < S; k += 64)
        sh_tab[k] = row[k];
    __syncthreads();
    const uint64_t b = (uint64_t) blockIdx.x * T, e = b + T < n ? b + T : n;
    for (uint64_t i0 = b; i0 < e; i0 += 64) {
        const uint64_t i = i0 + lane;
        const bool ok = i < e;
        const uint32_t s = ok ? sid[i] : S;
        const unsigned long long v = ok ? vout[i] : 0ull;
        const bool in = ok && s < S;
        unsigned long long x = in ? sh_tab[s] : 0ull;
        // a session twice among these 64 frames: its earlier lanes count too
        if (in)
            tag[s] = lane;
        __builtin_amdgcn_wave_barrier();
        const bool dup = in && tag[s] != lane;
        if (__builtin_amdgcn_ballot_w64(dup) != 0) {
            // one repeated session per round: the max over its earlier lanes
            // (an inclusive max-scan of its lanes' values, shifted by one)
            unsigned long long left = __builtin_amdgcn_ballot_w64(in);
            while (left) {
                const uint32_t lead = (uint32_t) __builtin_ctzll(left);
                const uint32_t sl = (uint32_t) __builtin_amdgcn_readlane((int) s, (int) lead);
                const bool mem = in && s == sl;
                const unsigned long long m = __builtin_amdgcn_ballot_w64(mem);
                left &= ~m;
                if ((m & (m - 1)) == 0)
                    continue; // one lane: nothing earlier in this group
                unsigned long long c = mem ? v : 0ull;
#pragma unroll
                for (uint32_t d = 1; d < 64; d <<= 1) {
                    const unsigned long long u = __shfl_up(c, d);
                    if (lane >= d && u > c)
                        c = u;
                }
                const unsigned long long ex = __shfl_up(c, 1);
                if (mem && lane > 0 && ex > x)
                    x = ex;
            }
        }
        if (ok)
            excl[i] = x;
        __builtin_amdgcn_wave_barrier();
        if (in && v)
            atomicMax(sh_tab + s, v);
        __builtin_amdgcn_wave_barrier();
    }
}

// ---------------------------------------------------------------- send nonces
// ZMQG_OPT_NONCE_AUTO over several sessions: frame i of session s takes
// send[s] + (frames of s before i in the batch), and send[s] advances by the
// session's frame count -- get_and_inc_nonce per message in batch order
// (src/curve_mechanism_base.hpp:41).  Same tile tables as the replay prefix,
// with counts and sums in place of maxima:
//   k_nonce_tiles    per tile, per-session frame counts -> tab[t][s]
//   k_nonce_colblk   per session and block of kReplayRB rows: the block sum
//   k_nonce_colscan  tab[t][s] := send[s] + frames of s in tiles < t; the last
//                    block advances send[s]
//   k_nonce_frames   one wave per tile: nonce = tab[t][sid] + earlier frames
//                    of the session in the tile (lanes grouped by session
//                    with ballots, 64 frames at a time)
__global__ __launch_bounds__(256) void k_nonce_tiles(uint32_t n, uint32_t T, uint32_t S,
                                                    const uint32_t *__restrict__ sid,
                                                    unsigned long long *__restrict__ tab)
{
    extern __shared__ unsigned long long sh_tab[];
    uint32_t *const cnt = (uint32_t *) sh_tab;
    for (uint32_t k = threadIdx.x; k < S; k += 256)
        cnt[k] = 0;
    __syncthreads();
    const uint64_t b = (uint64_t) blockIdx.x * T, e = b + T < n ? b + T : n;
    for (uint64_t i = b + threadIdx.x; i < e; i += 256) {
        const uint32_t s = sid[i];
        if (s < S)
            atomicAdd(cnt + s, 1u);
    }
    __syncthreads();
    unsigned long long *row = tab + (size_t) blockIdx.x * S;
    for (uint32_t k = threadIdx.x; k < S; k += 256)
        row[k] = cnt[k];
}

__global__ __launch_bounds__(256) void k_nonce_colblk(uint32_t tiles, uint32_t S,
                                                     const unsigned long long *__restrict__ tab,
                                                     unsigned long long *__restrict__ blk,
                                                     const unsigned long long *__restrict__ send,
                                                     unsigned long long *__restrict__ snap)
{
    const uint32_t s = blockIdx.x * 256 + threadIdx.x, rb = blockIdx.y;
    if (s >= S)
        return;
    if (rb == 0) // the send counters as they were before this call, for k_nonce_colscan
        snap[s] = send[s];
    const uint32_t r0 = rb * kReplayRB, r1 = r0 + kReplayRB < tiles ? r0 + kReplayRB : tiles;
    unsigned long long m = 0;
    for (uint32_t r = r0; r < r1; ++r)
        m += tab[(size_t) r * S + s];
    blk[(size_t) rb * S + s] = m;
}

__global__ __launch_bounds__(256) void k_nonce_colscan(uint32_t tiles, uint32_t S, unsigned long long *__restrict__ tab,
                                                      const unsigned long long *__restrict__ blk,
                                                      const unsigned long long *__restrict__ snap,
                                                      unsigned long long *__restrict__ send)
{
    const uint32_t s = blockIdx.x * 256 + threadIdx.x, rb = blockIdx.y;
    if (s >= S)
        return;
    // the base comes from the snapshot k_nonce_colblk took: the last row
    // block advances send[s] below, and nothing orders that store against
    // the other row blocks of this launch
    unsigned long long m = snap[s];
    for (uint32_t k = 0; k < rb; ++k)
        m += blk[(size_t) k * S + s];
    const uint32_t r0 = rb * kReplayRB, r1 = r0 + kReplayRB < tiles ? r0 + kReplayRB : tiles;
    for (uint32_t r = r0; r < r1; ++r) {
        unsigned long long *p = tab + (size_t) r * S + s;
        const unsigned long long x = *p;
        *p = m;
        m += x;
    }
    if (r1 == tiles) // (no block of this launch reads send[s])
        send[s] = m;
}

__global__ __launch_bounds__(64) void k_nonce_frames(uint32_t n, uint32_t T, uint32_t S,
                                                    const uint32_t *__restrict__ sid,
                                                    const unsigned long long *__restrict__ tab,
                                                    uint64_t *__restrict__ nonce)
{
    extern __shared__ unsigned long long sh_tab[]; // [S] the next nonce of each session
    const uint32_t lane = threadIdx.x;
    const unsigned long long *row = tab + (size_t) blockIdx.x * S;
    for (uint32_t k = lane; k < S; k += 64)
        sh_tab[k] = row[k];
    __syncthreads();
    const unsigned long long below = (1ull << lane) - 1ull;
    const uint64_t b = (uint64_t) blockIdx.x * T, e = b + T < n ? b + T : n;
    for (uint64_t i0 = b; i0 < e; i0 += 64) {
        const uint64_t i = i0 + lane;
        const bool in = i < e && sid[i] < S;
        const uint32_t s = in ? sid[i] : 0u;
        unsigned long long left = __builtin_amdgcn_ballot_w64(in);
        uint64_t v = 0;
        while (left) { // one session per round: its lanes, in lane (= batch) order
            const uint32_t lead = (uint32_t) __builtin_ctzll(left);
            const uint32_t sl = (uint32_t) __builtin_amdgcn_readlane((int) s, (int) lead);
            const unsigned long long m = __builtin_amdgcn_ballot_w64(in && s == sl);
            const unsigned long long base = sh_tab[sl];
            if (in && s == sl)
                v = base + (unsigned long long) __builtin_popcountll(m & below);
            __builtin_amdgcn_wave_barrier();
            if (lane == lead)
                sh_tab[sl] = base + (unsigned long long) __builtin_popcountll(m);
            __builtin_amdgcn_wave_barrier();
            left &= ~m;
        }
        if (i < e)
            nonce[i] = v;
    }
}

// ---------------------------------------------------------------- body
// One lane per chunk (2 Salsa20 blocks = 128 stream bytes = 8 Poly1305
// blocks); a tile is 64 consecutive chunks, one wave's worth, so a tile's
// input and output are each one (nearly) contiguous 8 KiB stream.  The
// kernel is persistent with two waves per SIMD (two workgroups of 4 waves
// per CU), and each wave walks a contiguous run of tiles as a two-stage
// software pipeline, so its HBM traffic for tile t+1 is in flight while it
// computes tile t (and the other wave on the SIMD covers the rest):
//
//   wait    s_waitcnt vmcnt(0): tile t's input is in LDS buffer t&1
//   issue   tile t+1's frame records, tile t+2's chunk-end window
//   compute window 0 of tile t (LDS only)
//   setup   tile t+1 (params, chunk factors) and its LDS-DMA into buffer ~t&1
//   compute window 1 of tile t
//   store   tile t's output image (coalesced granules + per-lane edges)
//   finish  Poly1305 segment sums, tags / status of the frames ending here
//
// Staging through LDS keeps every global access a coalesced, aligned
// 16-byte granule stream (a chunk's granules go to consecutive lanes):
//   1. LDS-DMA (global_load_lds_dwordx4): input granule q of chunk s lands
//      at slot s + 16q, slot = 144 bytes (9 granules), lane-linear.
//   2. each lane works on its own slot: stream byte b is at slot + (src&15)
//      + b; the output image (stream byte b at slot + (dst&15) + b) is
//      written in place, one window behind the input it has already read.
//   3. interior output granules go back with coalesced dwordx4 stores;
//      each lane then stores its own (at most two) edge granules, merging
//      the granule it shares with the next chunk of the same frame.
// Chunk parameters for the cooperative DMA/store rounds come from the
// owning lane by ds_bpermute, so LDS holds nothing but the two tile images.
constexpr int kSlotG = 9;
constexpr int kSlot = 16 * kSlotG;
constexpr int kBufLds = 64 * kSlot; // one tile image, 9 KiB
constexpr int kBodyWaves = kBodyThreads / 64;
constexpr int kBodyWgPerCu = 2;
static_assert(kBodyWgPerCu * kBodyWaves * 2 * kBufLds <= 160 * 1024, "two tile buffers per wave must fit");

typedef __attribute__((address_space(3))) void LdsVoid;
typedef __attribute__((address_space(1))) void GVoid;

__device__ __forceinline__ void wave_lds_fence()
{
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}

// bytes [lo, hi) of granule v at the 16-byte aligned address p
__device__ __forceinline__ void store_granule_range(GU8 *p, int lo, int hi, const u32x4 &v)
{
    const uint32_t o[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int a = lo > 4 * k ? lo : 4 * k;
        const int b = hi < 4 * k + 4 ? hi : 4 * k + 4;
        if (a == 4 * k && b == 4 * k + 4) {
            *(GU32 *) (p + 4 * k) = o[k];
        } else {
#pragma unroll
            for (int t = 0; t < 4; ++t)
                if (4 * k + t >= a && 4 * k + t < b)
                    p[4 * k + t] = (uint8_t) (o[k] >> (8 * t));
        }
    }
}

__device__ __forceinline__ uint32_t byte_mask_below(int e, int k) // bytes [4k, 4k+4) below e
{
    const int b = e - 4 * k;
    return b >= 4 ? 0xffffffffu : (b <= 0 ? 0u : ((1u << (8 * b)) - 1u));
}

// The frame records a lane of the next tile loads (one batch of independent
// dwordx4 loads, issued a compute window before they are used).  Kept as
// raw granules so that nothing here becomes a private-memory copy.
struct TileRecords {
    u32x4 h[6]; // FrameHot
    u32x4 p[9]; // FramePow
};
static_assert(sizeof(FrameHot) == 6 * 16 && sizeof(FramePow) == 9 * 16, "records");

// Unconditional loads (an idle lane reads frame 0's records and ignores
// them): a conditional load would need a register copy at the branch join,
// and that copy waits for the load.
__device__ __forceinline__ void load_records(TileRecords &R, uint32_t i, const FrameHot *__restrict__ hot,
                                             const FramePow *__restrict__ pw)
{
    const GCU4 *ph = (const GCU4 *) (hot + i), *pp = (const GCU4 *) (pw + i);
#pragma unroll
    for (int q = 0; q < 6; ++q)
        R.h[q] = ph[q];
#pragma unroll
    for (int q = 0; q < 9; ++q)
        R.p[q] = pp[q];
}

template <int W>
__device__ __forceinline__ uint32_t rec_word(const u32x4 *g)
{
    return (W & 3) == 0 ? g[W >> 2].x : (W & 3) == 1 ? g[W >> 2].y : (W & 3) == 2 ? g[W >> 2].z : g[W >> 2].w;
}

template <int W>
__device__ __forceinline__ fe rec_fe(const u32x4 *g)
{
    fe x;
    x.l[0] = rec_word<W>(g);
    x.l[1] = rec_word<W + 1>(g);
    x.l[2] = rec_word<W + 2>(g);
    x.l[3] = rec_word<W + 3>(g);
    x.l[4] = rec_word<W + 4>(g);
    return x;
}

// Per-lane state of one tile from its setup to its finish (plain words only).
struct TileLane {
    uint32_t key; // frame index, kIdle past the batch's last chunk
    uint32_t g0;  // the frame's first chunk
    uint32_t c;   // chunk index within the frame
    uint32_t L;   // stream bytes of this chunk (0 = nothing to do)
    uint32_t Ln;  // L of the next lane
    uint32_t di;  // input stream byte 0 within its granule
    uint32_t cont, prevcont;
    uint64_t dst; // output stream byte 0
    uint32_t P[5]; // r^(Poly1305 blocks of the later chunks of this chunk's frame segment in the tile)
    uint32_t sig;  // what P was computed for: later chunks | 64 when they include the frame's last
    uint32_t k[8], n0, n1, r[5], nch, flags; // from FrameHot
    int32_t status;
    uint64_t out_base;
};

// Sets up tile lane T from its frame's records and returns the chunk's
// input stream address (for the DMA).  `prev` is the wave's previous tile
// (its segment powers are reused when the tile has the same frame layout);
// `fresh` forces them to be computed.
template <bool DEC>
__device__ __forceinline__ uint64_t tile_setup(TileLane &T, const TileRecords &R, bool valid, const FrameLook &lk,
                                               uint32_t g, const TileLane &prev, bool fresh)
{
    const uint32_t lane = threadIdx.x & 63;
    // every loaded granule counts as used from here on: a record word that
    // is never read would free its register while the load is in flight,
    // and the next write to that register would wait for the load
#pragma unroll
    for (int q = 0; q < 6; ++q)
        asm volatile("" ::"v"(R.h[q]));
#pragma unroll
    for (int q = 0; q < 9; ++q)
        asm volatile("" ::"v"(R.p[q]));
    // FrameHot words: key 0-7, r 8-12, nch 13, mlen 14, hl 15, n0 16, n1 17,
    // status 18, flags 19, in_base 20-21, out_base 22-23
    T.k[0] = rec_word<0>(R.h);
    T.k[1] = rec_word<1>(R.h);
    T.k[2] = rec_word<2>(R.h);
    T.k[3] = rec_word<3>(R.h);
    T.k[4] = rec_word<4>(R.h);
    T.k[5] = rec_word<5>(R.h);
    T.k[6] = rec_word<6>(R.h);
    T.k[7] = rec_word<7>(R.h);
    T.r[0] = rec_word<8>(R.h);
    T.r[1] = rec_word<9>(R.h);
    T.r[2] = rec_word<10>(R.h);
    T.r[3] = rec_word<11>(R.h);
    T.r[4] = rec_word<12>(R.h);
    T.nch = rec_word<13>(R.h);
    const uint32_t mlen = rec_word<14>(R.h), hl = rec_word<15>(R.h);
    T.n0 = rec_word<16>(R.h);
    T.n1 = rec_word<17>(R.h);
    T.status = (int32_t) rec_word<18>(R.h);
    T.flags = rec_word<19>(R.h);
    const uint64_t in_base = ((uint64_t) rec_word<21>(R.h) << 32) | rec_word<20>(R.h);
    T.out_base = ((uint64_t) rec_word<23>(R.h) << 32) | rec_word<22>(R.h);

    uint64_t src = 0;
    T.key = kIdle;
    T.g0 = 0;
    T.c = 0;
    T.L = 0;
    T.dst = 0;
    T.di = 0;
    if (valid) {
        const uint32_t i = lk.i;
        T.key = i;
        T.g0 = lk.ce - T.nch; // chunk_end[i - 1]
        T.c = g - T.g0;
        const uint32_t P0 = 32 + kChunk * T.c; // first plaintext byte of this chunk
        uint32_t L = mlen > P0 ? (mlen - P0 < kChunk ? mlen - P0 : kChunk) : 0;
        if (DEC) {
            if (T.status != 0)
                L = 0;
            src = in_base + 32 + P0;     // ciphertext byte P0 on the wire
            T.dst = T.out_base + P0 - 1; // plaintext byte P0 = payload byte P0-1
        } else {
            src = in_base + (P0 - hl);    // payload byte = plaintext byte - hl
            T.dst = T.out_base + 32 + P0; // wire ciphertext
        }
        T.L = L;
        T.di = (uint32_t) (src & 15);
    }
    const uint32_t kn = __shfl_down(T.key, 1);
    T.Ln = __shfl_down(T.L, 1);
    T.cont = (lane < 63 && T.key != kIdle && kn == T.key && T.L == kChunk && T.Ln > 0) ? 1u : 0u;
    T.prevcont = (__shfl_up(T.cont, 1) != 0 && lane > 0) ? 1u : 0u;

    // Segment power: the lanes of one frame in this tile form a segment
    // [first, e]; lane l's Horner value is worth r^(Poly1305 blocks of chunks
    // l+1 .. e) at the segment's end: 8 per chunk, the frame's last chunk
    // blast (FramePow.rb).  A wave inside one frame keeps the same powers
    // tile after tile, so they are computed only when the layout changes.
    const uint32_t kp = __shfl_up(T.key, 1);
    const uint64_t bnd = __ballot(T.key == kIdle || lane == 0 || kp != T.key);
    const uint64_t above = lane == 63 ? 0ull : (bnd >> (lane + 1)) << (lane + 1);
    const uint32_t e = above ? (uint32_t) __builtin_ctzll(above) - 1u : 63u;
    uint32_t sig = kIdle;
    if (T.key != kIdle) {
        const bool last = T.c + (e - lane) + 1 == T.nch && e > lane; // the segment's last chunk ends the frame
        sig = (e - lane - (last ? 1u : 0u)) | (last ? 64u : 0u);
    }
    T.sig = sig;
    if (fresh || __any(sig != prev.sig || T.key != prev.key)) {
        // FramePow words: rb 0-4, t[k] = r^(8*2^k) at 5+5k
        static_assert(kPowInline == 6, "segment powers use r^(8*2^k), k < 6");
        fe P = fe_one();
        if (sig != kIdle) {
            if (sig & 64)
                P = rec_fe<0>(R.p);
            if (sig & 1)
                fe_mul(P, rec_fe<5>(R.p));
            if (sig & 2)
                fe_mul(P, rec_fe<10>(R.p));
            if (sig & 4)
                fe_mul(P, rec_fe<15>(R.p));
            if (sig & 8)
                fe_mul(P, rec_fe<20>(R.p));
            if (sig & 16)
                fe_mul(P, rec_fe<25>(R.p));
            if (sig & 32)
                fe_mul(P, rec_fe<30>(R.p));
        }
#pragma unroll
        for (int q = 0; q < 5; ++q)
            T.P[q] = P.l[q];
    } else {
#pragma unroll
        for (int q = 0; q < 5; ++q)
            T.P[q] = prev.P[q];
    }
    return src;
}

// r^(Poly1305 blocks after chunk c of list frame p) = r^blast * (r^8)^(nch-2-c)
// (c < nch - 1), from the frame's records.
__device__ fe frame_after_power(const FramePow *__restrict__ pw, const uint32_t *__restrict__ powtab, uint32_t p,
                                uint32_t nch, uint32_t c)
{
    const uint32_t *P = (const uint32_t *) (pw + p);
    fe f = load_fe(P);
    const uint32_t m = nch - 2 - c;
    for (int k = 0; (m >> k) != 0; ++k)
        if ((m >> k) & 1)
            fe_mul(f, load_fe(k < kPowInline ? P + 5 + 5 * k : powtab + (size_t) p * kMaxPow * 5 + 5 * k));
    return f;
}

// Chunk parameters of the cooperative rounds: in round k lane l moves
// granule q of chunk s, idx = 64k + l = kSlotG*s + q.  The rounds go in
// groups of kGroup: the group's chunk addresses and lengths are fetched from
// the owning lanes (ds_bpermute) together, so the rounds are not serialised
// on LDS latency, while the registers they need stay bounded.
constexpr uint32_t kGroup = 3;
static_assert(kSlotG % kGroup == 0, "round groups");

struct RoundParams {
    uint64_t a[kGroup]; // chunk stream byte 0 (input or output)
    uint32_t L[kGroup]; // chunk stream bytes
    uint32_t q[kGroup]; // granule of the chunk this lane moves
};

__device__ __forceinline__ void round_params(RoundParams &P, uint32_t k0, uint64_t addr, uint32_t L)
{
    uint32_t ln = threadIdx.x & 63;
    asm volatile("" : "+v"(ln)); // keep the round arithmetic out of the loop-invariant set
    const uint32_t alo = (uint32_t) addr, ahi = (uint32_t) (addr >> 32);
#pragma unroll
    for (uint32_t j = 0; j < kGroup; ++j) {
        const uint32_t idx = (k0 + j) * 64 + ln, s = idx / kSlotG;
        P.q[j] = idx - kSlotG * s;
        P.a[j] = ((uint64_t) (uint32_t) __shfl(ahi, (int) s) << 32) | (uint32_t) __shfl(alo, (int) s);
        P.L[j] = (uint32_t) __shfl(L, (int) s);
    }
}

// A uniform tile: 64 whole chunks of one frame, chunk s at a0 + 128 s (input
// and output alike).  Its rounds need no per-chunk parameters: round k of
// lane l moves granule q of chunk s, 64k + l = 9s + q, which sits 128s + 16q =
// 16(64k + l - s) bytes after the tile's first granule -- a per-lane constant
// (UniRounds, computed once per wave).  q = 8 is the granule past a chunk's
// 128 bytes: it holds input only when the tile is misaligned, and on output
// it (like q = 0 when misaligned) is an edge granule its lane stores.
struct UniRounds {
    uint32_t o[5]; // the offsets of rounds 2i (low half) and 2i+1 (high half)
    uint32_t f;    // bit k: q = 8 in round k; bit 16 + k: q = 0
};

__device__ __forceinline__ UniRounds uni_rounds()
{
    UniRounds U = {{0, 0, 0, 0, 0}, 0};
    const uint32_t lane = threadIdx.x & 63;
#pragma unroll
    for (uint32_t k = 0; k < kSlotG; ++k) {
        const uint32_t idx = 64 * k + lane, s = idx / kSlotG, q = idx - kSlotG * s;
        U.o[k >> 1] |= (16 * (idx - s)) << (16 * (k & 1));
        U.f |= (q == kSlotG - 1 ? 1u << k : 0u) | (q == 0 ? 1u << (16 + k) : 0u);
    }
    return U;
}

template <uint32_t K>
__device__ __forceinline__ uint32_t uni_off(const UniRounds &U)
{
    return (K & 1) ? U.o[K >> 1] >> 16 : U.o[K >> 1] & 0xffffu;
}

// LDS-DMA of a uniform tile's input (a0 = chunk 0's first stream byte).
__device__ __forceinline__ void tile_dma_uni(uint8_t *buf, uint64_t a0, const UniRounds &U)
{
    const uint32_t off = (uint32_t) a0 & 15u;
    const GU8 *base = (const GU8 *) (uintptr_t) (a0 - off);
    const bool all9 = off != 0; // (an aligned chunk's 128 bytes are 8 granules)
#define ZMQG_UNI_DMA(K)                                                                                         \
    if (all9 || !((U.f >> (K)) & 1u))                                                                            \
        __builtin_amdgcn_global_load_lds((GVoid *) (base + uni_off<K>(U)), (LdsVoid *) (buf + 1024 * (K)), 16, 0, 0);
    ZMQG_UNI_DMA(0) ZMQG_UNI_DMA(1) ZMQG_UNI_DMA(2) ZMQG_UNI_DMA(3) ZMQG_UNI_DMA(4)
    ZMQG_UNI_DMA(5) ZMQG_UNI_DMA(6) ZMQG_UNI_DMA(7) ZMQG_UNI_DMA(8)
#undef ZMQG_UNI_DMA
}

// Interior output granules of a uniform tile (d0 = chunk 0's first output byte).
__device__ __forceinline__ void tile_store_uni(const uint8_t *buf, uint64_t d0, const UniRounds &U)
{
    const uint32_t pO = (uint32_t) d0 & 15u;
    GU8 *base = (GU8 *) (uintptr_t) (d0 - pO);
    const uint32_t skip = (U.f & 0x1ffu) | (pO ? U.f >> 16 : 0u); // edge granules: their lanes store them
    const uint8_t *lb = buf + 16 * (threadIdx.x & 63);
#define ZMQG_UNI_ST(K)                                                 \
    {                                                                   \
        const u32x4 g = *(const u32x4 *) (lb + 1024 * (K));             \
        if (!((skip >> (K)) & 1u))                                      \
            *(GU4 *) (base + uni_off<K>(U)) = g;                        \
    }
    ZMQG_UNI_ST(0) ZMQG_UNI_ST(1) ZMQG_UNI_ST(2) ZMQG_UNI_ST(3) ZMQG_UNI_ST(4)
    ZMQG_UNI_ST(5) ZMQG_UNI_ST(6) ZMQG_UNI_ST(7) ZMQG_UNI_ST(8)
#undef ZMQG_UNI_ST
}

// Whether the tile is uniform, and its chunk 0 address.
__device__ __forceinline__ bool tile_uniform(uint32_t key, uint32_t L, uint64_t addr, uint64_t &a0)
{
    const uint32_t k0 = __builtin_amdgcn_readfirstlane(key);
    // (the builtin returns int: each half is taken as uint32_t before widening)
    a0 = ((uint64_t) (uint32_t) __builtin_amdgcn_readfirstlane((uint32_t) (addr >> 32)) << 32) |
         (uint32_t) __builtin_amdgcn_readfirstlane((uint32_t) addr);
    return __all(key == k0 && k0 != kIdle && L == kChunk);
}

// Coalesced LDS-DMA of a tile's input images into buf (no wait).
__device__ __forceinline__ void tile_dma(uint8_t *buf, uint64_t src, uint32_t L)
{
#pragma unroll
    for (uint32_t k0 = 0; k0 < kSlotG; k0 += kGroup) {
        RoundParams P;
        round_params(P, k0, src, L);
#pragma unroll
        for (uint32_t j = 0; j < kGroup; ++j) {
            const uint32_t off = (uint32_t) (P.a[j] & 15);
            if (P.L[j] && P.q[j] < ((off + P.L[j] + 15) >> 4))
                __builtin_amdgcn_global_load_lds((GVoid *) (uintptr_t) ((P.a[j] - off) + 16 * P.q[j]),
                                                 (LdsVoid *) (buf + 1024 * (k0 + j)), 16, 0, 0);
        }
    }
}

// Coalesced stores of a tile's interior output granules from buf: the
// whole granules of each chunk's output image (an edge granule, shared with
// a neighbour or partial, is stored by its lane).
__device__ __forceinline__ void tile_store_interior(const uint8_t *buf, uint64_t dst, uint32_t L)
{
#pragma unroll
    for (uint32_t k0 = 0; k0 < kSlotG; k0 += kGroup) {
        RoundParams P;
        round_params(P, k0, dst, L);
        u32x4 g[kGroup];
#pragma unroll
        for (uint32_t j = 0; j < kGroup; ++j)
            g[j] = *(const u32x4 *) (buf + 16 * ((k0 + j) * 64 + (threadIdx.x & 63)));
#pragma unroll
        for (uint32_t j = 0; j < kGroup; ++j) {
            const uint32_t pO = (uint32_t) (P.a[j] & 15);
            const uint32_t qfirst = pO ? 1u : 0u;                         // granule 0 is an edge when misaligned
            if (P.L[j] && P.q[j] >= qfirst && 16 * P.q[j] + 16 <= pO + P.L[j]) // whole granule inside the chunk
                *(GU4 *) (uintptr_t) ((P.a[j] - pO) + 16 * P.q[j]) = g[j];
        }
    }
}

// ---------------------------------------------------------------- post
// Decode, after the body kernel: the post list's zero fills and in-place
// moves, spread over the whole grid.  An entry of len bytes is cut into
// segments (64 KiB, or len/kPostSegs for longer moves) and segment j of
// entry e goes to workgroup (j + e) mod grid, so one long entry uses the
// whole chip and many short ones spread out.
//
// Move (dst = src - 33, overlapping): a segment reads its source in 4 KiB
// rounds in ascending order and writes each round after the whole workgroup
// has read it, so it only overwrites bytes it has read itself -- except that
// its first 33 destination bytes are the previous segment's last 33 source
// bytes, which another workgroup may not have read yet.  Those 33 bytes are
// saved to the frame's scratch (the body's power table, dead by now) and
// written by the last workgroup to finish.
constexpr uint32_t kPostSeg = 64 * 1024, kPostSegs = 12, kPostRound = 4096;
static_assert(kPostSegs * 36 <= kMaxPow * 5 * 4, "seam bytes fit the frame's power-table entry");

__device__ __forceinline__ uint64_t post_seg_len(const PostOp &o)
{
    if (o.kind != kPostMove)
        return kPostSeg;
    const uint64_t per = (o.len + kPostSegs - 1) / kPostSegs;
    const uint64_t r = (per + kPostRound - 1) / kPostRound * kPostRound;
    return r > kPostSeg ? r : kPostSeg;
}

// Workgroup zero fill of [p, p+len): dwordx4 stores, byte edges.
__device__ void wg_zero(uint8_t *p, uint64_t len)
{
    const uint64_t a = (uint64_t) (uintptr_t) p, e = a + len;
    const uint64_t a16 = (a + 15) & ~15ull, e16 = e & ~15ull;
    if (a16 >= e16) {
        for (uint64_t x = a + threadIdx.x; x < e; x += blockDim.x)
            *(GU8 *) (uintptr_t) x = 0;
        return;
    }
    if (threadIdx.x < a16 - a)
        *(GU8 *) (uintptr_t) (a + threadIdx.x) = 0;
    if (threadIdx.x < e - e16)
        *(GU8 *) (uintptr_t) (e16 + threadIdx.x) = 0;
    const u32x4 z = {0, 0, 0, 0};
    for (uint64_t x = a16 + 16ull * threadIdx.x; x < e16; x += 16ull * blockDim.x)
        *(GU4 *) (uintptr_t) x = z;
}

// Destination bytes [d0, d1) of a move by 33 (source = destination + 33),
// ascending 4 KiB rounds, each read by the workgroup before it writes.
__device__ void wg_move33(uint64_t d0, uint64_t d1)
{
    for (uint64_t r0 = d0; r0 < d1; r0 += kPostRound) {
        const uint64_t r1 = r0 + kPostRound < d1 ? r0 + kPostRound : d1;
        // thread t: destination bytes [r0 + 16t, +16) of the round
        const uint64_t x = r0 + 16ull * threadIdx.x;
        uint8_t b[16];
        const uint32_t nb = x < r1 ? (uint32_t) (r1 - x < 16 ? r1 - x : 16) : 0u;
#pragma unroll
        for (int k = 0; k < 16; ++k)
            b[k] = (uint32_t) k < nb ? *(const GU8 *) (uintptr_t) (x + 33 + k) : 0;
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 16; ++k)
            if ((uint32_t) k < nb)
                *(GU8 *) (uintptr_t) (x + k) = b[k];
        __syncthreads();
    }
}

__global__ __launch_bounds__(256) void k_post(ZState *__restrict__ zs, const PostOp *__restrict__ post,
                                              uint8_t *__restrict__ seam)
{
    const uint32_t np = zs->post_n; // appended by the kernels before this one (stream order)
    if (np == 0)
        return; // nothing listed: no fence, no counter (post_done stays 0)
    const uint32_t G = gridDim.x;
    for (uint32_t e = 0; e < np; ++e) {
        const PostOp o = post[e];
        const uint64_t seg = post_seg_len(o);
        const uint64_t nseg = (o.len + seg - 1) / seg;
        for (uint64_t j = (blockIdx.x + G - e % G) % G; j < nseg; j += G) {
            const uint64_t a = j * seg, b = a + seg < o.len ? a + seg : o.len;
            if (o.kind == kPostZero) {
                wg_zero((uint8_t *) (uintptr_t) (o.dst + a), b - a);
            } else {
                // segment j > 0: its first 33 destination bytes wait for the seam pass
                uint64_t w0 = o.dst + a;
                if (j > 0) {
                    const uint64_t ns = b - a < 33 ? b - a : 33;
                    if (threadIdx.x < ns)
                        seam[(size_t) o.p * (kMaxPow * 5 * 4) + 36 * j + threadIdx.x] =
                            *(const GU8 *) (uintptr_t) (w0 + 33 + threadIdx.x);
                    __syncthreads();
                    w0 += ns;
                }
                wg_move33(w0, o.dst + b);
            }
        }
    }
    // the last workgroup: the seams (every segment has read its source), reset
    __shared__ uint32_t sh_last;
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        const uint32_t d = __hip_atomic_fetch_add(&zs->post_done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        sh_last = d + 1u == G;
        if (sh_last)
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
    if (!sh_last)
        return;
    for (uint32_t e = 0; e < np; ++e) {
        const PostOp o = post[e];
        if (o.kind != kPostMove)
            continue;
        const uint64_t seg = post_seg_len(o);
        const uint64_t nseg = (o.len + seg - 1) / seg;
        for (uint64_t t = threadIdx.x; t < (nseg - 1) * 36; t += blockDim.x) {
            const uint64_t j = 1 + t / 36, k = t % 36;
            const uint64_t a = j * seg;
            if (k < 33 && a + k < o.len)
                *(GU8 *) (uintptr_t) (o.dst + a + k) = seam[(size_t) o.p * (kMaxPow * 5 * 4) + 36 * j + k];
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        __hip_atomic_store(&zs->post_n, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&zs->post_done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// The big-frame list (positions 0 .. n-1, built by the frame kernel's head
// calls) is read from the call state: n = entries, total = body chunks.
template <bool DEC>
// Issue priority by phase, as in k_frames_lds (curve_frames_lds.hpp): 3 while
// a wave issues a tile's loads, DMA and stores, 0 over its keystream, MAC and
// finish.  Configs 3 / 5 on one box, two alternating rounds: 538 / 534 and
// 590.5 / 590.2 GiB/s against 527 / 528 and 586 / 588 without (the body
// kernel already keeps the SIMDs' VALU ~98 % busy at config 5).
#ifndef ZMQG_BODY_PRIO
#define ZMQG_BODY_PRIO 1 // 0: no priorities
#endif
#define BODY_PRIO(lv)                                                                                  \
    do {                                                                                               \
        if (ZMQG_BODY_PRIO)                                                                            \
            __builtin_amdgcn_s_setprio(lv);                                                            \
    } while (0)
__global__ __launch_bounds__(kBodyThreads) __attribute__((amdgpu_waves_per_eu(2))) void k_body(
    ZState *__restrict__ zs, const uint32_t *__restrict__ chunk_end,
    const FrameHot *__restrict__ hot, const FramePow *__restrict__ pw, const FrameFin *__restrict__ fin,
    const uint32_t *__restrict__ powtab, uint8_t *__restrict__ flags_out, int32_t *__restrict__ status_out,
    unsigned long long *__restrict__ acc, uint32_t *__restrict__ cnt, const unsigned long long *__restrict__ excl,
    const unsigned long long *__restrict__ psnap, PostOp *__restrict__ post, const uint8_t *__restrict__ zflags)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[kBodyWaves * 2 * kBufLds];
    const uint32_t lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint8_t *const wlds = lds + wv * 2 * kBufLds;
    // the frame kernel before this one advanced the epoch: its list is parity epoch-1
    const unsigned long long lc = zs->list_ctr[(zs->epoch - 1u) & 1u];
    const uint32_t n = (uint32_t) (lc >> 40), total = (uint32_t) (lc & ((1ull << 40) - 1));
    if (n == 0)
        return;
    const uint64_t tiles = (total + 63) >> 6;
    const uint64_t W = (uint64_t) blockIdx.x * kBodyWaves + wv, NW = (uint64_t) gridDim.x * kBodyWaves;
    const uint32_t tb = (uint32_t) (tiles * W / NW), te = (uint32_t) (tiles * (W + 1) / NW);
    if (tb < te) {

    const UniRounds U = uni_rounds();
    // prologue: locate tile tb from scratch, set it up and start its DMA;
    // locate tile tb+1
    TileLane cur;
    FrameLook lkn = {kIdle, 0};
    {
        const uint32_t lo = wave_find_lo(chunk_end, n, 64 * tb);
        const uint32_t g = 64 * tb + lane;
        const FrameLook lk = window_find(window_load(chunk_end, n, lo), lo, n, g);
        TileRecords R;
        load_records(R, g < total ? lk.i : 0, hot, pw);
        const uint64_t src = tile_setup<DEC>(cur, R, g < total, lk, g, cur, true);
        uint64_t a0;
        if (tile_uniform(cur.key, cur.L, src, a0))
            tile_dma_uni(wlds, a0, U);
        else
            tile_dma(wlds, src, cur.L);
        if (tb + 1 < te) {
            const uint32_t lo1 = next_tile_lo(lk, 64 * (tb + 1));
            lkn = window_find(window_load(chunk_end, n, lo1), lo1, n, 64 * (tb + 1) + lane);
        }
    }

    // The open segment of the last tile (a frame that goes on into the next
    // tile): its value at its end, its frame, the chunks of it this wave has
    // processed.  Lane 0 of the next tile starts its Horner from it.
    fe cfe = fe_zero();
    uint32_t carry_key = kIdle, carry_cnt = 0;

#pragma unroll 1
    for (uint32_t t = tb; t < te; ++t) {
#if ZMQG_STAMPS
        unsigned long long st_[8];
#endif
        ZSTAMP(0);
        uint8_t *const cb = wlds + ((t - tb) & 1) * kBufLds;
        uint8_t *const nb = wlds + (((t - tb) & 1) ^ 1) * kBufLds;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); // tile t's DMA (and everything before it)
        wave_lds_fence();
        ZSTAMP(1);
        BODY_PRIO(3);
        const bool has_next = t + 1 < te;
        // ---- issue: next tile's records, the chunk-end window after it
        const uint32_t gn = 64 * (t + 1) + lane;
        TileRecords Rn;
        load_records(Rn, has_next && gn < total ? lkn.i : 0, hot, pw);
        // (unconditional: on the last two tiles this reads a clamped, unused window)
        const uint32_t lo2 = next_tile_lo(lkn, 64 * (t + 2));
        const uint32_t ce2 = window_load(chunk_end, n, lo2 < n ? lo2 : n - 1);
        // ---- issue: this tile's finish inputs (used after its stores, so that
        // waiting for them does not wait for the stores)
        u32x4 Fq[4];
        {
            const uint32_t fi = cur.key != kIdle ? cur.key : 0;
            const GCU4 *pf = (const GCU4 *) (fin + fi);
#pragma unroll
            for (int q = 0; q < 4; ++q)
                Fq[q] = pf[q];
        }
        // ---- compute: keystream, MAC, output image (in place, one window behind)
        uint64_t v[5] = {0, 0, 0, 0, 0};
        const uint32_t L = cur.L, nwin = (L + 63) >> 6;
        const uint32_t dO = (uint32_t) (cur.dst & 15), si = cur.di & 3, so = dO & 3;
        uint8_t *const myslot = cb + lane * kSlot;
        const uint32_t *inw = (const uint32_t *) (myslot + (cur.di & ~3u));
        uint32_t *outw = (uint32_t *) (myslot + (dO & ~3u));
        // the chunk's Horner in radix 2^32 (poly32_*: 0.75x the radix-2^26
        // instructions per block), back in 26-bit limbs for the segment sums
        const PolyKey32 pk = poly32_key_from_fe(cur.r);
        const bool cin = carry_key != kIdle && __builtin_amdgcn_readfirstlane(cur.key) == carry_key;
        Poly32 h = fe_to_poly32(cin && lane == 0 ? cfe : fe_zero());
        uint32_t d[17];
        uint32_t carry = 0;
        if (nwin) {
#pragma unroll
            for (int q = 0; q < 17; ++q)
                d[q] = inw[q];
        }
        auto window = [&](uint32_t tw) {
            const int nv = L - 64 * tw >= 64 ? 64 : (int) (L - 64 * tw);
            uint32_t w[16], ks[16];
#pragma unroll
            for (int q = 0; q < 16; ++q)
                w[q] = __builtin_amdgcn_alignbyte(d[q + 1], d[q], si);
            if (nv < 64)
                mask_tail(w, nv);
#if ZMQG_ABLATE == 2 // timing experiment only: memory traffic without keystream/MAC work
#pragma unroll
            for (int q = 0; q < 16; ++q)
                ks[q] = tw * 16 + q;
#else
            salsa20_block(ks, cur.k, cur.n0, cur.n1, 1 + 2 * cur.c + tw, 0);
#endif
            if (DEC && ZMQG_ABLATE != 2) {
                if (__all(nv == 64))
                    poly32_window_full(h, pk, w);
                else
                    poly32_window(h, pk, w, 0u, (uint32_t) nv);
            }
#pragma unroll
            for (int q = 0; q < 16; ++q)
                w[q] ^= ks[q];
            if (nv < 64)
                mask_tail(w, nv);
            if (!DEC && ZMQG_ABLATE != 2) {
                if (__all(nv == 64))
                    poly32_window_full(h, pk, w);
                else
                    poly32_window(h, pk, w, 0u, (uint32_t) nv);
            }
#if ZMQG_ABLATE == 2
            h.h0 ^= w[0];
#endif
            if (tw + 1 < nwin) { // read ahead before this window's output overwrites it
#pragma unroll
                for (int q = 0; q < 17; ++q)
                    d[q] = inw[16 * (tw + 1) + q];
            }
            // image dword (dO>>2) + 16tw + q holds stream bytes [64tw + 4q - so, +4)
            if (so == 0) {
#pragma unroll
                for (int q = 0; q < 16; ++q)
                    outw[16 * tw + q] = w[q];
            } else {
                outw[16 * tw] = __builtin_amdgcn_alignbyte(w[0], carry, 4 - so);
#pragma unroll
                for (int q = 1; q < 16; ++q)
                    outw[16 * tw + q] = __builtin_amdgcn_alignbyte(w[q], w[q - 1], 4 - so);
                carry = w[15];
                if (tw + 1 == nwin)
                    outw[16 * tw + 16] = __builtin_amdgcn_alignbyte(0u, w[15], 4 - so);
            }
        };
        BODY_PRIO(0);
        if (nwin > 0)
            window(0);
        BODY_PRIO(3);
        ZSTAMP(2);
        // ---- setup: next tile's params and its DMA; locate the tile after it
        // (on the wave's last tile this sets up an all-idle tile: no DMA)
        TileLane nx;
        {
            const uint64_t nsrc = tile_setup<DEC>(nx, Rn, has_next && gn < total, lkn, gn, cur, false);
            uint64_t a0;
            const bool uni = tile_uniform(nx.key, nx.L, nsrc, a0);
            if (ZMQG_ABLATE == 6) { // (timing experiments only)
            } else if (uni) {
                tile_dma_uni(nb, a0, U);
            } else {
                tile_dma(nb, nsrc, nx.L);
            }
        }
        const FrameLook lk2 = window_find(ce2, lo2, n, 64 * (t + 2) + lane);
        ZSTAMP(3);
        BODY_PRIO(0);
        if (nwin > 1)
            window(1);
        fe hf = poly32_to_fe(h);
        fe_mul(hf, load_fe(cur.P)); // (0 on idle lanes)
#pragma unroll
        for (int q = 0; q < 5; ++q)
            v[q] = hf.l[q];
        wave_lds_fence();
        ZSTAMP(4);
        BODY_PRIO(3);
        // ---- store: coalesced interior granules, then this lane's edges
        if (ZMQG_ABLATE != 5) // (timing experiments only)
        {
            uint64_t d0;
            if (tile_uniform(cur.key, L, cur.dst, d0))
                tile_store_uni(cb, d0, U);
            else
                tile_store_interior(cb, cur.dst, L);
        }
        if (L > 0 && ZMQG_ABLATE != 3) {
            const uint32_t end = dO + L;
            GU8 *gbase = (GU8 *) (uintptr_t) (cur.dst - dO);
            const uint32_t ql = end >> 4, el = end & 15; // granule of the last byte / its valid bytes
            if (dO && !cur.prevcont) { // front edge [dO, min(16, end)) (merged by the previous chunk otherwise)
                const u32x4 gv = *(const u32x4 *) myslot;
                store_granule_range(gbase, (int) dO, end < 16 ? (int) end : 16, gv);
            }
            if (el && (ql >= 1 || dO == 0)) { // back edge [0, el) (granule 0 with dO > 0 was the front edge)
                u32x4 gv = *(const u32x4 *) (myslot + 16 * ql);
                int hi = (int) el;
                if (cur.cont) { // the next chunk's bytes [el, el + L_next) complete it
                    const u32x4 nx4 = *(const u32x4 *) (myslot + kSlot);
                    const int hn = (int) el + (int) cur.Ln;
                    const uint32_t m0 = byte_mask_below(hi, 0), m1 = byte_mask_below(hi, 1),
                                   m2 = byte_mask_below(hi, 2), m3 = byte_mask_below(hi, 3);
                    gv.x = (gv.x & m0) | (nx4.x & ~m0);
                    gv.y = (gv.y & m1) | (nx4.y & ~m1);
                    gv.z = (gv.z & m2) | (nx4.z & ~m2);
                    gv.w = (gv.w & m3) | (nx4.w & ~m3);
                    hi = hn < 16 ? hn : 16;
                }
                if (hi == 16)
                    *(GU4 *) (gbase + 16 * ql) = gv;
                else
                    store_granule_range(gbase + 16 * ql, 0, hi, gv);
            }
        }
        ZSTAMP(5);
        BODY_PRIO(0);
        // ---- finish: Poly1305 combine and tag / status
#pragma unroll
        for (int q = 0; q < 4; ++q)
            asm volatile("" ::"v"(Fq[q])); // (see tile_setup: keep every loaded word's register)
        // Per frame segment of the tile (its sum on its first lane): a segment
        // that ends its frame is combined (or is the whole frame); the open
        // one goes on as the carry, or, on the wave's last tile, is moved to
        // the frame's end and combined.
        bool first = false, carried = false;
        if (ZMQG_ABLATE != 4) {
            const uint32_t k0 = __builtin_amdgcn_readfirstlane(cur.key);
            if (__all(cur.key == k0 && k0 != kIdle)) { // one frame's segment: plain wave sum
                wave_sum_all(v);
                const uint32_t c0 = __builtin_amdgcn_readfirstlane(cur.c), nch = __builtin_amdgcn_readfirstlane(cur.nch);
                if (c0 + 64 < nch && t + 1 < te) { // the frame goes on into the next tile: it is the carry
                    cfe = fe_from_wide(v);
                    carry_cnt = 64 + (cin ? carry_cnt : 0u);
                    carry_key = k0;
                    carried = true;
                } else {
                    first = lane == 0;
                }
            } else {
                first = wave_segment_sum(cur.key, v);
            }
        }
        uint32_t mine = 0, ce = 0;
        bool ends = false;
        {
            const uint32_t kp = __shfl_up(cur.key, 1);
            const uint64_t bnd = __ballot(cur.key == kIdle || lane == 0 || kp != cur.key);
            const uint64_t above = lane == 63 ? 0ull : (bnd >> (lane + 1)) << (lane + 1);
            const uint32_t e = above ? (uint32_t) __builtin_ctzll(above) - 1u : 63u;
            if (first) {
                mine = e - lane + 1 + (lane == 0 && cin ? carry_cnt : 0u);
                ce = cur.c + (e - lane);
                ends = ce + 1 == cur.nch;
            }
        }
        const bool open = first && !ends;
        const uint64_t ob = __ballot(open);
        if (!carried)
            carry_key = kIdle;
        if (ob) {
            const int fo = (int) __builtin_ctzll(ob);
            const fe S = fe_from_wide(v);
#pragma unroll
            for (int q = 0; q < 5; ++q)
                cfe.l[q] = (uint32_t) __shfl((int) S.l[q], fo);
            carry_key = (uint32_t) __shfl((int) cur.key, fo);
            carry_cnt = (uint32_t) __shfl((int) mine, fo);
        }
        bool done = false;
        if (first && ends) {
            done = frame_combine(cur.nch, mine, acc + (size_t) cur.key * 5, cnt + cur.key, v);
        } else if (open && t + 1 == te) {
            fe S = fe_from_wide(v);
            fe_mul(S, frame_after_power(pw, powtab, cur.key, cur.nch, ce));
#pragma unroll
            for (int q = 0; q < 5; ++q)
                v[q] = S.l[q];
            done = frame_combine(cur.nch, mine, acc + (size_t) cur.key * 5, cnt + cur.key, v);
        }
        {
            const uint32_t p = cur.key; // list position
            if (done) {
                // FrameFin words: hh 0-4, s 5-8, tag 9-12, wire_len 13, frame 14
                const fe hh = rec_fe<0>(Fq);
                const uint32_t fs[4] = {rec_word<5>(Fq), rec_word<6>(Fq), rec_word<7>(Fq), rec_word<8>(Fq)};
#pragma unroll
                for (int q = 0; q < 5; ++q)
                    v[q] += hh.l[q];
                if (!DEC) {
                    uint32_t tag[16];
                    poly_finish(fe_from_wide(v), fs, tag);
                    store_window((uint8_t *) (uintptr_t) cur.out_base + 16, 16, tag);
                } else {
                    const uint32_t wtag[4] = {rec_word<9>(Fq), rec_word<10>(Fq), rec_word<11>(Fq), rec_word<12>(Fq)};
                    const uint32_t wire_len = rec_word<13>(Fq), i = rec_word<14>(Fq);
                    // replay rule first (src/curve_mechanism_base.cpp:99-104), then the MAC
                    const unsigned long long nc = ((uint64_t) bswap32(cur.n0) << 32) | bswap32(cur.n1);
                    const unsigned long long ex = excl[i], ps = psnap[i];
                    uint32_t tag[4];
                    poly_finish(fe_from_wide(v), fs, tag);
                    const uint32_t diff =
                        (tag[0] ^ wtag[0]) | (tag[1] ^ wtag[1]) | (tag[2] ^ wtag[2]) | (tag[3] ^ wtag[3]);
                    const int32_t status = !(nc > ex && nc > ps) ? ZMQG_ERR_INVALID_SEQUENCE
                                           : diff              ? ZMQG_ERR_CRYPTOGRAPHIC // :277-281
                                                               : 0;
                    status_out[i] = status;
                    flags_out[i] = status == 0 ? (uint8_t) ((cur.flags & 3u) | zmtp_msg_bits(zflags, i)) : 0;
                    // k_post, after every tile of this call: a failed frame's
                    // region is zero-filled (its tiles' plaintext may still sit
                    // dirty in other XCDs' L2s, so not here), an in-place frame
                    // moved to the frame's start
                    const bool mv = (cur.flags & kHotMove) != 0;
                    if (status != 0)
                        post_append(zs, post, cur.out_base - (mv ? 33u : 0u), mv ? wire_len : wire_len - 33u,
                                    kPostZero, p);
                    else if (mv)
                        post_append(zs, post, cur.out_base - 33u, wire_len - 33u, kPostMove, p);
                }
            }
        }
#if ZMQG_STAMPS
        ZSTAMP(6);
        if (lane == 0) {
            const unsigned int slot = atomicAdd(&zmqg_stamp_ctr, 1u);
            if (slot < (1u << 17) / 8)
                for (int q = 0; q < 7; ++q)
                    zmqg_stamp_buf[slot * 8 + q] = st_[q] - st_[0];
        }
#endif
        cur = nx;
        lkn = lk2;
    }
    } // tb < te
}

} // namespace

// =====================================================================
// host side
// =====================================================================
namespace {

template <typename T>
int grow(zmqg_ctx *ctx, T *&p, size_t count, hipStream_t st)
{
    if (p)
        ZCHECK(ctx, hipFreeAsync(p, st));
    p = nullptr;
    ZCHECK(ctx, hipMallocAsync((void **) &p, count * sizeof(T) + 64, st));
    return 0;
}

__global__ void k_zstate_init(ZState *zs)
{
    if (threadIdx.x == 0) {
        ZState z{};
        z.epoch = 1;
        *zs = z;
    }
}

// Workspace for n frames, grown in stream order on the batch's stream: the
// old buffers are freed and the new ones allocated and initialised on `st`,
// after the work already queued there (no device-wide synchronisation).
int ensure_workspace(zmqg_ctx *ctx, uint64_t n, hipStream_t st)
{
    Workspace &w = ctx->ws;
    if (n > w.cap) {
        uint64_t cap = w.cap ? w.cap : 1024;
        while (cap < n)
            cap *= 2;
        int rc;
        if ((rc = grow(ctx, w.hot, cap, st)) || (rc = grow(ctx, w.pw, cap, st)) || (rc = grow(ctx, w.fin, cap, st)) ||
            (rc = grow(ctx, w.powtab, cap * kMaxPow * 5, st)) ||
            (rc = grow(ctx, w.acc, cap * 5, st)) || (rc = grow(ctx, w.cnt, cap, st)) || (rc = grow(ctx, w.nch, cap, st)) ||
            (rc = grow(ctx, w.chunk_end, cap, st)) || (rc = grow(ctx, w.v, cap, st)) || (rc = grow(ctx, w.excl, cap, st)) ||
            (rc = grow(ctx, w.v_s, cap, st)) || (rc = grow(ctx, w.excl_s, cap, st)) || (rc = grow(ctx, w.iota, cap, st)) ||
            (rc = grow(ctx, w.perm, cap, st)) || (rc = grow(ctx, w.keys_s, cap, st)) || (rc = grow(ctx, w.last, cap, st)) ||
            (rc = grow(ctx, w.list_frame, cap, st)) || (rc = grow(ctx, w.post, cap, st)) ||
            (rc = grow(ctx, w.psnap, cap, st)) || (rc = grow(ctx, w.blockmax, cap, st)) ||
            (rc = grow(ctx, w.lb_flag, cap, st)) || (rc = grow(ctx, w.lb_agg, cap, st)) || (rc = grow(ctx, w.lb_inc, cap, st)) ||
            (rc = grow(ctx, w.nonce, cap, st)))
            return rc;
        ZCHECK(ctx, hipMemsetAsync(w.lb_flag, 0, cap * sizeof(unsigned long long), st));
        if (!w.zs) {
            if ((rc = grow(ctx, w.zs, 1, st)))
                return rc;
            hipLaunchKernelGGL(k_zstate_init, dim3(1), dim3(64), 0, st, w.zs);
            ZCHECK(ctx, hipGetLastError());
        }
        w.cap = cap;
    }
    // hipCUB temporaries for n frames
    size_t need = 0, b = 0;
    const int nn = (int) n;
    if (ctx->sort_bits > 0 && ctx->max_sessions > kReplayMaxSessions) { // the sort fallback of replay_multi
        b = 0;
        ZCHECK(ctx, hipcub::DeviceRadixSort::SortPairs(nullptr, b, (const uint32_t *) nullptr, w.keys_s,
                                                        (const uint32_t *) nullptr, w.perm, nn, 0, ctx->sort_bits));
        need = b > need ? b : need;
        b = 0;
        ZCHECK(ctx, hipcub::DeviceScan::ExclusiveScanByKey(nullptr, b, w.keys_s, w.v_s, w.excl_s, hipcub::Max(),
                                                            0ull, nn));
        need = b > need ? b : need;
    }
    if (need > w.temp_bytes) {
        size_t cap = w.temp_bytes ? w.temp_bytes : 4096;
        while (cap < need)
            cap *= 2;
        if (w.temp)
            ZCHECK(ctx, hipFreeAsync(w.temp, st));
        w.temp = nullptr;
        ZCHECK(ctx, hipMallocAsync(&w.temp, cap, st));
        w.temp_bytes = cap;
    }
    return 0;
}

uint32_t body_grid(const zmqg_ctx *ctx)
{
    // persistent: kBodyWgPerCu workgroups of 4 waves per compute unit
    return kBodyWgPerCu * (ctx->cus > 0 ? (uint32_t) ctx->cus : 256u);
}

// ZMQG_OPT_REPLAY_HOST: a zeroed peer-nonce table for the frame kernels
int ensure_zero_peer(zmqg_ctx *ctx, hipStream_t st)
{
    if (ctx->zero_peer)
        return 0;
    ZCHECK(ctx, hipMallocAsync((void **) &ctx->zero_peer, sizeof(unsigned long long) * ctx->max_sessions, st));
    ZCHECK(ctx, hipMemsetAsync(ctx->zero_peer, 0, sizeof(unsigned long long) * ctx->max_sessions, st));
    return 0;
}

int check_n(uint64_t n)
{
    return n > 0x7fffffffull ? -EINVAL : 0;
}

hipEvent_t pool_event(zmqg_ctx *ctx)
{
    if (!ctx->event_pool.empty()) {
        hipEvent_t e = ctx->event_pool.back();
        ctx->event_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess)
        return nullptr;
    return e;
}

// RAII-free pair recorder: begin() before the launch, end() after.
struct ProfSpan {
    zmqg_ctx *ctx;
    int kind;
    hipStream_t st;
    hipEvent_t a = nullptr;
    ProfSpan(zmqg_ctx *c, int k, hipStream_t s) : ctx(c), kind(k), st(s)
    {
        if (ctx->profiling && (a = pool_event(ctx)))
            (void) hipEventRecord(a, st);
    }
    void end()
    {
        if (!a)
            return;
        hipEvent_t b = pool_event(ctx);
        if (b) {
            (void) hipEventRecord(b, st);
            ctx->prof[kind].push_back({a, b});
        } else {
            ctx->event_pool.push_back(a);
        }
        a = nullptr;
    }
};

// Frame-kernel variant, from the batch size in units of the device's wave
// slots (slots = CUs x 4 SIMDs x 64 lanes: one wave per SIMD; 65,536 on
// MI355X).  Every variant is VALU-bound at one wave per SIMD, so the
// choice is about spreading the keystream work evenly over the SIMDs:
//   n <  slots/2      G = 4 lanes per frame (k_frames)
//   n <  2 slots/3    G = 2
//   n <= slots        k_frames_seq (0), one lane per frame
//   n <= 3 slots/2    k_frames_split (16 + GT): the first `slots` frames one
//                     lane each, the remainder GT lanes each in the same
//                     launch, GT the largest of 8, 4, 2 that keeps the
//                     remainder within one wave per SIMD
//   beyond            k_frames_lds (8), LDS-staged coalesced traffic
// The thresholds are the measured crossovers of the 1 KiB sweep in
// DESIGN.md section 3 (32,768 ... 131,072 frames, every variant forced).
// ZMQG_FRAMES_G (0, 1, 2, 4, 8, 18, 20, 24) forces one of these variants
// whatever the batch size (a split needs more than `slots` frames: below,
// k_frames_seq runs), so the parity tests cover every variant the rule can
// pick.
static uint64_t device_slots(const zmqg_ctx *ctx)
{
    return 256ull * (uint64_t) (ctx->cus > 0 ? ctx->cus : 256);
}

static int split_variant(const zmqg_ctx *ctx, uint32_t n)
{
    const uint64_t slots = device_slots(ctx), r = n - slots;
    return r * 8 <= slots ? 24 : r * 4 <= slots ? 20 : 18;
}

int lanes_per_frame(const zmqg_ctx *ctx, uint32_t n)
{
    const uint64_t slots = device_slots(ctx);
    if (ctx->force_g >= 0)
        return ctx->force_g >= 16 && n <= slots ? 0 : ctx->force_g;
    const uint64_t n2 = 2ull * n, n3 = 3ull * n;
    return n2 < slots ? 4 : n3 < 2 * slots ? 2 : n <= slots ? 0 : n2 <= 3 * slots ? split_variant(ctx, n) : 8;
}

// The grid of a frame-kernel launch (workgroups of kFramesBS threads).
static uint64_t frames_grid(const zmqg_ctx *ctx, int G, uint32_t n)
{
    if (G >= 16) {
        const uint64_t sn = device_slots(ctx);
        return sn / kFramesBS + ((n - sn) * (uint64_t) (G - 16) + kFramesBS - 1) / kFramesBS;
    }
    return ((uint64_t) n * (G == 1 || G == 2 || G == 4 ? G : 1) + kFramesBS - 1) / kFramesBS;
}

// Workgroups of the decode frame kernel the device holds at once (occupancy
// query x CUs; the kernel is VGPR-limited, where the query is exact --
// MI355X_MICROARCH.md, Residency), cached per variant.
int frames_capacity(zmqg_ctx *ctx, int G, bool so = false)
{
    int &c = ctx->frames_cap[G == 0 && so ? 8 : G == 24 ? 7 : G == 20 ? 6 : G == 18 ? 5 : G == 8 ? 4 : G == 0 ? 3 : G == 1 ? 0
                             : G == 2 ? 1 : 2];
    if (c == 0) {
        int nb = 0;
        hipError_t e =
            G == 24  ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_frames_split<true, 8, DecodeHead>, kFramesBS, 0)
            : G == 20 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_frames_split<true, 4, DecodeHead>, kFramesBS, 0)
            : G == 18 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_frames_split<true, 2, DecodeHead>, kFramesBS, 0)
            : G == 8  ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_frames_lds<true, DecodeHead>, kFramesBS, 0)
            : G == 0 && so ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_frames_seq<true, DecodeHead, true>, kFramesBS, 0)
            : G == 0  ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_frames_seq<true, DecodeHead>, kFramesBS, 0)
            : G == 1  ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_frames<true, 1, DecodeHead>, kFramesBS, 0)
            : G == 2  ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_frames<true, 2, DecodeHead>, kFramesBS, 0)
                      : hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_frames<true, 4, DecodeHead>, kFramesBS, 0);
        c = (e == hipSuccess && nb > 0) ? nb * ctx->cus : -1;
    }
    return c;
}

template <bool DEC, class BigOp>
void launch_frames(const zmqg_ctx *ctx, int G, uint32_t n, hipStream_t st, const uint32_t *sid, const uint64_t *nonce,
                   const uint8_t *flags, const uint64_t *in_off, const uint32_t *len, const uint8_t *in,
                   const uint64_t *out_off, uint8_t *out, const DevSession *sessions, uint32_t max_sessions,
                   uint8_t *flags_out, int32_t *status_out, ReplayOut rp, BigOp big, ZState *zs, FrameCtl ctl)
{
    const dim3 grid((uint32_t) frames_grid(ctx, G, n));
    if (G >= 16) {
        // (the split points: ctl carries them into both bodies)
        const uint32_t sn = (uint32_t) device_slots(ctx);
        ctl.split_wg = sn / kFramesBS;
        ctl.split_n = sn;
#define ZMQG_LAUNCH_SPLIT(GT)                                                                                        \
    hipLaunchKernelGGL((k_frames_split<DEC, GT, BigOp>), grid, dim3(kFramesBS), 0, st, n, sid, nonce, flags, in_off, \
                       len, in, out_off, out, sessions, max_sessions, kMaxFrameStream, flags_out, status_out, rp, big, \
                       zs, ctl)
        if (G == 24)
            ZMQG_LAUNCH_SPLIT(8);
        else if (G == 20)
            ZMQG_LAUNCH_SPLIT(4);
        else
            ZMQG_LAUNCH_SPLIT(2);
#undef ZMQG_LAUNCH_SPLIT
        return;
    }
    if (G == 8) {
        hipLaunchKernelGGL((k_frames_lds<DEC, BigOp>), grid, dim3(kFramesBS), 0, st, n, sid, nonce, flags, in_off, len, in,
                           out_off, out, sessions, max_sessions, kMaxFrameStream, flags_out, status_out, rp, big, zs,
                           ctl);
        return;
    }
    if (G == 0) {
        if (ctl.stream_out) { // ZMQG_OPT_STREAM_OUT: whole-window output stores
            hipLaunchKernelGGL((k_frames_seq<DEC, BigOp, true>), grid, dim3(kFramesBS), 0, st, n, sid, nonce, flags,
                               in_off, len, in, out_off, out, sessions, max_sessions, kMaxFrameStream, flags_out,
                               status_out, rp, big, zs, ctl);
            return;
        }
        hipLaunchKernelGGL((k_frames_seq<DEC, BigOp>), grid, dim3(kFramesBS), 0, st, n, sid, nonce, flags, in_off, len, in,
                           out_off, out, sessions, max_sessions, kMaxFrameStream, flags_out, status_out, rp, big, zs,
                           ctl);
        return;
    }
#define ZMQG_LAUNCH_FRAMES(GG)                                                                                        \
    hipLaunchKernelGGL((k_frames<DEC, GG, BigOp>), grid, dim3(kFramesBS), 0, st, n, sid, nonce, flags, in_off, len, in,      \
                       out_off, out, sessions, max_sessions, kMaxFrameStream, flags_out, status_out, rp, big, zs, \
                       ctl)
    if (G == 1)
        ZMQG_LAUNCH_FRAMES(1);
    else if (G == 2)
        ZMQG_LAUNCH_FRAMES(2);
    else
        ZMQG_LAUNCH_FRAMES(4);
#undef ZMQG_LAUNCH_FRAMES
}

// Frames per tile of the session tables (k_replay_*, k_nonce_*): at least
// 256 and at least the session count (a tile's table row costs S entries,
// so that stays below its frames' work), doubled until there are at most
// kReplayMaxTiles tiles.  Small batches get many tiles, so the per-tile walk
// (k_*_frames, one wave each) spreads over the chip.
uint32_t replay_tile_frames(uint32_t nn, uint32_t S)
{
    uint32_t T = 256;
    while (T < S)
        T *= 2;
    while ((nn + T - 1) / T > kReplayMaxTiles)
        T *= 2;
    return T;
}

// ZMQG_OPT_NONCE_AUTO over several sessions: each frame's nonce into w.nonce
// (k_nonce_*), advancing the sessions' send counters, on `st` before the
// frame kernel.
int nonce_multi(zmqg_ctx *ctx, uint32_t nn, const uint32_t *sid, hipStream_t st)
{
    Workspace &w = ctx->ws;
    const uint32_t S = ctx->max_sessions;
    const uint32_t T = replay_tile_frames(nn, S);
    const uint32_t tiles = (nn + T - 1) / T, rbs = (tiles + kReplayRB - 1) / kReplayRB;
    const size_t need = ((size_t) tiles + rbs + 1) * S; // tables, block sums, send snapshot
    if (need > w.rt_cap) {
        if (w.rt)
            ZCHECK(ctx, hipFreeAsync(w.rt, st));
        w.rt = nullptr;
        ZCHECK(ctx, hipMallocAsync((void **) &w.rt, need * sizeof(unsigned long long), st));
        w.rt_cap = need;
    }
    unsigned long long *tab = w.rt, *blk = w.rt + (size_t) tiles * S, *snap = blk + (size_t) rbs * S;
    hipLaunchKernelGGL(k_nonce_tiles, dim3(tiles), dim3(256), S * sizeof(uint32_t), st, nn, T, S, sid, tab);
    ZCHECK(ctx, hipGetLastError());
    const dim3 cg((S + 255) / 256, rbs);
    hipLaunchKernelGGL(k_nonce_colblk, cg, dim3(256), 0, st, tiles, S, (const unsigned long long *) tab, blk,
                       (const unsigned long long *) ctx->send, snap);
    ZCHECK(ctx, hipGetLastError());
    hipLaunchKernelGGL(k_nonce_colscan, cg, dim3(256), 0, st, tiles, S, tab, (const unsigned long long *) blk,
                       (const unsigned long long *) snap, ctx->send);
    ZCHECK(ctx, hipGetLastError());
    hipLaunchKernelGGL(k_nonce_frames, dim3(tiles), dim3(64), S * sizeof(unsigned long long), st, nn, T, S, sid,
                       (const unsigned long long *) tab, w.nonce);
    ZCHECK(ctx, hipGetLastError());
    return 0;
}

// Multi-session replay prefix (k_fixup's excl) after the frame kernel: the
// replay tables for up to kReplayMaxSessions sessions, else sort by session +
// segmented scan (hipCUB).  Writes each session's new peer nonce (and its
// batch max into smax when given).
int replay_multi(zmqg_ctx *ctx, uint32_t nn, const uint32_t *sid, hipStream_t st, unsigned long long *smax)
{
    Workspace &w = ctx->ws;
    const uint32_t S = ctx->max_sessions;
    if (S <= kReplayMaxSessions) {
        const uint32_t T = replay_tile_frames(nn, S);
        const uint32_t tiles = (nn + T - 1) / T, rbs = (tiles + kReplayRB - 1) / kReplayRB;
        const size_t need = ((size_t) tiles + rbs + 1) * S; // tables, block sums, send snapshot
        if (need > w.rt_cap) {
            if (w.rt)
                ZCHECK(ctx, hipFreeAsync(w.rt, st));
            w.rt = nullptr;
            ZCHECK(ctx, hipMallocAsync((void **) &w.rt, need * sizeof(unsigned long long), st));
            w.rt_cap = need;
        }
        unsigned long long *tab = w.rt, *blk = w.rt + (size_t) tiles * S;
        hipLaunchKernelGGL(k_replay_tiles, dim3(tiles), dim3(256), S * sizeof(unsigned long long), st, nn, T, S, sid,
                           (const unsigned long long *) w.v, tab);
        ZCHECK(ctx, hipGetLastError());
        const dim3 cg((S + 255) / 256, rbs);
        hipLaunchKernelGGL(k_replay_colblk, cg, dim3(256), 0, st, tiles, S, (const unsigned long long *) tab, blk);
        ZCHECK(ctx, hipGetLastError());
        hipLaunchKernelGGL(k_replay_colscan, cg, dim3(256), 0, st, tiles, S, tab, (const unsigned long long *) blk,
                           ctx->peer, smax);
        ZCHECK(ctx, hipGetLastError());
        hipLaunchKernelGGL(k_replay_frames, dim3(tiles), dim3(64), S * (sizeof(unsigned long long) + 4), st, nn, T, S,
                           sid, (const unsigned long long *) w.v, (const unsigned long long *) tab, w.excl);
        ZCHECK(ctx, hipGetLastError());
        w.use_last = false;
        return 0;
    }
    const dim3 hgrid((nn + kHeadThreads - 1) / kHeadThreads);
    size_t tb = w.temp_bytes;
    ZCHECK(ctx, hipcub::DeviceRadixSort::SortPairs(w.temp, tb, sid, w.keys_s, w.iota, w.perm, (int) nn, 0,
                                                    ctx->sort_bits, st));
    hipLaunchKernelGGL(k_gather_u64, hgrid, dim3(kHeadThreads), 0, st, nn, w.perm, w.v, w.v_s);
    ZCHECK(ctx, hipGetLastError());
    tb = w.temp_bytes;
    ZCHECK(ctx, hipcub::DeviceScan::ExclusiveScanByKey(w.temp, tb, w.keys_s, w.v_s, w.excl_s, hipcub::Max(),
                                                        0ull, (int) nn, hipcub::Equality(), st));
    hipLaunchKernelGGL(k_scatter_replay, hgrid, dim3(kHeadThreads), 0, st, nn, w.perm, w.keys_s, w.excl_s, w.excl,
                       w.last);
    ZCHECK(ctx, hipGetLastError());
    w.use_last = true;
    return 0;
}

} // namespace

// k_msg with the message inline in its arguments when it fits one of the
// tiers (the argument block is copied whole, so small messages take a small
// tier), else read from the mapped buffer.
template <bool DEC>
static void launch_msg(hipStream_t st, const MsgArgs &a, const uint8_t *msg, uint32_t n)
{
    auto go = [&](auto inl) {
        memset(inl.w, 0, sizeof inl.w);
        if (n)
            memcpy(inl.w, msg, n);
        hipLaunchKernelGGL((k_msg<DEC, sizeof inl.w>), dim3(1), dim3(kMsgThreads), 0, st, a, inl);
    };
    if (n <= 256u)
        go(MsgInline<256>{});
    else if (n <= 1024)
        go(MsgInline<1024>{});
    else if (n <= kMsgInlineMax)
        go(MsgInline<kMsgInlineMax>{});
    else
        hipLaunchKernelGGL((k_msg<DEC, 0>), dim3(1), dim3(kMsgThreads), 0, st, a, MsgInline<0>{});
}

extern "C" {

int zmqg_abi_version(void)
{
    return ZMQG_CURVE_ABI_VERSION;
}

int zmqg_ctx_create(int device, uint32_t max_sessions, zmqg_ctx **ctx_out)
{
    if (!ctx_out || max_sessions == 0)
        return -EINVAL;
    *ctx_out = nullptr;
    zmqg_ctx *ctx = new (std::nothrow) zmqg_ctx;
    if (!ctx)
        return -ENOMEM;
    ctx->device = device;
    ctx->max_sessions = max_sessions;
    int bits = 0;
    while (bits < 32 && (1ull << bits) < max_sessions)
        ++bits;
    ctx->sort_bits = bits;
    ctx->h_downgrade.assign(max_sessions, 0);
    if (const char *fg = getenv("ZMQG_FRAMES_G")) {
        const int g = atoi(fg);
        if (g == 0 || g == 1 || g == 2 || g == 4 || g == 8 || g == 18 || g == 20 || g == 24)
            ctx->force_g = g;
    }
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess)
        e = hipStreamCreateWithFlags(&ctx->own_stream, hipStreamNonBlocking);
    // The tables are cleared on the ctx's own stream and that stream alone is
    // waited for (a null-stream memset is not ordered before the non-blocking
    // streams the batches run on: a session installed right after could be
    // cleared by the late memset).  No device-wide synchronisation.
    if (e == hipSuccess)
        e = hipMalloc((void **) &ctx->sessions, sizeof(DevSession) * max_sessions);
    if (e == hipSuccess)
        e = hipMemsetAsync(ctx->sessions, 0, sizeof(DevSession) * max_sessions, ctx->own_stream);
    if (e == hipSuccess)
        e = hipMalloc((void **) &ctx->peer, sizeof(unsigned long long) * max_sessions);
    if (e == hipSuccess)
        e = hipMemsetAsync(ctx->peer, 0, sizeof(unsigned long long) * max_sessions, ctx->own_stream);
    if (e == hipSuccess)
        e = hipMalloc((void **) &ctx->send, sizeof(unsigned long long) * max_sessions);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_fill_u64, dim3((max_sessions + 255) / 256), dim3(256), 0, ctx->own_stream, ctx->send,
                           max_sessions, 1ull);
        e = hipGetLastError();
    }
    if (e == hipSuccess)
        e = hipStreamSynchronize(ctx->own_stream);
    if (e == hipSuccess)
        e = hipDeviceGetAttribute(&ctx->cus, hipDeviceAttributeMultiprocessorCount, device);
    if (e != hipSuccess) {
        fprintf(stderr, "zmqg_ctx_create: %s\n", hipGetErrorString(e));
        zmqg_ctx_destroy(ctx);
        return -EIO;
    }
    *ctx_out = ctx;
    return 0;
}

int zmqg_ctx_destroy(zmqg_ctx *ctx)
{
    if (!ctx)
        return -EINVAL;
    (void) hipSetDevice(ctx->device);
    // the ctx's work is on its last batch stream and its own stream
    if (ctx->has_last && ctx->last_stream != ctx->own_stream)
        (void) hipStreamSynchronize(ctx->last_stream);
    if (ctx->own_stream)
        (void) hipStreamSynchronize(ctx->own_stream);
    Workspace &w = ctx->ws;
    void *ptrs[] = {w.hot, w.pw, w.fin, w.powtab, w.acc, w.cnt, w.nch, w.chunk_end, w.v, w.excl, w.v_s,
                    w.excl_s, w.iota, w.perm, w.keys_s, w.last, w.list_frame, w.post, w.psnap, w.blockmax, w.zs,
                    w.lb_flag, w.lb_agg, w.lb_inc, w.temp, w.rt, w.nonce, w.stage, ctx->sessions, ctx->peer, ctx->send, ctx->zero_peer, ctx->dbuf};
    for (void *p : ptrs)
        if (p)
            (void) hipFree(p);
    {
        ZmtpWs &z = ctx->zw;
        void *zp[] = {z.F,      z.wire_off, z.cand_wg, z.count_wg, z.off_wg, z.cand, z.nb,   z.first_w,
                      z.wid,    z.run,      z.runpre,  z.sid_fill, z.fflags, z.walk, z.temp, z.count16, z.cdesc, z.cflag};
        for (void *p : zp)
            if (p)
                (void) hipFree(p);
        if (z.res)
            (void) hipHostFree(z.res);
    }
    if (ctx->pin)
        (void) hipHostFree(ctx->pin);
    if (ctx->mpin)
        (void) hipHostFree(ctx->mpin);
    if (ctx->sinst_done) {
        (void) hipEventSynchronize(ctx->sinst_done);
        (void) hipEventDestroy(ctx->sinst_done);
    }
    if (ctx->sinst)
        (void) hipHostFree(ctx->sinst);
    if (ctx->order_ev)
        (void) hipEventDestroy(ctx->order_ev);
    // notification host functions still queued hold the ctx: after ~10 s
    // without them the ctx is left allocated (leaked, not freed under them)
    const int quiet = notify_wait(ctx);
    if (ctx->own_stream)
        (void) hipStreamDestroy(ctx->own_stream);
    for (auto &v : ctx->prof)
        for (auto &p : v) {
            (void) hipEventDestroy(p.first);
            (void) hipEventDestroy(p.second);
        }
    for (hipEvent_t e : ctx->event_pool)
        (void) hipEventDestroy(e);
    for (auto &f : ctx->fences)
        (void) hipEventDestroy(f.second);
    for (hipEvent_t e : ctx->fence_pool)
        (void) hipEventDestroy(e);
    if (quiet != 0)
        return quiet;
    delete ctx;
    return 0;
}

int zmqg_ctx_set_profiling(zmqg_ctx *ctx, int enable)
{
    if (!ctx)
        return -EINVAL;
    ctx->profiling = enable != 0;
    return 0;
}

int zmqg_ctx_get_profile(zmqg_ctx *ctx, int kind, double *ms_total, uint64_t *launches)
{
    if (!ctx || kind < 0 || kind > 5 || !ms_total || !launches)
        return -EINVAL;
    ZCHECK(ctx, hipSetDevice(ctx->device));
    double tot = 0;
    for (auto &p : ctx->prof[kind]) {
        float ms = 0;
        ZCHECK(ctx, hipEventSynchronize(p.second));
        ZCHECK(ctx, hipEventElapsedTime(&ms, p.first, p.second));
        tot += ms;
        ctx->event_pool.push_back(p.first);
        ctx->event_pool.push_back(p.second);
    }
    *ms_total = tot;
    *launches = ctx->prof[kind].size();
    ctx->prof[kind].clear();
    return 0;
}

#if ZMQG_STAMPS
// diagnostic build only: copy out (and reset) the per-wave phase stamps
int zmqg_debug_stamps(unsigned long long *out, uint32_t max_records, uint32_t *count)
{
    unsigned int n = 0;
    if (hipDeviceSynchronize() != hipSuccess || hipMemcpyFromSymbol(&n, HIP_SYMBOL(zmqg_stamp_ctr), sizeof n) != hipSuccess)
        return -EIO;
    if (n > (1u << 17) / 8)
        n = (1u << 17) / 8;
    if (n > max_records)
        n = max_records;
    if (n && hipMemcpyFromSymbol(out, HIP_SYMBOL(zmqg_stamp_buf), (size_t) n * 8 * sizeof(unsigned long long)) !=
                 hipSuccess)
        return -EIO;
    unsigned int z = 0;
    if (hipMemcpyToSymbol(HIP_SYMBOL(zmqg_stamp_ctr), &z, sizeof z) != hipSuccess)
        return -EIO;
    *count = n;
    return 0;
}
#endif

const char *zmqg_last_error(zmqg_ctx *ctx)
{
    return ctx ? ctx->last_error : "null ctx";
}

int zmqg_session_set(zmqg_ctx *ctx, uint32_t sid, const uint8_t precom[32], const uint8_t enc_prefix[16],
                     const uint8_t dec_prefix[16], int downgrade_sub, uint64_t peer_nonce)
{
    if (!ctx || !precom || !enc_prefix || !dec_prefix || sid >= ctx->max_sessions)
        return -EINVAL;
    std::lock_guard<std::mutex> lk(ctx->mu);
    ZCHECK(ctx, hipSetDevice(ctx->device));
    uint32_t in[19];
    memcpy(in, precom, 32);
    memcpy(in + 8, enc_prefix, 16);
    memcpy(in + 12, dec_prefix, 16);
    in[16] = downgrade_sub ? 1u : 0u;
    in[17] = (uint32_t) peer_nonce;
    in[18] = (uint32_t) (peer_nonce >> 32);
    ctx->h_downgrade[sid] = downgrade_sub ? 1 : 0;
    // after whatever the ctx queued on its last stream (an earlier
    // asynchronous install of the same sid, frames still using its keys)
    int orc = order_after_last(ctx, ctx->own_stream);
    if (orc)
        return orc;
    uint32_t *d = nullptr;
    ZCHECK(ctx, hipMalloc((void **) &d, sizeof in));
    hipError_t e = hipMemcpyAsync(d, in, sizeof in, hipMemcpyHostToDevice, ctx->own_stream);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_session_setup, dim3(1), dim3(64), 0, ctx->own_stream, ctx->sessions, ctx->peer, ctx->send,
                           sid, d);
        e = hipGetLastError();
    }
    if (e == hipSuccess)
        e = hipStreamSynchronize(ctx->own_stream);
    (void) hipFree(d);
    ZCHECK(ctx, e);
    return 0;
}

int zmqg_session_set_batch(zmqg_ctx *ctx, uint64_t n, const uint32_t *sid, const uint8_t *precom,
                           const uint8_t enc_prefix[16], const uint8_t dec_prefix[16], const uint8_t *downgrade,
                           const uint64_t *peer_nonce, void *stream)
{
    return zmqg_session_set_batch_ex(ctx, n, sid, precom, enc_prefix, dec_prefix, downgrade, peer_nonce, nullptr,
                                     stream);
}

int zmqg_session_set_batch_ex(zmqg_ctx *ctx, uint64_t n, const uint32_t *sid, const uint8_t *precom,
                              const uint8_t enc_prefix[16], const uint8_t dec_prefix[16], const uint8_t *downgrade,
                              const uint64_t *peer_nonce, const uint64_t *send_nonce, void *stream)
{
    if (!ctx || check_n(n))
        return -EINVAL;
    if (n == 0)
        return 0;
    if (!sid || !precom || ((uintptr_t) precom & 3u) || !enc_prefix || !dec_prefix)
        return -EINVAL;
    std::lock_guard<std::mutex> lk(ctx->mu);
    {
        std::vector<uint8_t> seen(ctx->max_sessions, 0); // distinct, known sids (the install has no order)
        for (uint64_t i = 0; i < n; ++i) {
            if (sid[i] >= ctx->max_sessions || seen[sid[i]])
                return -EINVAL;
            seen[sid[i]] = 1;
        }
    }
    ZCHECK(ctx, hipSetDevice(ctx->device));
    const size_t o_peer = (4 * n + 7) & ~(size_t) 7, o_send = o_peer + 8 * n, o_down = o_send + 8 * n,
                 need = o_down + n;
    if (ctx->sinst_done)
        ZCHECK(ctx, hipEventSynchronize(ctx->sinst_done)); // the previous install has read its descriptors
    else
        ZCHECK(ctx, hipEventCreateWithFlags(&ctx->sinst_done, hipEventDisableTiming));
    if (need > ctx->sinst_bytes) {
        if (ctx->sinst)
            ZCHECK(ctx, hipHostFree(ctx->sinst));
        ctx->sinst = nullptr;
        ctx->sinst_bytes = 0;
        hipError_t e = hipHostMalloc((void **) &ctx->sinst, need, hipHostMallocMapped | hipHostMallocPortable);
        if (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation)
            return -ENOMEM;
        ZCHECK(ctx, e);
        void *dp = nullptr;
        ZCHECK(ctx, hipHostGetDevicePointer(&dp, ctx->sinst, 0));
        ctx->sinst_dev = (uint8_t *) dp;
        ctx->sinst_bytes = need;
    }
    memcpy(ctx->sinst, sid, 4 * n);
    uint64_t *pn = (uint64_t *) (ctx->sinst + o_peer);
    for (uint64_t i = 0; i < n; ++i)
        pn[i] = peer_nonce ? peer_nonce[i] : 1u;
    uint64_t *sn = (uint64_t *) (ctx->sinst + o_send);
    for (uint64_t i = 0; i < n; ++i)
        sn[i] = send_nonce ? send_nonce[i] : 1u;
    for (uint64_t i = 0; i < n; ++i) {
        const uint8_t dg = downgrade && downgrade[i] ? 1 : 0;
        ctx->sinst[o_down + i] = dg;
        ctx->h_downgrade[sid[i]] = dg;
    }
    Prefixes pfx;
    memcpy(pfx.w, enc_prefix, 16);
    memcpy(pfx.w + 4, dec_prefix, 16);
    hipStream_t st = (hipStream_t) stream;
    // the install overwrites sessions that work queued on the previous
    // stream may still be using: it runs after that work
    int orc = order_after_last(ctx, st);
    if (orc)
        return orc;
    hipLaunchKernelGGL(k_session_setup_batch, dim3((uint32_t) ((n + 255) / 256)), dim3(256), 0, st, (uint32_t) n,
                       (const uint8_t *) ctx->sinst_dev, (const uint32_t *) precom, pfx, ctx->sessions, ctx->peer,
                       ctx->send);
    ZCHECK(ctx, hipGetLastError());
    ZCHECK(ctx, hipEventRecord(ctx->sinst_done, st));
    return 0;
}

// A session's u64 counter (peer nonce, send nonce), in order after the work
// already issued on the ctx's last batch stream.
static int session_u64_set(zmqg_ctx *ctx, unsigned long long *arr, uint32_t sid, uint64_t v)
{
    if (!ctx || sid >= ctx->max_sessions)
        return -EINVAL;
    ZCHECK(ctx, hipSetDevice(ctx->device));
    hipStream_t st = ctx->has_last ? ctx->last_stream : ctx->own_stream;
    hipLaunchKernelGGL(k_set_peer, dim3(1), dim3(64), 0, st, arr, sid, (unsigned long long) v);
    ZCHECK(ctx, hipGetLastError());
    ZCHECK(ctx, hipStreamSynchronize(st));
    return 0;
}

static int session_u64_get(zmqg_ctx *ctx, const unsigned long long *arr, uint32_t sid, uint64_t *out)
{
    if (!ctx || sid >= ctx->max_sessions || !out)
        return -EINVAL;
    ZCHECK(ctx, hipSetDevice(ctx->device));
    hipStream_t st = ctx->has_last ? ctx->last_stream : ctx->own_stream;
    unsigned long long v = 0;
    ZCHECK(ctx, hipMemcpyAsync(&v, arr + sid, sizeof v, hipMemcpyDeviceToHost, st));
    ZCHECK(ctx, hipStreamSynchronize(st));
    *out = v;
    return 0;
}

int zmqg_session_set_peer_nonce(zmqg_ctx *ctx, uint32_t sid, uint64_t peer_nonce)
{
    return session_u64_set(ctx, ctx ? ctx->peer : nullptr, sid, peer_nonce);
}

int zmqg_session_get_peer_nonce(zmqg_ctx *ctx, uint32_t sid, uint64_t *peer_nonce_out)
{
    return session_u64_get(ctx, ctx ? ctx->peer : nullptr, sid, peer_nonce_out);
}

int zmqg_session_set_nonce(zmqg_ctx *ctx, uint32_t sid, uint64_t nonce)
{
    return session_u64_set(ctx, ctx ? ctx->send : nullptr, sid, nonce);
}

int zmqg_session_get_nonce(zmqg_ctx *ctx, uint32_t sid, uint64_t *nonce_out)
{
    return session_u64_get(ctx, ctx ? ctx->send : nullptr, sid, nonce_out);
}

uint64_t zmqg_wire_size(uint8_t msg_flags, int downgrade_sub, uint64_t payload_len)
{
    const uint32_t ct = msg_flags & 0x1c;
    uint64_t hl = 1;
    if (ct == ZMQG_MSG_SUBSCRIBE || ct == ZMQG_MSG_CANCEL)
        hl = downgrade_sub ? 2 : (ct == ZMQG_MSG_CANCEL ? 8 : 11);
    return 32 + hl + payload_len;
}

// opts of a caller built against the struct before out_bytes: the fields
// it has are read, out_bytes is taken as 0
static int check_opts(const zmqg_batch_opts *o)
{
    return o && o->size < offsetof(zmqg_batch_opts, out_bytes) ? -EINVAL : 0;
}

static uint64_t opt_out_bytes(const zmqg_batch_opts *o)
{
    return o && o->size >= offsetof(zmqg_batch_opts, out_bytes) + sizeof(uint64_t) ? o->out_bytes : 0;
}

static const int32_t *opt_verdict_in(const zmqg_batch_opts *o)
{
    return o && o->size >= offsetof(zmqg_batch_opts, verdict_in) + sizeof(void *) ? o->verdict_in : nullptr;
}

// ZMQG_OPT_VERIFY_FIRST: frame i's payload, decoded into the staging area at
// the same offset (and the same alignment mod 16) as in `out`, goes to `out`
// once its status is known: the payload if the frame verified, zeros if it
// failed; a frame the decode left as it was (above the bound, or shorter
// than the 33-byte MESSAGE minimum) is left as it was here too.  One
// workgroup per frame; 16-byte stores in the aligned middle.
// ZMQG_OPT_REPLAY_HOST: `verdict` (the host's header / replay verdict per
// frame) comes first; the kernels' status stands only where it is 0, and a
// frame it fails gets that status and flags 0.
__global__ __launch_bounds__(256) void k_verify_copy(uint32_t n, const uint8_t *__restrict__ stage,
                                                     uint8_t *__restrict__ out, const uint64_t *__restrict__ out_off,
                                                     const uint32_t *__restrict__ wire_len,
                                                     int32_t *__restrict__ status,
                                                     const int32_t *__restrict__ verdict,
                                                     uint8_t *__restrict__ flags_out)
{
    for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
        const uint32_t wl = wire_len[i];
        int32_t stt = status[i];
        if (verdict) {
            const int32_t vd = verdict[i];
            if (vd != 0 && stt != ZMQG_ERR_BOUND && stt != ZMQG_ERR_SESSION) {
                __syncthreads(); // (every thread has read status[i])
                if (threadIdx.x == 0) {
                    status[i] = vd;
                    flags_out[i] = 0;
                }
                stt = vd;
            }
        }
        if (wl <= 33u || stt == ZMQG_ERR_BOUND)
            continue;
        const uint64_t L = wl - 33u, o = out_off[i];
        const bool ok = stt == 0;
        const uint8_t *src = stage + o;
        uint8_t *dst = out + o;
        const uint64_t head = (16u - ((uintptr_t) dst & 15u)) & 15u;
        const uint64_t h = head < L ? head : L;
        const uint64_t body = (L - h) & ~15ull;
        for (uint64_t k = threadIdx.x; k < h; k += blockDim.x)
            dst[k] = ok ? src[k] : 0;
        const u32x4 z = {0, 0, 0, 0};
        for (uint64_t k = h + 16ull * threadIdx.x; k < h + body; k += 16ull * blockDim.x)
            *(GU4 *) (uintptr_t) (dst + k) = ok ? *(const GCU4 *) (uintptr_t) (src + k) : z;
        for (uint64_t k = h + body + threadIdx.x; k < L; k += blockDim.x)
            dst[k] = ok ? src[k] : 0;
    }
}

int zmqg_encode_batch_ex(zmqg_ctx *ctx, uint64_t n, const uint32_t *sid, const uint64_t *nonce, const uint8_t *flags,
                         const uint64_t *in_off, const uint32_t *len, const uint8_t *in, const uint64_t *out_off,
                         uint8_t *out, const zmqg_batch_opts *opts, void *stream)
{
    if (!ctx || check_n(n) || check_opts(opts))
        return -EINVAL;
    const bool auto_nonce = opts && (opts->flags & ZMQG_OPT_NONCE_AUTO);
    if (auto_nonce && ctx->max_sessions > kReplayMaxSessions)
        return -EINVAL;
    if (n == 0)
        return 0;
    if (!sid || (!nonce && !auto_nonce) || !flags || !in_off || !len || !in || !out_off || !out)
        return -EINVAL;
    hipStream_t st = (hipStream_t) stream;
    ZCHECK(ctx, hipSetDevice(ctx->device));
    // the workspace and the call state are shared with the ctx's other
    // streams: this call runs after the work queued on the last one
    int rc = order_after_last(ctx, st);
    if (rc)
        return rc;
    rc = ensure_workspace(ctx, n, st);
    if (rc)
        return rc;
    Workspace &w = ctx->ws;
    const uint32_t nn = (uint32_t) n;
    const int G = lanes_per_frame(ctx, nn);
    FrameCtl ctl{};
    if (opts) {
        ctl.enc_status = opts->status_out;
        ctl.max_len = opts->max_len;
        ctl.stream_out = (opts->flags & ZMQG_OPT_STREAM_OUT) ? 1u : 0u;
        // every frame within the bound fits the frame kernel: no body launch
        ctl.no_body = opts->max_len && opts->max_len <= kMaxFrameStream - 43u; // (no wrap near UINT64_MAX)
    }
    const BigRecords R{w.hot, w.pw, w.fin, w.powtab, w.acc, w.cnt, w.chunk_end, w.list_frame};
    ProfSpan call(ctx, ZMQG_PROF_ENCODE_CALL, st);
    if (auto_nonce) {
        if (ctx->max_sessions == 1) {
            ctl.nonce_ctr = ctx->send; // in the frame kernel
        } else {
            if ((rc = nonce_multi(ctx, nn, sid, st)))
                return rc;
            nonce = w.nonce;
        }
    }
    ProfSpan main(ctx, ZMQG_PROF_ENCODE_MAIN, st);
    launch_frames<false>(ctx, G, nn, st, sid, nonce, flags, in_off, len, in, out_off, out, ctx->sessions,
                         ctx->max_sessions, nullptr, nullptr, ReplayOut{},
                         EncodeHead{sid, nonce, flags, in_off, len, in, out_off, out, ctx->sessions,
                                    ctx->max_sessions, R, ctl.nonce_ctr},
                         w.zs, ctl);
    ZCHECK(ctx, hipGetLastError());
    main.end();
    if (!ctl.no_body) {
        ProfSpan body(ctx, ZMQG_PROF_ENCODE_BODY, st);
        hipLaunchKernelGGL(k_body<false>, dim3(body_grid(ctx)), dim3(kBodyThreads), 0, st, w.zs, w.chunk_end, w.hot,
                           w.pw, w.fin, w.powtab, (uint8_t *) nullptr, (int32_t *) nullptr, w.acc, w.cnt,
                           (const unsigned long long *) nullptr, (const unsigned long long *) nullptr,
                           (PostOp *) nullptr, (const uint8_t *) nullptr);
        ZCHECK(ctx, hipGetLastError());
        body.end();
    }
    call.end();
    return 0;
}

int zmqg_encode_batch(zmqg_ctx *ctx, uint64_t n, const uint32_t *sid, const uint64_t *nonce, const uint8_t *flags,
                      const uint64_t *in_off, const uint32_t *len, const uint8_t *in, const uint64_t *out_off,
                      uint8_t *out, void *stream)
{
    return zmqg_encode_batch_ex(ctx, n, sid, nonce, flags, in_off, len, in, out_off, out, nullptr, stream);
}

// zmqg_decode_batch_ex; zflags (zmqg_decode_zmtp): each frame's ZMTP flags
// byte, whose MORE / COMMAND bits the decode ORs into flags_out
static int decode_batch_impl(zmqg_ctx *ctx, uint64_t n, const uint32_t *sid, const uint64_t *in_off,
                             const uint32_t *wire_len, const uint8_t *in, const uint64_t *out_off, uint8_t *out,
                             uint8_t *flags_out, int32_t *status_out, const zmqg_batch_opts *opts,
                             const uint8_t *zflags, const ZmtpWalk *zwalk, zmqg_zmtp_result *zres, void *stream)
{
    if (!ctx || check_n(n) || check_opts(opts))
        return -EINVAL;
    if (n == 0)
        return 0;
    if (!sid || !in_off || !wire_len || !in || !out_off || !out || !flags_out || !status_out)
        return -EINVAL;
    const bool verify_first = opts && (opts->flags & ZMQG_OPT_VERIFY_FIRST);
    // the host applied the header and replay rules (opts->verdict_in)
    const bool replay_host = opts && (opts->flags & ZMQG_OPT_REPLAY_HOST);
    const int32_t *verdict = replay_host ? opt_verdict_in(opts) : nullptr;
    if (replay_host && (!verify_first || !verdict || zres))
        return -EINVAL;
    // (out_bytes may be 0 under VERIFY_FIRST: a batch of frames with no
    // payload bytes -- empty or under the 33-byte minimum -- stages nothing,
    // and each such frame still gets its own status)
    const uint64_t out_bytes = opt_out_bytes(opts);
    hipStream_t st = (hipStream_t) stream;
    ZCHECK(ctx, hipSetDevice(ctx->device));
    // the workspace and the call state are shared with the ctx's other
    // streams: this call runs after the work queued on the last one
    int rc = order_after_last(ctx, st);
    if (rc)
        return rc;
    rc = ensure_workspace(ctx, n, st);
    if (rc)
        return rc;
    Workspace &w = ctx->ws;
    uint8_t *const out_user = out;
    if (verify_first) {
        // the staging area mirrors `out`: same offsets, same alignment mod 16
        const size_t need = out_bytes + 16;
        if (need > w.stage_cap) {
            if (w.stage)
                ZCHECK(ctx, hipFreeAsync(w.stage, st));
            w.stage = nullptr;
            ZCHECK(ctx, hipMallocAsync((void **) &w.stage, need, st));
            w.stage_cap = need;
        }
        out = w.stage + ((uintptr_t) out_user & 15u);
    }
    const uint32_t nn = (uint32_t) n;
    int G = lanes_per_frame(ctx, nn);
    // several sessions: the replay tables after the frame kernel; the host's
    // verdicts need neither those nor the one-session look-back
    const bool multi = ctx->sort_bits > 0 && !replay_host;
    FrameCtl ctl{};
    ctl.post = w.post;
    unsigned long long *smax = nullptr;
    if (opts) {
        ctl.max_len = opts->max_len;
        ctl.no_body = opts->max_len && opts->max_len <= kMaxFrameStream;
        ctl.stream_out = (opts->flags & ZMQG_OPT_STREAM_OUT) ? 1u : 0u;
        smax = (unsigned long long *) opts->session_max_out;
    }
    if (verify_first) { // frames whose payload would leave the staging area fail with ZMQG_ERR_BOUND
        ctl.out_check = 1;
        ctl.out_limit = out_bytes;
    }
    const BigRecords R{w.hot, w.pw, w.fin, w.powtab, w.acc, w.cnt, w.chunk_end, w.list_frame};
    ReplayOut rp{};
    rp.vout = w.v;
    rp.psnap = w.psnap;
    rp.peer = ctx->peer;
    if (replay_host) {
        // the frame kernels' peer-nonce snapshot reads zeros (the device
        // table is the host's to keep), and the big-frame finisher's replay
        // prefix is zero: their replay test passes every header-valid frame
        // and k_verify_copy applies the host's verdict over it
        if ((rc = ensure_zero_peer(ctx, st)))
            return rc;
        rp.peer = ctx->zero_peer;
        if (!ctl.no_body)
            ZCHECK(ctx, hipMemsetAsync(w.excl, 0, sizeof(unsigned long long) * nn, st));
    } else if (multi) {
        if (ctx->max_sessions > kReplayMaxSessions)
            rp.iota = w.iota; // (the sort fallback's values)
        if (smax)
            ZCHECK(ctx, hipMemsetAsync(smax, 0, sizeof(unsigned long long) * ctx->max_sessions, st));
    } else {
        rp.excl = w.excl;
        rp.lb_flag = w.lb_flag;
        rp.lb_agg = w.lb_agg;
        rp.lb_inc = w.lb_inc;
        rp.smax = smax;
        // A grid that fits the device at once can use blockIdx as the
        // look-back order (every workgroup becomes resident eventually,
        // whatever the dispatch order); a larger one takes tickets.
        // (a split launch needs that order: its two bodies are told apart by
        // blockIdx; without it the batch runs one lane per frame)
        if (G >= 16 && frames_grid(ctx, G, nn) > (uint64_t) frames_capacity(ctx, G, ctl.stream_out))
            G = 0;
        rp.ordered = frames_grid(ctx, G, nn) <= (uint64_t) frames_capacity(ctx, G, ctl.stream_out) ? 1u : 0u;
    }
    ProfSpan call(ctx, ZMQG_PROF_DECODE_CALL, st);
    ProfSpan main(ctx, ZMQG_PROF_DECODE_MAIN, st);
    launch_frames<true>(ctx, G, nn, st, sid, nullptr, nullptr, in_off, wire_len, in, out_off, out, ctx->sessions,
                        ctx->max_sessions, flags_out, status_out, rp,
                        DecodeHead{sid, in_off, wire_len, in, out_off, out, ctx->sessions, ctx->max_sessions, R,
                                   zflags, (const unsigned long long *) zwalk, (unsigned long long *) zres},
                        w.zs, ctl);
    ZCHECK(ctx, hipGetLastError());
    main.end();
    if (multi && (rc = replay_multi(ctx, nn, sid, st, smax)))
        return rc;
    if (!ctl.no_body) {
        ProfSpan body(ctx, ZMQG_PROF_DECODE_BODY, st);
        hipLaunchKernelGGL(k_body<true>, dim3(body_grid(ctx)), dim3(kBodyThreads), 0, st, w.zs, w.chunk_end, w.hot,
                           w.pw, w.fin, w.powtab, flags_out, status_out, w.acc, w.cnt, w.excl, w.psnap, w.post, zflags);
        ZCHECK(ctx, hipGetLastError());
        hipLaunchKernelGGL(k_post, dim3(body_grid(ctx)), dim3(256), 0, st, w.zs, (const PostOp *) w.post,
                           (uint8_t *) w.powtab);
        ZCHECK(ctx, hipGetLastError());
        body.end();
    }
    if (multi) {
        hipLaunchKernelGGL(k_fixup, dim3((nn + kFixupThreads - 1) / kFixupThreads), dim3(kFixupThreads), 0, st, nn,
                           kMaxFrameStream, w.v, w.psnap, w.excl, w.use_last ? w.last : nullptr, sid,
                           ctx->max_sessions, wire_len, out_off, out, status_out, flags_out, ctx->peer, smax);
        ZCHECK(ctx, hipGetLastError());
    }
    if (verify_first) {
        const uint32_t g = nn < 65536u ? nn : 65536u;
        hipLaunchKernelGGL(k_verify_copy, dim3(g), dim3(256), 0, st, nn, (const uint8_t *) out, out_user, out_off,
                           wire_len, status_out, verdict, flags_out);
        ZCHECK(ctx, hipGetLastError());
    }
    call.end();
    return 0;
}

int zmqg_decode_batch_ex(zmqg_ctx *ctx, uint64_t n, const uint32_t *sid, const uint64_t *in_off,
                         const uint32_t *wire_len, const uint8_t *in, const uint64_t *out_off, uint8_t *out,
                         uint8_t *flags_out, int32_t *status_out, const zmqg_batch_opts *opts, void *stream)
{
    return decode_batch_impl(ctx, n, sid, in_off, wire_len, in, out_off, out, flags_out, status_out, opts, nullptr,
                             nullptr, nullptr, stream);
}

int zmqg_decode_batch(zmqg_ctx *ctx, uint64_t n, const uint32_t *sid, const uint64_t *in_off,
                      const uint32_t *wire_len, const uint8_t *in, const uint64_t *out_off, uint8_t *out,
                      uint8_t *flags_out, int32_t *status_out, void *stream)
{
    return zmqg_decode_batch_ex(ctx, n, sid, in_off, wire_len, in, out_off, out, flags_out, status_out, nullptr,
                                stream);
}

int zmqg_session_max_batch(zmqg_ctx *ctx, uint64_t n, const uint32_t *sid, const uint64_t *in_off,
                           const uint32_t *wire_len, const uint8_t *in, uint64_t *session_max_out, void *stream)
{
    if (!ctx || check_n(n) || !session_max_out)
        return -EINVAL;
    if (n > 0 && (!sid || !in_off || !wire_len || !in))
        return -EINVAL;
    hipStream_t st = (hipStream_t) stream;
    ZCHECK(ctx, hipSetDevice(ctx->device));
    ZCHECK(ctx, hipMemsetAsync(session_max_out, 0, sizeof(uint64_t) * ctx->max_sessions, st));
    if (n == 0)
        return 0;
    hipLaunchKernelGGL(k_session_max, dim3((unsigned) ((n + 255) / 256)), dim3(256), 0, st, (uint32_t) n, sid, in_off,
                       wire_len, in, ctx->max_sessions, (unsigned long long *) session_max_out);
    ZCHECK(ctx, hipGetLastError());
    return 0;
}

// ---------------------------------------------------------------- host forms
static int stage(zmqg_ctx *ctx, size_t bytes)
{
    if (bytes > ctx->pin_bytes) {
        if (ctx->pin)
            ZCHECK(ctx, hipHostFree(ctx->pin));
        ctx->pin = nullptr;
        ctx->pin_bytes = 0;
        ZCHECK(ctx, hipHostMalloc((void **) &ctx->pin, bytes));
        ctx->pin_bytes = bytes;
    }
    if (bytes > ctx->dbuf_bytes) {
        if (ctx->dbuf)
            ZCHECK(ctx, hipFree(ctx->dbuf));
        ctx->dbuf = nullptr;
        ctx->dbuf_bytes = 0;
        ZCHECK(ctx, hipMalloc((void **) &ctx->dbuf, bytes));
        ctx->dbuf_bytes = bytes;
    }
    return 0;
}

static size_t al(size_t x)
{
    return (x + 255) & ~(size_t) 255;
}

int zmqg_encode_host(zmqg_ctx *ctx, uint64_t n, const uint32_t *sid, const uint64_t *nonce, const uint8_t *flags,
                     const uint64_t *in_off, const uint32_t *len, const uint8_t *in, uint64_t in_bytes,
                     const uint64_t *out_off, uint8_t *out, uint64_t out_bytes)
{
    if (!ctx || check_n(n))
        return -EINVAL;
    if (n == 0)
        return 0;
    if (!sid || !nonce || !flags || !in_off || !len || !in || !out_off || !out)
        return -EINVAL;
    std::lock_guard<std::mutex> lk(ctx->mu);
    for (uint64_t i = 0; i < n; ++i) {
        if (sid[i] >= ctx->max_sessions || in_off[i] + len[i] > in_bytes)
            return -EINVAL;
        if (out_off[i] + zmqg_wire_size(flags[i], ctx->h_downgrade[sid[i]], len[i]) > out_bytes)
            return -EINVAL;
    }
    const size_t o_sid = 0, o_nonce = al(o_sid + 4 * n), o_flags = al(o_nonce + 8 * n), o_inoff = al(o_flags + n),
                 o_len = al(o_inoff + 8 * n), o_outoff = al(o_len + 4 * n), o_in = al(o_outoff + 8 * n),
                 o_out = al(o_in + in_bytes), total = al(o_out + out_bytes);
    int rc = stage(ctx, total);
    if (rc)
        return rc;
    uint8_t *h = ctx->pin, *d = ctx->dbuf;
    memcpy(h + o_sid, sid, 4 * n);
    memcpy(h + o_nonce, nonce, 8 * n);
    memcpy(h + o_flags, flags, n);
    memcpy(h + o_inoff, in_off, 8 * n);
    memcpy(h + o_len, len, 4 * n);
    memcpy(h + o_outoff, out_off, 8 * n);
    memcpy(h + o_in, in, in_bytes);
    hipStream_t st = ctx->own_stream;
    ZCHECK(ctx, hipSetDevice(ctx->device));
    ZCHECK(ctx, hipMemcpyAsync(d, h, o_out, hipMemcpyHostToDevice, st));
    rc = zmqg_encode_batch(ctx, n, (uint32_t *) (d + o_sid), (uint64_t *) (d + o_nonce), d + o_flags,
                           (uint64_t *) (d + o_inoff), (uint32_t *) (d + o_len), d + o_in,
                           (uint64_t *) (d + o_outoff), d + o_out, st);
    if (rc)
        return rc;
    ZCHECK(ctx, hipMemcpyAsync(h + o_out, d + o_out, out_bytes, hipMemcpyDeviceToHost, st));
    ZCHECK(ctx, hipStreamSynchronize(st));
    memcpy(out, h + o_out, out_bytes);
    return 0;
}

// The per-message buffer: page-locked and device-mapped, the kernels read the
// message and write the result in place.
static int msg_stage(zmqg_ctx *ctx, size_t bytes)
{
    if (bytes <= ctx->mpin_bytes)
        return 0;
    size_t cap = ctx->mpin_bytes ? ctx->mpin_bytes : 65536;
    while (cap < bytes)
        cap *= 2;
    if (ctx->mpin)
        ZCHECK(ctx, hipHostFree(ctx->mpin));
    ctx->mpin = nullptr;
    ctx->mpin_bytes = 0;
    hipError_t e = hipHostMalloc((void **) &ctx->mpin, cap, hipHostMallocMapped | hipHostMallocPortable);
    if (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation)
        return -ENOMEM;
    ZCHECK(ctx, e);
    void *d = nullptr;
    ZCHECK(ctx, hipHostGetDevicePointer(&d, ctx->mpin, 0));
    ctx->mpin_dev = (uint8_t *) d;
    ctx->mpin_bytes = cap;
    return 0;
}

// how long a per-message call polls its completion word before it
// synchronises the stream instead
static const int kMsgSpinUs = 200;

// descriptors of the one message: sid, len, nonce / in_off, out_off, flags
struct MsgDesc {
    uint32_t sid, len;
    uint64_t nonce, in_off, out_off;
    uint8_t flags, flags_out, pad[2];
    int32_t status;
    uint32_t done; // k_msg's completion word
};

// Wait for k_msg's completion word (the kernel's last write, system scope)
// rather than for the stream: a poll of host memory sees it a few
// microseconds before a stream synchronisation returns.  The spin is bounded
// by a few times the kernel's own latency (~5-7 us at <= 4 KiB, DESIGN.md
// section 6): a call queued behind a long batch on another stream, or a
// failed launch, falls back to the stream synchronisation instead of
// holding a core (and the ctx's lock) in the loop.
static int msg_wait(zmqg_ctx *ctx, const MsgDesc *h, hipStream_t st)
{
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t spin = 0;; ++spin) {
        if (__atomic_load_n(&h->done, __ATOMIC_ACQUIRE))
            return 0;
        if ((spin & 63u) == 63u &&
            std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(kMsgSpinUs))
            break;
    }
    ZCHECK(ctx, hipStreamSynchronize(st));
    return __atomic_load_n(&h->done, __ATOMIC_ACQUIRE) ? 0 : -EIO;
}

// The per-message calls run on the ctx's own stream; work the ctx issued
// before on another stream (a batch on the caller's stream) shares the
// session tables and the workspace, so own_stream waits for it first.
static int msg_order(zmqg_ctx *ctx)
{
    return order_after_last(ctx, ctx->own_stream);
}

int zmqg_encode_msg(zmqg_ctx *ctx, uint32_t sid, uint64_t nonce, uint8_t flags, const uint8_t *in, uint32_t len,
                    uint8_t *out)
{
    if (!ctx || (len && !in) || !out)
        return -EINVAL;
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (sid >= ctx->max_sessions)
        return -EINVAL;
    const uint64_t W = zmqg_wire_size(flags, ctx->h_downgrade[sid], len);
    const size_t o_in = al(sizeof(MsgDesc)), o_out = al(o_in + len);
    int rc = msg_stage(ctx, o_out + W);
    if (rc)
        return rc;
    MsgDesc *h = (MsgDesc *) ctx->mpin;
    *h = MsgDesc{sid, len, nonce, 0, 0, flags, 0, {0, 0}, 0, 0};
    if (len && (W > kMsgMaxStream || len > kMsgInlineMax)) // (else the message travels as a kernel argument)
        memcpy(ctx->mpin + o_in, in, len);
    uint8_t *d = ctx->mpin_dev;
    MsgDesc *dd = (MsgDesc *) d;
    hipStream_t st = ctx->own_stream;
    ZCHECK(ctx, hipSetDevice(ctx->device));
    if ((rc = msg_order(ctx)))
        return rc;
    if (W <= kMsgMaxStream) {
        // one wave, descriptors as arguments (curve_msg.hpp)
        MsgArgs a{d + o_in, d + o_out, ctx->sessions, ctx->peer, nullptr, &dd->status, &dd->done, nonce, sid, len,
                  ctx->max_sessions, flags};
        launch_msg<false>(st, a, in, len);
        ZCHECK(ctx, hipGetLastError());
        if ((rc = msg_wait(ctx, h, st)))
            return rc;
        memcpy(out, ctx->mpin + o_out, W);
        return 0;
    }
    // the frame's length bounds the batch: a frame within the frame kernel's
    // range is one launch, with no large-frame launches behind it
    zmqg_batch_opts o{};
    o.size = sizeof o;
    o.max_len = len ? len : 1u;
    rc = zmqg_encode_batch_ex(ctx, 1, &dd->sid, &dd->nonce, &dd->flags, &dd->in_off, &dd->len, d + o_in,
                              &dd->out_off, d + o_out, &o, st);
    if (rc)
        return rc;
    ZCHECK(ctx, hipStreamSynchronize(st));
    memcpy(out, ctx->mpin + o_out, W);
    return 0;
}

int zmqg_decode_msg(zmqg_ctx *ctx, uint32_t sid, const uint8_t *in, uint32_t wire_len, uint8_t *out,
                    uint8_t *flags_out, int32_t *status_out)
{
    if (!ctx || (wire_len && !in) || (wire_len > 33u && !out) || !flags_out || !status_out)
        return -EINVAL;
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (sid >= ctx->max_sessions)
        return -EINVAL;
    const uint64_t P = wire_len >= 33u ? wire_len - 33u : 0u; // (a shorter frame fails its header checks)
    const size_t o_in = al(sizeof(MsgDesc)), o_out = al(o_in + wire_len);
    int rc = msg_stage(ctx, o_out + P);
    if (rc)
        return rc;
    MsgDesc *h = (MsgDesc *) ctx->mpin;
    *h = MsgDesc{sid, wire_len, 0, 0, 0, 0, 0, {0, 0}, 0, 0};
    if (wire_len && (wire_len > kMsgMaxStream || wire_len > kMsgInlineMax))
        memcpy(ctx->mpin + o_in, in, wire_len);
    uint8_t *d = ctx->mpin_dev;
    MsgDesc *dd = (MsgDesc *) d;
    hipStream_t st = ctx->own_stream;
    ZCHECK(ctx, hipSetDevice(ctx->device));
    if ((rc = msg_order(ctx)))
        return rc;
    if (wire_len <= kMsgMaxStream) {
        MsgArgs a{d + o_in, d + o_out, ctx->sessions, ctx->peer, &dd->flags_out, &dd->status, &dd->done, 0, sid,
                  wire_len, ctx->max_sessions, 0};
        launch_msg<true>(st, a, in, wire_len);
        ZCHECK(ctx, hipGetLastError());
        if ((rc = msg_wait(ctx, h, st)))
            return rc;
        *status_out = h->status;
        *flags_out = h->status == 0 ? h->flags_out : 0;
        if (h->status == 0 && P)
            memcpy(out, ctx->mpin + o_out, P);
        return 0;
    }
    zmqg_batch_opts o{};
    o.size = sizeof o;
    o.max_len = wire_len ? wire_len : 1u;
    rc = zmqg_decode_batch_ex(ctx, 1, &dd->sid, &dd->in_off, &dd->len, d + o_in, &dd->out_off, d + o_out,
                              &dd->flags_out, &dd->status, &o, st);
    if (rc)
        return rc;
    ZCHECK(ctx, hipStreamSynchronize(st));
    *status_out = h->status;
    *flags_out = h->status == 0 ? h->flags_out : 0;
    if (h->status == 0 && P)
        memcpy(out, ctx->mpin + o_out, P);
    return 0;
}

int zmqg_decode_host(zmqg_ctx *ctx, uint64_t n, const uint32_t *sid, const uint64_t *in_off,
                     const uint32_t *wire_len, const uint8_t *in, uint64_t in_bytes, const uint64_t *out_off,
                     uint8_t *out, uint64_t out_bytes, uint8_t *flags_out, int32_t *status_out)
{
    if (!ctx || check_n(n))
        return -EINVAL;
    if (n == 0)
        return 0;
    if (!sid || !in_off || !wire_len || !in || !out_off || !out || !flags_out || !status_out)
        return -EINVAL;
    std::lock_guard<std::mutex> lk(ctx->mu);
    for (uint64_t i = 0; i < n; ++i) {
        if (sid[i] >= ctx->max_sessions || in_off[i] + wire_len[i] > in_bytes)
            return -EINVAL;
        if (wire_len[i] >= 33 && out_off[i] + wire_len[i] - 33 > out_bytes)
            return -EINVAL;
    }
    const size_t o_sid = 0, o_inoff = al(o_sid + 4 * n), o_wl = al(o_inoff + 8 * n), o_outoff = al(o_wl + 4 * n),
                 o_in = al(o_outoff + 8 * n), o_out = al(o_in + in_bytes), o_fl = al(o_out + out_bytes),
                 o_st = al(o_fl + n), total = al(o_st + 4 * n);
    int rc = stage(ctx, total);
    if (rc)
        return rc;
    uint8_t *h = ctx->pin, *d = ctx->dbuf;
    memcpy(h + o_sid, sid, 4 * n);
    memcpy(h + o_inoff, in_off, 8 * n);
    memcpy(h + o_wl, wire_len, 4 * n);
    memcpy(h + o_outoff, out_off, 8 * n);
    memcpy(h + o_in, in, in_bytes);
    memcpy(h + o_out, out, out_bytes); // bytes of `out` outside the frames are preserved
    hipStream_t st = ctx->own_stream;
    ZCHECK(ctx, hipSetDevice(ctx->device));
    ZCHECK(ctx, hipMemcpyAsync(d, h, o_fl, hipMemcpyHostToDevice, st));
    rc = zmqg_decode_batch(ctx, n, (uint32_t *) (d + o_sid), (uint64_t *) (d + o_inoff), (uint32_t *) (d + o_wl),
                           d + o_in, (uint64_t *) (d + o_outoff), d + o_out, d + o_fl, (int32_t *) (d + o_st), st);
    if (rc)
        return rc;
    ZCHECK(ctx, hipMemcpyAsync(h + o_out, d + o_out, total - o_out, hipMemcpyDeviceToHost, st));
    ZCHECK(ctx, hipStreamSynchronize(st));
    memcpy(out, h + o_out, out_bytes);
    memcpy(flags_out, h + o_fl, n);
    memcpy(status_out, h + o_st, 4 * n);
    return 0;
}

static int zmtp_temp(zmqg_ctx *ctx, size_t need, hipStream_t st)
{
    ZmtpWs &z = ctx->zw;
    if (need <= z.temp_bytes)
        return 0;
    size_t cap = z.temp_bytes ? z.temp_bytes : 4096;
    while (cap < need)
        cap *= 2;
    if (z.temp)
        ZCHECK(ctx, hipFreeAsync(z.temp, st));
    z.temp = nullptr;
    z.temp_bytes = 0;
    ZCHECK(ctx, hipMallocAsync(&z.temp, cap, st));
    z.temp_bytes = cap;
    return 0;
}

int zmqg_encode_zmtp(zmqg_ctx *ctx, uint64_t n, const uint32_t *sid, const uint64_t *nonce, const uint8_t *flags,
                     const uint64_t *in_off, const uint32_t *len, const uint8_t *in, uint8_t *out,
                     uint64_t *frame_off, void *stream)
{
    if (!ctx || check_n(n))
        return -EINVAL;
    if (!frame_off)
        return -EINVAL;
    hipStream_t st = (hipStream_t) stream;
    ZCHECK(ctx, hipSetDevice(ctx->device));
    if (n == 0)
        return hipMemsetAsync(frame_off, 0, sizeof(uint64_t), st) == hipSuccess ? 0 : -EIO;
    if (!sid || !nonce || !flags || !in_off || !len || !in || !out)
        return -EINVAL;
    ZmtpWs &z = ctx->zw;
    int rc;
    if (n > z.n_cap) {
        uint64_t cap = z.n_cap ? z.n_cap : 1024;
        while (cap < n)
            cap *= 2;
        if ((rc = grow(ctx, z.F, cap + 1, st)) || (rc = grow(ctx, z.wire_off, cap, st)))
            return rc;
        z.n_cap = cap;
    }
    size_t need = 0;
    ZCHECK(ctx, hipcub::DeviceScan::ExclusiveSum(nullptr, need, z.F, frame_off, (int) (n + 1), st));
    if ((rc = zmtp_temp(ctx, need, st)))
        return rc;
    const unsigned g1 = (unsigned) ((n + 1 + 255) / 256), g0 = (unsigned) ((n + 255) / 256);
    hipLaunchKernelGGL(k_zmtp_sizes, dim3(g1), dim3(256), 0, st, n, sid, flags, len, ctx->sessions,
                       ctx->max_sessions, z.F);
    ZCHECK(ctx, hipGetLastError());
    size_t tb = z.temp_bytes;
    ZCHECK(ctx, hipcub::DeviceScan::ExclusiveSum(z.temp, tb, z.F, frame_off, (int) (n + 1), st));
    hipLaunchKernelGGL(k_zmtp_headers, dim3(g0), dim3(256), 0, st, n, frame_off, out, z.wire_off);
    ZCHECK(ctx, hipGetLastError());
    return zmqg_encode_batch(ctx, n, sid, nonce, flags, in_off, len, in, z.wire_off, out, stream);
}

int zmqg_decode_zmtp_async(zmqg_ctx *ctx, uint32_t sid, const uint8_t *in, uint64_t in_bytes, int64_t max_msg_size,
                           uint64_t max_frames, uint64_t *frame_in_off, uint32_t *frame_len, uint64_t *out_off,
                           uint8_t *out, uint8_t *flags_out, int32_t *status_out, zmqg_zmtp_result *result,
                           void *stream)
{
    if (!ctx || !result || sid >= ctx->max_sessions || in_bytes > 0x7fffffffull || check_n(max_frames))
        return -EINVAL;
    hipStream_t st = (hipStream_t) stream;
    ZCHECK(ctx, hipSetDevice(ctx->device));
    if (in_bytes == 0 || max_frames == 0) {
        ZCHECK(ctx, hipMemsetAsync(result, 0, sizeof *result, st));
        return 0;
    }
    if (!in || !frame_in_off || !frame_len || !out_off || !out || !flags_out || !status_out)
        return -EINVAL;
    std::lock_guard<std::mutex> lk(ctx->mu);
    ZmtpWs &z = ctx->zw;
    int rc;
    const uint64_t nwg = (in_bytes + kZmtpWgBytes - 1) / kZmtpWgBytes;
    if (nwg > z.g_cap) {
        uint64_t cap = z.g_cap ? z.g_cap : 64;
        while (cap < nwg)
            cap *= 2;
        if ((rc = grow(ctx, z.cand_wg, cap * kZmtpWgCap, st)) || (rc = grow(ctx, z.count_wg, cap + 1, st)) ||
            (rc = grow(ctx, z.off_wg, cap + 1, st)) || (rc = grow(ctx, z.first_w, cap + 1, st)) ||
            (rc = grow(ctx, z.count16, cap + 8, st)))
            return rc;
        z.g_cap = cap;
    }
    // candidates: signatures are >= 8 bytes apart, one candidate each
    const uint64_t ccap = in_bytes / 8 + 2;
    if (ccap > z.c_cap) {
        uint64_t cap = z.c_cap ? z.c_cap : 1024;
        while (cap < ccap)
            cap *= 2;
        if ((rc = grow(ctx, z.cand, cap, st)) || (rc = grow(ctx, z.nb, cap, st)) || (rc = grow(ctx, z.wid, cap, st)) ||
            (rc = grow(ctx, z.cdesc, cap, st)) || (rc = grow(ctx, z.cflag, cap, st)))
            return rc;
        z.c_cap = cap;
    }
    if (max_frames > z.f_cap) {
        uint64_t cap = z.f_cap ? z.f_cap : 1024;
        while (cap < max_frames)
            cap *= 2;
        if ((rc = grow(ctx, z.run, 2 * (cap + 1), st)) || (rc = grow(ctx, z.runpre, cap + 1, st)) ||
            (rc = grow(ctx, z.sid_fill, cap, st)) || (rc = grow(ctx, z.fflags, cap, st)))
            return rc;
        z.f_cap = cap;
    }
    if (!z.walk && (rc = grow(ctx, z.walk, 1, st)))
        return rc;
    const uint32_t g = (uint32_t) nwg;
    // persistent grids over device-side counts: enough workgroups to cover
    // config-2-sized streams in one pass
    const uint32_t pg = (uint32_t) (ctx->cus > 0 ? 4 * ctx->cus : 1024);
    const uint64_t *m_p = z.off_wg + nwg; // the candidate count, on the device
    // 1. candidates, in stream order: per-workgroup lists, their counts'
    // exclusive sum, the lists concatenated with their links
    hipLaunchKernelGGL(k_zmtp_scan, dim3(g), dim3(kZmtpThreads), 0, st, in, in_bytes, max_msg_size, z.cand_wg,
                       z.count_wg, z.count16);
    ZCHECK(ctx, hipGetLastError());
    // The lists' offsets: up to 8,192 lists (128 MiB of stream) each
    // compaction workgroup sums the 16-bit counts before its own list (a few
    // 16-byte loads per thread, L2-resident) -- no launch of their own; above
    // that, one hipCUB scan of the counts.  (ZMQG_ZMTP_CUB: the large-stream
    // form at any size, for its tests)
    const bool inline_sum = nwg <= kZmtpInlineSumLists && !getenv("ZMQG_ZMTP_CUB");
    if (!inline_sum) {
        size_t need = 0;
        ZCHECK(ctx, hipcub::DeviceScan::ExclusiveSum(nullptr, need, z.count_wg, z.off_wg, (int) (nwg + 1), st));
        if ((rc = zmtp_temp(ctx, need, st)))
            return rc;
        ZCHECK(ctx, hipMemsetAsync(z.count_wg + nwg, 0, sizeof(uint64_t), st));
        size_t tb = z.temp_bytes;
        ZCHECK(ctx, hipcub::DeviceScan::ExclusiveSum(z.temp, tb, z.count_wg, z.off_wg, (int) (nwg + 1), st));
    }
    hipLaunchKernelGGL(k_zmtp_compact, dim3((g + kZmtpCompactLists - 1) / kZmtpCompactLists), dim3(kZmtpThreads), 0, st, in, in_bytes, (const uint64_t *) z.cand_wg,
                       (const uint64_t *) z.count_wg, inline_sum ? (const uint16_t *) z.count16 : nullptr, z.off_wg,
                       g, z.cand, z.cdesc, z.cflag, z.nb, z.first_w, z.wid);
    ZCHECK(ctx, hipGetLastError());
    // 2. the first unlinked candidate after each list, then the walk (one launch)
    hipLaunchKernelGGL(k_zmtp_next_walk, dim3(1), dim3(kZmtpNextThreads), 0, st, in, in_bytes, max_msg_size,
                       max_frames, (const uint64_t *) z.cand, (const uint64_t *) z.cdesc, m_p,
                       (const uint64_t *) z.nb, z.first_w,
                       (const uint32_t *) z.wid, nwg, z.run, z.runpre, z.walk);
    ZCHECK(ctx, hipGetLastError());
    // 3. descriptors (empty frames up to max_frames); each payload goes to
    // its body's offset in `out`, so no offsets scan is needed
    hipLaunchKernelGGL(k_zmtp_frames, dim3(pg), dim3(kZmtpThreads), 0, st, in, in_bytes, (const uint64_t *) z.cdesc,
                       (const uint8_t *) z.cflag, m_p,
                       (const uint64_t *) z.run, (const uint64_t *) z.runpre, (const ZmtpWalk *) z.walk, max_frames,
                       frame_in_off, frame_len, z.fflags, z.sid_fill, sid, out_off,
                       (unsigned long long *) ((char *) z.walk + offsetof(ZmtpWalk, out_bytes)));
    ZCHECK(ctx, hipGetLastError());
    // the decode over max_frames (the empty frames fail as malformed and
    // write nothing else); a maxmsgsize within the frame kernel's range bounds
    // every frame, so the large-frame launches are skipped
    zmqg_batch_opts o{};
    o.size = sizeof o;
    if (max_msg_size >= 0 && (uint64_t) max_msg_size <= kMaxFrameStream)
        o.max_len = max_msg_size > 0 ? (uint64_t) max_msg_size : 1u;
    // (the frames' MORE / COMMAND bits ORed into flags_out, and the call's
    // result copied from the parse state, by the decode's frame kernel)
    return decode_batch_impl(ctx, max_frames, z.sid_fill, frame_in_off, frame_len, in, out_off, out, flags_out,
                             status_out, o.max_len ? &o : nullptr, z.fflags, z.walk, result, stream);
}

int zmqg_decode_zmtp(zmqg_ctx *ctx, uint32_t sid, const uint8_t *in, uint64_t in_bytes, int64_t max_msg_size,
                     uint64_t max_frames, uint64_t *frame_in_off, uint32_t *frame_len, uint64_t *out_off,
                     uint8_t *out, uint8_t *flags_out, int32_t *status_out, zmqg_zmtp_result *result, void *stream)
{
    if (!ctx || !result)
        return -EINVAL;
    memset(result, 0, sizeof *result);
    hipStream_t st = (hipStream_t) stream;
    ZCHECK(ctx, hipSetDevice(ctx->device));
    int rc;
    ZmtpWs &z = ctx->zw;
    if (!z.res) {
        // the result lands in mapped host memory: after the stream's
        // synchronisation the host reads it there, with no copy queued behind
        // the decode (a device-to-host copy into the caller's pageable
        // struct cost a staged transfer per call: 154-157 against 139-142 us
        // for the config-2 stream; polling a completion word set by one more
        // kernel instead of synchronising measured 153 us)
        ZCHECK(ctx, hipHostMalloc((void **) &z.res, sizeof *z.res, hipHostMallocMapped | hipHostMallocPortable));
        void *d = nullptr;
        ZCHECK(ctx, hipHostGetDevicePointer(&d, z.res, 0));
        z.res_dev = (ZmtpResHost *) d;
    }
    rc = zmqg_decode_zmtp_async(ctx, sid, in, in_bytes, max_msg_size, max_frames, frame_in_off, frame_len, out_off,
                                out, flags_out, status_out, &z.res_dev->r, stream);
    if (rc)
        return rc;
    ZCHECK(ctx, hipStreamSynchronize(st));
    memcpy(result, &z.res->r, sizeof *result); // the one read back of the call
    return 0;
}

int zmqg_scalarmult_batch(zmqg_ctx *ctx, uint64_t n, const uint8_t *scalar, const uint8_t *point, uint8_t *out,
                          int32_t *status_out, void *stream)
{
    if (!ctx || check_n(n))
        return -EINVAL;
    if (n == 0)
        return 0;
    if (!scalar || !out || !status_out)
        return -EINVAL;
    ZCHECK(ctx, hipSetDevice(ctx->device));
    hipLaunchKernelGGL(k_scalarmult, dim3((unsigned) ((n + 63) / 64)), dim3(64), 0, (hipStream_t) stream,
                       (uint32_t) n, scalar, point, out, status_out);
    ZCHECK(ctx, hipGetLastError());
    return 0;
}

int zmqg_box_beforenm_batch(zmqg_ctx *ctx, uint64_t n, const uint8_t *pk, const uint8_t *sk, uint8_t *k_out,
                            int32_t *status_out, void *stream)
{
    if (!ctx || check_n(n))
        return -EINVAL;
    if (n == 0)
        return 0;
    if (!pk || !sk || !k_out || !status_out)
        return -EINVAL;
    ZCHECK(ctx, hipSetDevice(ctx->device));
    hipLaunchKernelGGL(k_beforenm, dim3((unsigned) ((n + 63) / 64)), dim3(64), 0, (hipStream_t) stream,
                       (uint32_t) n, pk, sk, k_out, status_out);
    ZCHECK(ctx, hipGetLastError());
    return 0;
}

int zmqg_box_afternm_batch(zmqg_ctx *ctx, uint64_t n, const uint8_t *key, const uint8_t *nonce,
                           const uint64_t *in_off, const uint32_t *len, const uint8_t *in, const uint64_t *out_off,
                           uint8_t *out, void *stream)
{
    if (!ctx || check_n(n))
        return -EINVAL;
    if (n == 0)
        return 0;
    if (!key || !nonce || !in_off || !len || !in || !out_off || !out)
        return -EINVAL;
    ZCHECK(ctx, hipSetDevice(ctx->device));
    hipLaunchKernelGGL(k_box<false>, dim3((unsigned) ((n + 63) / 64)), dim3(64), 0, (hipStream_t) stream,
                       (uint32_t) n, key, nonce, in_off, len, in, out_off, out, (int32_t *) nullptr);
    ZCHECK(ctx, hipGetLastError());
    return 0;
}

int zmqg_box_open_afternm_batch(zmqg_ctx *ctx, uint64_t n, const uint8_t *key, const uint8_t *nonce,
                                const uint64_t *in_off, const uint32_t *len, const uint8_t *in,
                                const uint64_t *out_off, uint8_t *out, int32_t *status_out, void *stream)
{
    if (!ctx || check_n(n))
        return -EINVAL;
    if (n == 0)
        return 0;
    if (!key || !nonce || !in_off || !len || !in || !out_off || !out || !status_out)
        return -EINVAL;
    ZCHECK(ctx, hipSetDevice(ctx->device));
    hipLaunchKernelGGL(k_box<true>, dim3((unsigned) ((n + 63) / 64)), dim3(64), 0, (hipStream_t) stream,
                       (uint32_t) n, key, nonce, in_off, len, in, out_off, out, status_out);
    ZCHECK(ctx, hipGetLastError());
    return 0;
}

int zmqg_z85_encode_batch(zmqg_ctx *ctx, uint64_t n, const uint64_t *in_off, const uint32_t *len, const uint8_t *in,
                          const uint64_t *out_off, char *out, int32_t *status_out, void *stream)
{
    if (!ctx || check_n(n))
        return -EINVAL;
    if (n == 0)
        return 0;
    if (!in_off || !len || !in || !out_off || !out || !status_out)
        return -EINVAL;
    ZCHECK(ctx, hipSetDevice(ctx->device));
    hipLaunchKernelGGL(k_z85_encode, dim3((unsigned) ((n + 255) / 256)), dim3(256), 0, (hipStream_t) stream,
                       (uint32_t) n, in_off, len, in, out_off, out, status_out);
    ZCHECK(ctx, hipGetLastError());
    return 0;
}

int zmqg_z85_decode_batch(zmqg_ctx *ctx, uint64_t n, const uint64_t *in_off, const uint32_t *len, const char *in,
                          const uint64_t *out_off, uint8_t *out, int32_t *status_out, void *stream)
{
    if (!ctx || check_n(n))
        return -EINVAL;
    if (n == 0)
        return 0;
    if (!in_off || !len || !in || !out_off || !out || !status_out)
        return -EINVAL;
    ZCHECK(ctx, hipSetDevice(ctx->device));
    hipLaunchKernelGGL(k_z85_decode, dim3((unsigned) ((n + 255) / 256)), dim3(256), 0, (hipStream_t) stream,
                       (uint32_t) n, in_off, len, in, out_off, out, status_out);
    ZCHECK(ctx, hipGetLastError());
    return 0;
}

int zmqg_host_alloc(zmqg_ctx *ctx, uint64_t bytes, void **ptr_out)
{
    if (!ctx || !ptr_out || bytes == 0)
        return -EINVAL;
    *ptr_out = nullptr;
    ZCHECK(ctx, hipSetDevice(ctx->device));
    // page-locked and mapped; coherent (fine-grained), so kernel writes are
    // visible to the host once a fence behind the batch has been reached
    void *p = nullptr;
    hipError_t e = hipHostMalloc(&p, bytes, hipHostMallocMapped | hipHostMallocPortable);
    if (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation)
        return -ENOMEM;
    ZCHECK(ctx, e);
    *ptr_out = p;
    return 0;
}

int zmqg_host_free(zmqg_ctx *ctx, void *ptr)
{
    if (!ctx || !ptr)
        return -EINVAL;
    ZCHECK(ctx, hipHostFree(ptr));
    return 0;
}

int zmqg_ctx_stream(zmqg_ctx *ctx, void **stream_out)
{
    if (!ctx || !stream_out)
        return -EINVAL;
    *stream_out = (void *) ctx->own_stream;
    return 0;
}

int zmqg_fence_record(zmqg_ctx *ctx, void *stream, uint64_t *fence_out)
{
    if (!ctx || !fence_out)
        return -EINVAL;
    std::lock_guard<std::mutex> lk(ctx->fence_mu);
    hipEvent_t ev;
    if (!ctx->fence_pool.empty()) {
        ev = ctx->fence_pool.back();
        ctx->fence_pool.pop_back();
    } else {
        ZCHECK(ctx, hipSetDevice(ctx->device));
        ZCHECK(ctx, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    }
    hipError_t e = hipEventRecord(ev, (hipStream_t) stream);
    if (e != hipSuccess) {
        ctx->fence_pool.push_back(ev);
        ZCHECK(ctx, e);
    }
    ctx->fences.emplace_back(++ctx->fence_ctr, ev);
    *fence_out = ctx->fence_ctr;
    return 0;
}

// The host function behind a notifying fence (zmqg_fence_record_notify): it
// runs on a HIP runtime thread once the stream has passed the fence, marks
// the fence reached and writes the caller's eventfd.  No HIP call in here.
namespace {
struct FenceNote {
    zmqg_ctx *ctx;
    uint64_t id;
    int fd;
};
} // namespace

static void fence_notify_fn(void *p)
{
    FenceNote *n = (FenceNote *) p;
    zmqg_ctx *ctx = n->ctx;
    {
        std::lock_guard<std::mutex> lk(ctx->notify_mu);
        ctx->notified.push_back(n->id);
    }
    const uint64_t one = 1;
    ssize_t r;
    do
        r = write(n->fd, &one, sizeof one);
    while (r < 0 && errno == EINTR);
    delete n;
    ctx->notify_pending.fetch_sub(1, std::memory_order_release); // (last touch of the ctx)
}

#ifndef ZMQG_BUILD_ID
#define ZMQG_BUILD_ID "unstamped unstamped"
#endif
const char *zmqg_build_id(void)
{
    return ZMQG_BUILD_ID;
}

int zmqg_fence_record_notify(zmqg_ctx *ctx, void *stream, int fd, uint64_t *fence_out)
{
    if (!ctx || !fence_out || fd < 0)
        return -EINVAL;
    int rc = zmqg_fence_record(ctx, stream, fence_out);
    if (rc)
        return rc;
    FenceNote *n = new FenceNote{ctx, *fence_out, fd};
    ctx->notify_pending.fetch_add(1, std::memory_order_relaxed);
    // after the fence's event in stream order: when it runs, the event has
    // completed and so has every kernel of the batches before it
    hipError_t e = hipLaunchHostFunc((hipStream_t) stream, fence_notify_fn, n);
    if (e != hipSuccess) {
        delete n;
        ctx->notify_pending.fetch_sub(1, std::memory_order_release);
        ZCHECK(ctx, e);
    }
    return 0;
}

// Wait for the notifications queued on the ctx, at most ~10 s: a stream that
// never reaches its host function (a stuck kernel, a stream error) leaves
// -ETIMEDOUT instead of a hang; the caller must then keep the eventfd open.
static int notify_wait(zmqg_ctx *ctx)
{
    const auto t_end = std::chrono::steady_clock::now() + std::chrono::seconds(10);
    while (ctx->notify_pending.load(std::memory_order_acquire) > 0) {
        if (std::chrono::steady_clock::now() > t_end)
            return -ETIMEDOUT;
        sched_yield();
    }
    return 0;
}

int zmqg_notify_quiesce(zmqg_ctx *ctx)
{
    if (!ctx)
        return -EINVAL;
    return notify_wait(ctx);
}

// whether fence `id` has been marked reached by its notification (and
// forget the marks of fences no longer pending)
static bool fence_notified(zmqg_ctx *ctx, uint64_t id)
{
    std::lock_guard<std::mutex> lk(ctx->notify_mu);
    bool hit = false;
    for (size_t i = 0; i < ctx->notified.size();) {
        const uint64_t v = ctx->notified[i];
        bool pending = false;
        for (auto &f : ctx->fences)
            pending = pending || f.first == v;
        if (v == id)
            hit = true;
        if (v == id || !pending)
            ctx->notified.erase(ctx->notified.begin() + (long) i);
        else
            ++i;
    }
    return hit;
}

// 1 reached (and released), 0 pending, <0 error; `block` waits for it
static int fence_check(zmqg_ctx *ctx, uint64_t fence, bool block)
{
    if (!ctx || fence == 0)
        return -EINVAL;
    std::lock_guard<std::mutex> lk(ctx->fence_mu);
    if (fence > ctx->fence_ctr)
        return -EINVAL;
    for (size_t i = 0; i < ctx->fences.size(); ++i) {
        if (ctx->fences[i].first != fence)
            continue;
        hipEvent_t ev = ctx->fences[i].second;
        if (!fence_notified(ctx, fence)) {
            hipError_t e = block ? hipEventSynchronize(ev) : hipEventQuery(ev);
            if (e == hipErrorNotReady)
                return 0;
            ZCHECK(ctx, e);
        }
        ctx->fences.erase(ctx->fences.begin() + (long) i);
        ctx->fence_pool.push_back(ev);
        return 1;
    }
    return 1; // released earlier
}

int zmqg_fence_query(zmqg_ctx *ctx, uint64_t fence)
{
    return fence_check(ctx, fence, false);
}

int zmqg_fence_wait(zmqg_ctx *ctx, uint64_t fence)
{
    const int rc = fence_check(ctx, fence, true);
    return rc < 0 ? rc : 0;
}

} // extern "C"
