// curve_zmtp.hpp -- ZMTP framing of CURVE MESSAGE commands on the device
// (SURVEY.md section 8f row 2).
//
// Send side.  After curve_encoding_t::encode the engine's ZMTP encoder
// frames the boxed message (a fresh msg_t: no MORE / COMMAND flag,
// src/curve_mechanism_base.cpp:166-177) as  flags | size | body  with
// flags = LARGE (2) when the body is longer than 255 bytes and the size as
// one byte or a big-endian uint64 (src/v3_1_encoder.cpp:23-60,
// src/v2_encoder.cpp:23-60).  k_zmtp_sizes / k_zmtp_headers lay the frames of
// a batch out back to back in one send buffer (offsets by an exclusive scan
// on the device) and write the headers; the frame kernel writes the bodies.
//
// Receive side.  The ZMTP decoder (src/v2_decoder.cpp:35-140) reads a flags
// byte, a 1- or 8-byte size (LARGE), checks the size against maxmsgsize
// (EMSGSIZE) and takes the body.  Frame boundaries are a sequential chain
// (each size locates the next frame), so the device finds them without
// walking byte by byte, and without the host reading anything back until the
// call's result:
//   1. candidates: every offset p whose header and body lie inside the
//      buffer, whose size passes maxmsgsize, and whose body starts with
//      "\x07MESSAGE" -- a superset of the true MESSAGE frame starts (a
//      peer can plant the signature inside a body) -- less the shadow a
//      LARGE header's size field casts; gathered per 16 KiB workgroup in
//      stream order and concatenated (k_zmtp_scan, k_zmtp_compact);
//   2. links: candidate k is linked when the frame at cand[k] ends exactly
//      at cand[k+1]; each candidate learns the next unlinked one
//      (k_zmtp_links, k_zmtp_segnext; normally only the last is unlinked);
//   3. one thread walks the chain from offset 0 over whole linked runs,
//      jumping only at unlinked candidates (a binary search for the next
//      frame's offset among the candidates), and records the runs;
//   4. one thread per candidate turns the runs into frame descriptors, and
//      the entries up to max_frames into empty frames, so the decode runs
//      over max_frames with the frame count left on the device.
// A clean stream costs two parallel passes and a one-step walk; planted
// signatures add one binary search per frame that carries one.  The frame
// after the chain decides the rest, as the reference decoder would: a
// complete non-MESSAGE frame is returned as the last frame (its decode
// status is the mechanism's error), an oversized one stops the parse with
// EMSGSIZE, an incomplete one is left for the next buffer.
#pragma once

#include <errno.h>
#include <stdint.h>

namespace zmqg {

constexpr uint8_t kZmtpMore = 1, kZmtpLarge = 2, kZmtpCommand = 4; // src/v2_protocol.hpp:14-19

// Header of the frame at p: header bytes (2 or 9) and body size; false when
// the header is not complete inside [0, n).
__device__ __forceinline__ bool zmtp_header(const uint8_t *b, uint64_t n, uint64_t p, uint32_t &hdr, uint64_t &size)
{
    if (p + 2 > n)
        return false;
    const uint8_t f = b[p];
    if (f & kZmtpLarge) {
        if (p + 9 > n)
            return false;
        uint64_t s = 0;
#pragma unroll
        for (int k = 1; k <= 8; ++k)
            s = (s << 8) | b[p + k];
        hdr = 9;
        size = s;
    } else {
        hdr = 2;
        size = b[p + 1];
    }
    return true;
}

// size passes the decoder's checks: maxmsgsize (src/v2_decoder.cpp:74-79)
// and this path's 32-bit frame lengths
__device__ __forceinline__ bool zmtp_size_ok(uint64_t size, int64_t max_msg)
{
    if (max_msg >= 0 && size > (uint64_t) max_msg)
        return false;
    return size <= 0xffffffffull;
}

struct ZmtpIsCandidate {
    const uint8_t *b;
    uint64_t n;
    int64_t max_msg;
    __device__ bool operator()(const uint64_t &p) const
    {
        uint32_t hdr;
        uint64_t size;
        if (!zmtp_header(b, n, p, hdr, size) || !zmtp_size_ok(size, max_msg))
            return false;
        if (size < 8 || size > n - p - hdr)
            return false;
        const uint8_t *q = b + p + hdr;
        return q[0] == 0x07 && q[1] == 'M' && q[2] == 'E' && q[3] == 'S' && q[4] == 'S' && q[5] == 'A' &&
               q[6] == 'G' && q[7] == 'E';
    }
};

// Candidate scan (k_zmtp_scan): one workgroup per 16 KiB of the stream, in
// chunks of 16 bytes, consecutive lanes on consecutive chunks.  Every 0x07 byte q that starts "\x07MESSAGE"
// is a body start; the frame starts it can belong to are q-9 (LARGE header)
// and q-2 (short header).  A LARGE frame's size field ends "<b7> <b8>" right
// before its body, so whenever <b7> has no LARGE bit q-2 also reads as a
// short header (size <b8>) with the same signature: a shadow inside the true
// frame's header.  When q-9 is a candidate, q-2 is therefore dropped.  (A
// true frame never starts inside another true frame's header; a planted LARGE
// candidate at q-9 whose header covers a true start at q-2 only ends the walk
// early: that frame is then taken as the frame after the chain, and the next
// call resumes behind it.)
// Ordering: signatures are at least 8 bytes apart (0x07 does not occur in
// "MESSAGE"), so a candidate's offset orders like its signature's, and a
// workgroup's candidates, written in thread order after a block scan of the
// threads' counts, are sorted; the workgroups' lists, concatenated in
// workgroup order (k_zmtp_compact), are the sorted candidate array -- no sort
// and no count read back by the host.
constexpr uint32_t kZmtpThreads = 256;
constexpr uint32_t kZmtpWgBytes = 64u * kZmtpThreads;    // 16 KiB of stream per workgroup
constexpr uint32_t kZmtpWgCap = kZmtpWgBytes / 8u;         // candidates a workgroup can hold
constexpr unsigned long long kZmtpNone = ~0ull;

// byte o (static) of a little-endian register window
template <int O, int NW>
__device__ __forceinline__ uint32_t zmtp_byte(const uint32_t (&w)[NW])
{
    static_assert(O >= 0 && O / 4 < NW, "byte inside the window");
    return (w[O / 4] >> (8 * (O % 4))) & 0xffu;
}

// The candidate for a "\x07MESSAGE" at stream offset qq, whose byte is at
// offset O of the register window w (which holds the 16 bytes before the
// chunk too): the frame start it belongs to -- qq-9 (LARGE header) or qq-2
// (short) -- when that header passes ZmtpIsCandidate's tests, else none.
// Header bytes come from the registers: no memory access.
template <int O, int NW>
__device__ __forceinline__ uint64_t zmtp_cand_at(const uint32_t (&w)[NW], uint64_t qq, uint64_t n, int64_t max_msg)
{
    if (qq >= 9 && (zmtp_byte<O - 9>(w) & kZmtpLarge)) {
        uint64_t size = 0;
        size = (size << 8) | zmtp_byte<O - 8>(w);
        size = (size << 8) | zmtp_byte<O - 7>(w);
        size = (size << 8) | zmtp_byte<O - 6>(w);
        size = (size << 8) | zmtp_byte<O - 5>(w);
        size = (size << 8) | zmtp_byte<O - 4>(w);
        size = (size << 8) | zmtp_byte<O - 3>(w);
        size = (size << 8) | zmtp_byte<O - 2>(w);
        size = (size << 8) | zmtp_byte<O - 1>(w);
        const uint64_t p = qq - 9;
        if (zmtp_size_ok(size, max_msg) && size >= 8 && size <= n - p - 9)
            return p;
    }
    if (qq >= 2 && !(zmtp_byte<O - 2>(w) & kZmtpLarge)) {
        const uint64_t size = zmtp_byte<O - 1>(w), p = qq - 2;
        if (zmtp_size_ok(size, max_msg) && size >= 8 && size <= n - p - 2)
            return p;
    }
    return kZmtpNone;
}

// four 16-bit counts, one per chunk round k: exclusive sum over the
// workgroup's threads of each, the workgroup totals to every thread
__device__ __forceinline__ uint64_t zmtp_block_excl4(uint64_t v, uint64_t &total)
{
    __shared__ unsigned long long sh4[kZmtpThreads / 64];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    uint64_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t o = __shfl_up(x, d);
        if ((int) lane >= d)
            x += o;
    }
    if (lane == 63)
        sh4[wv] = x;
    __syncthreads();
    uint64_t base = 0;
    total = 0;
#pragma unroll
    for (uint32_t k = 0; k < kZmtpThreads / 64; ++k) {
        if (k < wv)
            base += sh4[k];
        total += sh4[k];
    }
    return base + x - v;
}

// NB stream bytes at off (NB = 8 or 16) as words, zero outside [0, n)
template <int NB>
__device__ __forceinline__ void zmtp_load_words(const uint8_t *b, uint64_t n, int64_t off, uint32_t (&x)[NB / 4])
{
    if (off >= 0 && (uint64_t) off + NB <= n) {
        if constexpr (NB == 16) {
            const uint4 v = *(const uint4 *) (b + off);
            x[0] = v.x;
            x[1] = v.y;
            x[2] = v.z;
            x[3] = v.w;
        } else {
            const uint2 v = *(const uint2 *) (b + off);
            x[0] = v.x;
            x[1] = v.y;
        }
        return;
    }
#pragma unroll
    for (int q = 0; q < NB / 4; ++q) {
        uint32_t v = 0;
        for (int j = 0; j < 4; ++j) {
            const int64_t p = off + 4 * q + j;
            v |= (uint32_t) (p >= 0 && (uint64_t) p < n ? b[p] : 0u) << (8 * j);
        }
        x[q] = v;
    }
}

// SHFL (round 4): each lane loads only its own 16-byte chunk; the 16 bytes
// before it and the 8 after come from the neighbouring lanes by shuffles,
// lanes 0 and 63 load theirs (one coalesced load per chunk instead of three
// overlapping ones).
template <bool SHFL>
__global__ __launch_bounds__(kZmtpThreads) void k_zmtp_scan(const uint8_t *b, uint64_t n, int64_t max_msg,
                                                            uint64_t *cand_wg, uint64_t *count_wg)
{
    // Chunk (k, thread) = stream bytes [wg0 + 16 (256 k + thread), +16), k =
    // 0..3: consecutive lanes read consecutive chunks (coalesced), each with
    // the 16 bytes before it (a header) and the 8 after (a signature's tail),
    // so the signature and header tests run on registers.  All four rounds'
    // loads go out first; candidates go out in (k, thread) order, which is
    // stream order, after one block scan of the four rounds' counts packed in
    // 16-bit fields (a workgroup holds at most kZmtpWgCap = 2048 of them).
    constexpr uint32_t R = kZmtpWgBytes / 16u / kZmtpThreads; // 4 rounds
    static_assert(R == 4, "four 16-bit count fields");
    const uint64_t wg0 = (uint64_t) blockIdx.x * kZmtpWgBytes;
    uint64_t *const dst0 = cand_wg + (size_t) blockIdx.x * kZmtpWgCap;
    uint32_t w[R][10]; // round k: stream bytes [base_k - 16, base_k + 24), zero outside [0, n)
    if (SHFL) {
        const uint32_t lane = threadIdx.x & 63u;
        uint32_t c[R][4];
#pragma unroll
        for (uint32_t k = 0; k < R; ++k)
            zmtp_load_words<16>(b, n, (int64_t) (wg0 + 16ull * (k * kZmtpThreads + threadIdx.x)), c[k]);
#pragma unroll
        for (uint32_t k = 0; k < R; ++k) {
            const int64_t base = (int64_t) (wg0 + 16ull * (k * kZmtpThreads + threadIdx.x));
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                w[k][q] = (uint32_t) __shfl_up((int) c[k][q], 1);
                w[k][4 + q] = c[k][q];
            }
            w[k][8] = (uint32_t) __shfl_down((int) c[k][0], 1);
            w[k][9] = (uint32_t) __shfl_down((int) c[k][1], 1);
            if (lane == 0) {
                uint32_t p[4];
                zmtp_load_words<16>(b, n, base - 16, p);
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    w[k][q] = p[q];
            }
            if (lane == 63) {
                uint32_t p[2];
                zmtp_load_words<8>(b, n, base + 16, p);
                w[k][8] = p[0];
                w[k][9] = p[1];
            }
        }
    } else {
#pragma unroll
    for (uint32_t k = 0; k < R; ++k) {
        const uint64_t base = wg0 + 16ull * (k * kZmtpThreads + threadIdx.x);
        if (base >= 16 && base + 24 <= n) {
            const uint4 v0 = *(const uint4 *) (b + base - 16);
            const uint4 v1 = *(const uint4 *) (b + base);
            const uint2 v2 = *(const uint2 *) (b + base + 16);
            w[k][0] = v0.x;
            w[k][1] = v0.y;
            w[k][2] = v0.z;
            w[k][3] = v0.w;
            w[k][4] = v1.x;
            w[k][5] = v1.y;
            w[k][6] = v1.z;
            w[k][7] = v1.w;
            w[k][8] = v2.x;
            w[k][9] = v2.y;
        } else {
#pragma unroll
            for (int q = 0; q < 10; ++q) {
                uint32_t x = 0;
                for (int j = 0; j < 4; ++j) {
                    const int64_t p = (int64_t) base - 16 + 4 * q + j;
                    x |= (uint32_t) (p >= 0 && (uint64_t) p < n ? b[p] : 0u) << (8 * j);
                }
                w[k][q] = x;
            }
        }
    }
    }
    uint64_t f[R][2]; // (at most 2 per chunk: signatures are >= 8 bytes apart)
    uint32_t cnt[R];
#pragma unroll
    for (uint32_t k = 0; k < R; ++k) {
        const uint64_t base = wg0 + 16ull * (k * kZmtpThreads + threadIdx.x);
        uint64_t f0 = 0, f1 = 0;
        uint32_t c = 0;
        auto at = [&](uint64_t p) { // (registers only: no dynamically indexed array)
            if (p != kZmtpNone && c < 2u) {
                f1 = c ? p : f1;
                f0 = c ? f0 : p;
                ++c;
            }
        };
        const uint32_t(&wk)[10] = w[k];
#define ZMTP_SIG(Q, J)                                                                                           \
    if (__builtin_amdgcn_alignbyte(wk[5 + Q], wk[4 + Q], J) == 0x53454d07u &&                                    \
        __builtin_amdgcn_alignbyte(wk[6 + Q], wk[5 + Q], J) == 0x45474153u && base + 4 * Q + J + 8 <= n)         \
        at(zmtp_cand_at<16 + 4 * Q + J>(wk, base + 4 * Q + J, n, max_msg));
#define ZMTP_WORD(Q)                                                                                             \
    {                                                                                                            \
        const uint32_t x = wk[4 + Q] ^ 0x07070707u;                                                              \
        if ((x - 0x01010101u) & ~x & 0x80808080u) { /* a 0x07 byte in this word */                              \
            ZMTP_SIG(Q, 0)                                                                                       \
            ZMTP_SIG(Q, 1)                                                                                       \
            ZMTP_SIG(Q, 2)                                                                                       \
            ZMTP_SIG(Q, 3)                                                                                       \
        }                                                                                                        \
    }
        ZMTP_WORD(0)
        ZMTP_WORD(1)
        ZMTP_WORD(2)
        ZMTP_WORD(3)
#undef ZMTP_WORD
#undef ZMTP_SIG
        f[k][0] = f0;
        f[k][1] = f1;
        cnt[k] = c;
    }
    uint64_t packed = 0;
#pragma unroll
    for (uint32_t k = 0; k < R; ++k)
        packed |= (uint64_t) cnt[k] << (16 * k);
    uint64_t tot;
    const uint64_t ex = zmtp_block_excl4(packed, tot);
    uint32_t base_out = 0;
#pragma unroll
    for (uint32_t k = 0; k < R; ++k) {
        const uint32_t off = base_out + (uint32_t) ((ex >> (16 * k)) & 0xffffu);
        if (cnt[k] > 0u)
            dst0[off] = f[k][0];
        if (cnt[k] > 1u)
            dst0[off + 1] = f[k][1];
        base_out += (uint32_t) ((tot >> (16 * k)) & 0xffffu);
    }
    if (threadIdx.x == 0)
        count_wg[blockIdx.x] = base_out;
}

// Workgroup lists -> the sorted candidate array (off_wg: exclusive sum of the
// counts, off_wg[nwg] = m).
__global__ __launch_bounds__(kZmtpThreads) void k_zmtp_compact(const uint64_t *cand_wg, const uint64_t *count_wg,
                                                               const uint64_t *off_wg, uint64_t *cand)
{
    const uint32_t w = blockIdx.x, c = (uint32_t) count_wg[w];
    const uint64_t o = off_wg[w];
    for (uint32_t k = threadIdx.x; k < c; k += kZmtpThreads)
        cand[o + k] = cand_wg[(size_t) w * kZmtpWgCap + k];
}

// Links: candidate k is unlinked when its frame does not end at candidate
// k+1 (the last one never does).  Over segments of 256 candidates (a
// persistent grid; m is read on the device): nb[k] = the first unlinked index
// >= k inside k's segment (or none), first_seg[s] = nb of segment s's first
// candidate.
constexpr uint32_t kZmtpSeg = 256;
__device__ __forceinline__ void zmtp_links_seg(const uint8_t *b, uint64_t n, const uint64_t *cand, uint64_t m,
                                               uint64_t sg, uint64_t *nb, uint64_t *first_seg);
__global__ __launch_bounds__(kZmtpSeg) void k_zmtp_links(const uint8_t *b, uint64_t n, const uint64_t *cand,
                                                         const uint64_t *m_p, uint64_t *nb, uint64_t *first_seg)
{
    const uint64_t m = *m_p, nseg = (m + kZmtpSeg - 1) / kZmtpSeg;
    for (uint64_t sg = blockIdx.x; sg < nseg; sg += gridDim.x)
        zmtp_links_seg(b, n, cand, m, sg, nb, first_seg);
}

// Links of segment sg (256 threads, one candidate each): see k_zmtp_links.
__device__ __forceinline__ void zmtp_links_seg(const uint8_t *b, uint64_t n, const uint64_t *cand, uint64_t m,
                                               uint64_t sg, uint64_t *nb, uint64_t *first_seg)
{
    __shared__ unsigned long long sh[kZmtpSeg / 64];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint64_t k = sg * kZmtpSeg + threadIdx.x;
    unsigned long long u = kZmtpNone;
    if (k < m) {
        bool unl = k + 1 >= m;
        if (!unl) {
            uint32_t hdr;
            uint64_t size;
            zmtp_header(b, n, cand[k], hdr, size);
            unl = cand[k + 1] != cand[k] + hdr + size;
        }
        u = unl ? k : kZmtpNone;
    }
    // suffix minimum: within the wave, then over the later waves
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const unsigned long long o = __shfl_down(u, d);
        if (lane + d < 64u && o < u)
            u = o;
    }
    if (lane == 0)
        sh[wv] = u;
    __syncthreads();
    for (uint32_t q = wv + 1; q < kZmtpSeg / 64; ++q)
        if (sh[q] < u)
            u = sh[q];
    if (k < m)
        nb[k] = u;
    if (threadIdx.x == 0)
        first_seg[sg] = u;
    __syncthreads();
}

// first_seg -> its suffix minimum over segments, in place (one workgroup of
// T threads, each a contiguous run of segments): the first unlinked
// candidate in segments >= s.
constexpr uint32_t kZmtpNextThreads = 1024;
template <uint32_t T>
__device__ void zmtp_segnext(uint64_t *first_seg, uint64_t m)
{
    __shared__ unsigned long long sh[T];
    const uint64_t nseg = (m + kZmtpSeg - 1) / kZmtpSeg;
    const uint64_t per = (nseg + T - 1) / T;
    const uint64_t r0 = threadIdx.x * per, r1 = r0 + per < nseg ? r0 + per : nseg;
    unsigned long long mn = kZmtpNone;
    for (uint64_t s = r0; s < r1; ++s)
        mn = first_seg[s] < mn ? first_seg[s] : mn;
    sh[threadIdx.x] = mn;
    __syncthreads();
    for (uint32_t d = 1; d < T; d <<= 1) {
        const unsigned long long o = threadIdx.x + d < T ? sh[threadIdx.x + d] : kZmtpNone;
        __syncthreads();
        if (o < sh[threadIdx.x])
            sh[threadIdx.x] = o;
        __syncthreads();
    }
    unsigned long long c = threadIdx.x + 1 < T ? sh[threadIdx.x + 1] : kZmtpNone;
    for (uint64_t s = r1; s-- > r0;) {
        const unsigned long long x = first_seg[s];
        c = x < c ? x : c;
        first_seg[s] = c;
    }
}

// Exclusive sum of v[0..n) into o[0..n] (o[n] = total) by one workgroup of
// 1024 threads, each a contiguous run: the small scans of this path (the
// workgroups' candidate counts; the frames' payload sizes) in one launch.
constexpr uint32_t kZmtpScan1 = 1024;
__global__ __launch_bounds__(kZmtpScan1) void k_zmtp_exsum(const uint64_t *v, uint64_t n, uint64_t *o)
{
    __shared__ unsigned long long sh[kZmtpScan1];
    const uint64_t per = (n + kZmtpScan1 - 1) / kZmtpScan1;
    const uint64_t r0 = threadIdx.x * per, r1 = r0 + per < n ? r0 + per : n;
    unsigned long long t = 0;
    for (uint64_t i = r0; i < r1; ++i)
        t += v[i];
    sh[threadIdx.x] = t;
    __syncthreads();
    for (uint32_t d = 1; d < kZmtpScan1; d <<= 1) {
        const unsigned long long x = threadIdx.x >= d ? sh[threadIdx.x - d] : 0ull;
        __syncthreads();
        sh[threadIdx.x] += x;
        __syncthreads();
    }
    unsigned long long acc = sh[threadIdx.x] - t;
    for (uint64_t i = r0; i < r1; ++i) {
        const unsigned long long x = v[i];
        o[i] = acc;
        acc += x;
    }
    if (threadIdx.x == kZmtpScan1 - 1)
        o[n] = sh[kZmtpScan1 - 1];
}

// Parse state written by k_zmtp_walk (device).
struct ZmtpWalk {
    unsigned long long frames;   // frames returned (chain + an extra last one)
    unsigned long long consumed; // bytes of the buffer those frames cover
    unsigned long long runs;     // linked runs on the chain
    int32_t error;               // 0 or EMSGSIZE
    uint32_t extra;              // 1: the last frame is a complete non-MESSAGE frame at `extra_off`
    unsigned long long extra_off;
    unsigned long long out_bytes; // payload bytes of the returned frames (k_zmtp_frames adds them up)
};

// Thread 0 walks the chain (see the file comment).  run[2r], run[2r+1]: the
// first and last candidate of run r; runpre[r]: frames before run r.  The
// next unlinked candidate >= cur is nb[cur], or (none left in cur's
// segment) first_seg[cur / kZmtpSeg + 1].
__device__ void zmtp_walk(const uint8_t *b, uint64_t n, int64_t max_msg, uint64_t max_frames, const uint64_t *cand,
                          const uint64_t *m_p, const uint64_t *nb, const uint64_t *first_seg, uint64_t *run,
                          uint64_t *runpre, ZmtpWalk *out)
{
    const uint64_t m = *m_p, nseg = (m + kZmtpSeg - 1) / kZmtpSeg;
    uint64_t frames = 0, runs = 0, q = 0;
    bool full = false;
    if (m > 0 && cand[0] == 0 && max_frames > 0) {
        uint64_t cur = 0;
        for (;;) {
            uint64_t last = nb[cur];
            if (last == kZmtpNone) {
                const uint64_t sg = cur / kZmtpSeg + 1u;
                last = sg < nseg ? first_seg[sg] : kZmtpNone;
            }
            if (last == kZmtpNone)
                last = m - 1; // (the last candidate is always unlinked)
            if (frames + (last - cur + 1) >= max_frames) {
                last = cur + (max_frames - frames) - 1;
                full = true;
            }
            run[2 * runs] = cur;
            run[2 * runs + 1] = last;
            runpre[runs] = frames;
            ++runs;
            frames += last - cur + 1;
            uint32_t hdr;
            uint64_t size;
            zmtp_header(b, n, cand[last], hdr, size);
            q = cand[last] + hdr + size;
            if (full)
                break;
            // the next frame starts at q: a candidate further on, or the end
            uint64_t lo = last + 1, hi = m;
            while (lo < hi) {
                const uint64_t mid = (lo + hi) >> 1;
                if (cand[mid] < q)
                    lo = mid + 1;
                else
                    hi = mid;
            }
            if (lo < m && cand[lo] == q) {
                cur = lo;
                continue;
            }
            break;
        }
    }
    ZmtpWalk w{};
    w.frames = frames;
    w.runs = runs;
    w.consumed = q;
    if (!full && q < n) {
        uint32_t hdr;
        uint64_t size;
        if (zmtp_header(b, n, q, hdr, size)) {
            if (!zmtp_size_ok(size, max_msg)) {
                w.error = EMSGSIZE; // src/v2_decoder.cpp:74-84: the decoder fails here
            } else if (size <= n - q - hdr) {
                // complete, and not a MESSAGE: returned for the mechanism to reject
                w.extra = 1;
                w.extra_off = q;
                w.frames = frames + 1;
                w.consumed = q + hdr + size;
            }
        }
    }
    *out = w;
}

// first_seg's suffix minimum (k_zmtp_segnext), then thread 0 walks.
__global__ __launch_bounds__(kZmtpNextThreads) void k_zmtp_next_walk(const uint8_t *b, uint64_t n, int64_t max_msg,
                                                                     uint64_t max_frames, const uint64_t *cand,
                                                                     const uint64_t *m_p, const uint64_t *nb,
                                                                     uint64_t *first_seg, uint64_t *run,
                                                                     uint64_t *runpre, ZmtpWalk *out)
{
    zmtp_segnext<kZmtpNextThreads>(first_seg, *m_p);
    __threadfence_block();
    __syncthreads();
    if (threadIdx.x == 0)
        zmtp_walk(b, n, max_msg, max_frames, cand, m_p, nb, first_seg, run, runpre, out);
}

// Frame descriptors from the runs: one workgroup per candidate segment
// (k_zmtp_links's layout).  Entries [frames, max_frames) get an empty frame
// (offset 0, length 0: the decode reports it malformed and writes nothing
// else), so the decode can run over max_frames without the frame count
// reaching the host.
__device__ __forceinline__ void zmtp_frames_body(const uint8_t *b, uint64_t n, const uint64_t *cand, uint64_t m,
                                                 const uint64_t *run, const uint64_t *runpre, const ZmtpWalk *walk,
                                                 uint64_t max_frames, uint64_t *f_off, uint32_t *f_len,
                                                 uint8_t *f_flags, uint32_t *sid_fill, uint32_t sid,
                                                 uint64_t *out_off, unsigned long long *out_bytes, bool pad)
{
    const uint64_t runs = walk->runs, frames = walk->frames;
    __shared__ unsigned long long sh_pb[kZmtpThreads / 64];
    unsigned long long pb = 0; // this thread's payload bytes
    const uint64_t stride = (uint64_t) gridDim.x * kZmtpThreads;
    // padding and the per-frame session over max_frames
    for (uint64_t j = (uint64_t) blockIdx.x * kZmtpThreads + threadIdx.x; pad && j < max_frames; j += stride) {
        sid_fill[j] = sid;
        if (j >= frames) {
            f_off[j] = 0;
            f_len[j] = 0;
            f_flags[j] = 0;
            out_off[j] = 0;
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0 && walk->extra) {
        uint32_t hdr;
        uint64_t size;
        const uint64_t q = walk->extra_off;
        zmtp_header(b, n, q, hdr, size);
        const uint64_t j = frames - 1;
        f_off[j] = q + hdr;
        f_len[j] = (uint32_t) size;
        f_flags[j] = b[q];
        out_off[j] = q + hdr;
        pb += size >= 33u ? size - 33u : 0u;
    }
    for (uint64_t k = (uint64_t) blockIdx.x * kZmtpThreads + threadIdx.x; runs > 0 && k < m; k += stride) {
        // the run holding k: last run whose first candidate <= k
        uint64_t lo = 0, hi = runs;
        while (hi - lo > 1) {
            const uint64_t mid = (lo + hi) >> 1;
            if (run[2 * mid] <= k)
                lo = mid;
            else
                hi = mid;
        }
        if (k < run[2 * lo] || k > run[2 * lo + 1])
            continue; // not on the chain
        const uint64_t j = runpre[lo] + (k - run[2 * lo]);
        uint32_t hdr;
        uint64_t size;
        zmtp_header(b, n, cand[k], hdr, size);
        f_off[j] = cand[k] + hdr;
        f_len[j] = (uint32_t) size;
        f_flags[j] = b[cand[k]];
        out_off[j] = cand[k] + hdr; // the payload at its body's offset (see zmqg_decode_zmtp)
        pb += size >= 33u ? size - 33u : 0u;
    }
    // the call's payload bytes: one atomic per workgroup (walk->out_bytes
    // starts at 0, written by the walk)
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1)
        pb += __shfl_xor(pb, d);
    if ((threadIdx.x & 63u) == 0)
        sh_pb[threadIdx.x >> 6] = pb;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long tot = 0;
        for (uint32_t q = 0; q < kZmtpThreads / 64; ++q)
            tot += sh_pb[q];
        if (tot)
            atomicAdd(out_bytes, tot);
    }
}

__global__ __launch_bounds__(kZmtpThreads) void k_zmtp_frames(const uint8_t *b, uint64_t n, const uint64_t *cand,
                                                              const uint64_t *m_p, const uint64_t *run,
                                                              const uint64_t *runpre, const ZmtpWalk *walk,
                                                              uint64_t max_frames, uint64_t *f_off, uint32_t *f_len,
                                                              uint8_t *f_flags, uint32_t *sid_fill, uint32_t sid,
                                                              uint64_t *out_off, unsigned long long *out_bytes)
{
    zmtp_frames_body(b, n, cand, *m_p, run, runpre, walk, max_frames, f_off, f_len, f_flags, sid_fill, sid, out_off,
                     out_bytes, true);
}

// ---- the middle of the receive side in one launch (round 4)
// k_zmtp_chain runs what k_zmtp_exsum, k_zmtp_compact, k_zmtp_links,
// k_zmtp_next_walk and k_zmtp_frames do, separated by grid barriers, in one
// launch of one workgroup per CU (far below what the device holds at once, so
// every workgroup becomes resident while the others wait):
//   P0a  empty descriptors over max_frames (so a decode after an abandoned
//        launch reads only empty frames), each workgroup's share of the
//        per-16-KiB candidate counts summed;
//   --   barrier
//   P0b  each workgroup's base = the sum of the shares before it, its counts
//        scanned in LDS, its candidates copied into the sorted array;
//   --   barrier
//   P1   links per 256-candidate segment;
//   --   barrier; the last workgroup to arrive takes the suffix minimum over
//        segments and walks the chain before it releases the others
//   P2   frame descriptors from the runs;
//   the last workgroup to finish writes the call's result (frames,
//   consumed, payload bytes, error).
// A barrier gives up after ~200 ms (s_memrealtime ticks at 100 MHz): that
// workgroup leaves, and the result keeps the ETIMEDOUT its first phase put
// there.  The MORE / COMMAND bits of each frame are ORed into flags_out by
// the decode itself (FrameCtl::zflags), so no flags launch follows.
// Arrivals go through kZmtpBarGroups counters (workgroup b at b mod
// kZmtpBarGroups), whose last arrivals meet at the top counter: same-address
// device-scope atomics serialise (~20 ns each), so 256 arrivals at one word
// cost ~6 us a barrier, through 16 + 16 ~1 us.  Each word sits on a cache
// line of its own, so arrivals do not queue behind the polls of gen.
constexpr uint32_t kZmtpBarGroups = 16;
struct ZmtpBar {
    struct alignas(256) Word {
        unsigned int v;
    };
    Word sub[kZmtpBarGroups]; // workgroups of each group arrived at the current barrier
    Word count;               // groups complete at the current barrier
    Word gen;                 // barriers completed
};

struct ZmtpChainArgs {
    const uint8_t *b;
    uint64_t n;
    int64_t max_msg;
    uint64_t max_frames;
    const uint64_t *cand_wg;
    const uint64_t *count_wg;
    uint64_t nwg;
    uint64_t *off_wg; // off_wg[nwg] = the candidate count (m_p of the other kernels)
    unsigned long long *part;
    uint64_t *cand, *nb, *first_seg, *run, *runpre;
    ZmtpWalk *walk;
    uint64_t *f_off;
    uint32_t *f_len;
    uint8_t *f_flags;
    uint32_t *sid_fill;
    uint32_t sid;
    uint64_t *out_off;
    ZmtpBar *bar;
    zmqg_zmtp_result *res;
    unsigned long long *clk; // diagnostics (ZMQG_ZMTP_CLK): 8 s_memrealtime stamps per workgroup, or null
};

constexpr unsigned long long kZmtpBarTicks = 20000000ull; // 200 ms of s_memrealtime

// Thread 0: count this workgroup in (two levels); true for the last one of
// the grid.  The caller resets count when it is done with it.
__device__ __forceinline__ bool zmtp_count_in(ZmtpBar *bar)
{
    const uint32_t G = gridDim.x, grp = blockIdx.x % kZmtpBarGroups;
    const uint32_t ng = G < kZmtpBarGroups ? G : kZmtpBarGroups;
    const uint32_t gsize = (G - grp + kZmtpBarGroups - 1) / kZmtpBarGroups;
    const unsigned int c = __hip_atomic_fetch_add(&bar->sub[grp].v, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (c + 1u != gsize)
        return false;
    __hip_atomic_store(&bar->sub[grp].v, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned int c2 = __hip_atomic_fetch_add(&bar->count.v, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    return c2 + 1u == ng;
}

// Arrive at a barrier: true for the last workgroup to arrive (which must call
// zmtp_release when it is done), after waiting for that release otherwise;
// ok = false when the wait gave up.
__device__ __forceinline__ bool zmtp_arrive(ZmtpBar *bar, bool &ok)
{
    __shared__ uint32_t sh_state; // 0 released, 1 last, 2 gave up
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent"); // the workgroup's writes of the phase
        const unsigned int g = __hip_atomic_load(&bar->gen.v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        uint32_t s = 0;
        if (zmtp_count_in(bar)) {
            s = 1;
        } else {
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
            while (__hip_atomic_load(&bar->gen.v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == g) {
                __builtin_amdgcn_s_sleep(8); // (~512 cycles between polls)
                if (__builtin_amdgcn_s_memrealtime() - t0 > kZmtpBarTicks) {
                    s = 2;
                    break;
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        sh_state = s;
    }
    __syncthreads();
    ok = sh_state != 2;
    return sh_state == 1;
}

__device__ __forceinline__ void zmtp_release(ZmtpBar *bar)
{
    __syncthreads();
    if (threadIdx.x == 0) {
        __hip_atomic_store(&bar->count.v, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(&bar->gen.v, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
}

__device__ __forceinline__ bool zmtp_grid_sync(ZmtpBar *bar)
{
    bool ok;
    if (zmtp_arrive(bar, ok))
        zmtp_release(bar);
    return ok;
}

// sum over the workgroup (every thread gets it)
__device__ __forceinline__ unsigned long long zmtp_block_sum(unsigned long long v)
{
    __shared__ unsigned long long sh[kZmtpThreads / 64];
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1)
        v += __shfl_xor(v, d);
    __syncthreads();
    if ((threadIdx.x & 63u) == 0)
        sh[threadIdx.x >> 6] = v;
    __syncthreads();
    unsigned long long t = 0;
#pragma unroll
    for (uint32_t q = 0; q < kZmtpThreads / 64; ++q)
        t += sh[q];
    return t;
}

__global__ __launch_bounds__(kZmtpThreads) void k_zmtp_chain(ZmtpChainArgs a)
{
    const uint32_t G = gridDim.x, wb = blockIdx.x, tid = threadIdx.x;
    const uint64_t stride = (uint64_t) G * kZmtpThreads;
    auto stamp = [&](int k) {
        if (a.clk && tid == 0)
            a.clk[8ull * wb + k] = __builtin_amdgcn_s_memrealtime();
    };
    stamp(0);
    // P0a
    if (wb == 0 && tid == 0) {
        zmqg_zmtp_result r{};
        r.error = ETIMEDOUT; // replaced by the last workgroup unless a barrier gives up
        *a.res = r;
    }
    for (uint64_t j = (uint64_t) wb * kZmtpThreads + tid; j < a.max_frames; j += stride) {
        a.sid_fill[j] = a.sid;
        a.f_off[j] = 0;
        a.f_len[j] = 0;
        a.f_flags[j] = 0;
        a.out_off[j] = 0;
    }
    const uint64_t per = (a.nwg + G - 1) / G;
    const uint64_t r0 = (uint64_t) wb * per < a.nwg ? (uint64_t) wb * per : a.nwg;
    const uint64_t r1 = r0 + per < a.nwg ? r0 + per : a.nwg;
    unsigned long long s = 0;
    for (uint64_t w = r0 + tid; w < r1; w += kZmtpThreads)
        s += a.count_wg[w];
    s = zmtp_block_sum(s);
    if (tid == 0)
        a.part[wb] = s;
    stamp(1);
    if (!zmtp_grid_sync(a.bar))
        return;
    stamp(2);
    // P0b: base and total from the shares, then the copies
    unsigned long long before = 0, all = 0;
    for (uint32_t q = tid; q < G; q += kZmtpThreads) {
        const unsigned long long v = a.part[q];
        all += v;
        before += q < wb ? v : 0ull;
    }
    before = zmtp_block_sum(before);
    const uint64_t m = zmtp_block_sum(all);
    if (wb == 0 && tid == 0)
        a.off_wg[a.nwg] = m;
    __shared__ unsigned long long sh_off[kZmtpThreads + 1];
    unsigned long long base = before;
    for (uint64_t c0 = r0; c0 < r1; c0 += kZmtpThreads) {
        // this chunk's counts, scanned in LDS
        const uint64_t w = c0 + tid;
        const unsigned long long cnt = w < r1 ? a.count_wg[w] : 0ull;
        unsigned long long x = cnt;
        const uint32_t lane = tid & 63u, wv = tid >> 6;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const unsigned long long o = __shfl_up(x, d);
            if ((int) lane >= d)
                x += o;
        }
        __shared__ unsigned long long sh_w[kZmtpThreads / 64];
        __syncthreads();
        if (lane == 63)
            sh_w[wv] = x;
        __syncthreads();
        unsigned long long wbase = 0, tot = 0;
#pragma unroll
        for (uint32_t q = 0; q < kZmtpThreads / 64; ++q) {
            wbase += q < wv ? sh_w[q] : 0ull;
            tot += sh_w[q];
        }
        sh_off[tid] = wbase + x - cnt; // exclusive, within the chunk
        if (tid == 0)
            sh_off[kZmtpThreads] = tot;
        __syncthreads();
        const uint32_t nw = (uint32_t) (r1 - c0 < kZmtpThreads ? r1 - c0 : kZmtpThreads);
        // copy item q of the chunk: the count slot holding it by binary search
        for (unsigned long long q = tid; q < tot; q += kZmtpThreads) {
            uint32_t lo = 0, hi = nw;
            while (hi - lo > 1) {
                const uint32_t mid = (lo + hi) >> 1;
                if (sh_off[mid] <= q)
                    lo = mid;
                else
                    hi = mid;
            }
            a.cand[base + q] = a.cand_wg[(size_t) (c0 + lo) * kZmtpWgCap + (q - sh_off[lo])];
        }
        base += tot;
        __syncthreads();
    }
    stamp(3);
    if (!zmtp_grid_sync(a.bar))
        return;
    stamp(4);
    // P1: links
    const uint64_t nseg = (m + kZmtpSeg - 1) / kZmtpSeg;
    for (uint64_t sg = wb; sg < nseg; sg += G)
        zmtp_links_seg(a.b, a.n, a.cand, m, sg, a.nb, a.first_seg);
    stamp(5);
    bool ok;
    if (zmtp_arrive(a.bar, ok)) {
        // the last to arrive: suffix minimum over segments, then the walk
        zmtp_segnext<kZmtpThreads>(a.first_seg, m);
        __threadfence_block();
        __syncthreads();
        if (tid == 0)
            zmtp_walk(a.b, a.n, a.max_msg, a.max_frames, a.cand, a.off_wg + a.nwg, a.nb, a.first_seg, a.run,
                      a.runpre, a.walk);
        zmtp_release(a.bar);
    } else if (!ok) {
        return;
    }
    stamp(6);
    // P2: descriptors of the chain's frames (the padding was P0a's)
    zmtp_frames_body(a.b, a.n, a.cand, m, a.run, a.runpre, a.walk, a.max_frames, a.f_off, a.f_len, a.f_flags,
                     a.sid_fill, a.sid, a.out_off, (unsigned long long *) &a.walk->out_bytes, false);
    stamp(7);
    // the last workgroup writes the result
    __shared__ uint32_t sh_last;
    __syncthreads();
    if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        sh_last = zmtp_count_in(a.bar);
        if (sh_last) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            __hip_atomic_store(&a.bar->count.v, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const ZmtpWalk w = *a.walk;
            zmqg_zmtp_result r{};
            r.frames = w.frames;
            r.consumed = w.consumed;
            r.error = w.error;
            r.out_bytes = __hip_atomic_load((unsigned long long *) &a.walk->out_bytes, __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT);
            *a.res = r;
        }
    }
}

// msg_t flags of a decoded frame: the ZMTP frame's MORE / COMMAND bits
// (src/v2_decoder.cpp:35-41) ORed with the plaintext's (set_flags ORs,
// src/msg.cpp:433-436); 0 for a frame that failed.
// (and, thread 0, the call's result: frames, bytes consumed, payload
// bytes, error -- one read back, or none for the asynchronous form)
__global__ void k_zmtp_flags(const ZmtpWalk *walk, uint64_t max_frames, const uint8_t *f_flags, const int32_t *status,
                             uint8_t *flags_out, zmqg_zmtp_result *res)
{
    const uint64_t j = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (j == 0) {
        zmqg_zmtp_result r{};
        r.frames = walk->frames;
        r.consumed = walk->consumed;
        r.error = walk->error;
        r.out_bytes = walk->out_bytes;
        *res = r;
    }
    if (j >= max_frames || j >= walk->frames || status[j] != 0)
        return;
    const uint8_t z = f_flags[j];
    flags_out[j] |= (uint8_t) (((z & kZmtpMore) ? 1u : 0u) | ((z & kZmtpCommand) ? 2u : 0u));
}

// Send side: bytes of each frame (header + encoded body); F[n] = 0 so the
// exclusive scan's last entry is the total.
__global__ void k_zmtp_sizes(uint64_t n, const uint32_t *sid, const uint8_t *flags, const uint32_t *len,
                             const DevSession *sessions, uint32_t max_sessions, uint64_t *F)
{
    const uint64_t i = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (i > n)
        return;
    if (i == n) {
        F[n] = 0;
        return;
    }
    const uint32_t s = sid[i] < max_sessions ? sid[i] : 0u;
    const uint32_t f = flags[i], ct = f & 0x1cu;
    const uint64_t extra = (ct == 12u || ct == 16u) ? (sessions[s].downgrade_sub ? 1u : (ct == 12u ? 10u : 7u)) : 0u;
    const uint64_t W = 32u + 1u + extra + len[i];
    F[i] = (W > 255u ? 9u : 2u) + W;
}

__global__ void k_zmtp_headers(uint64_t n, const uint64_t *frame_off, uint8_t *out, uint64_t *wire_off)
{
    const uint64_t i = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    const uint64_t F = frame_off[i + 1] - frame_off[i];
    uint8_t *h = out + frame_off[i];
    if (F <= 257u) { // body <= 255 bytes: flags 0, one size byte
        h[0] = 0;
        h[1] = (uint8_t) (F - 2u);
        wire_off[i] = frame_off[i] + 2u;
    } else {
        const uint64_t W = F - 9u;
        h[0] = kZmtpLarge;
#pragma unroll
        for (int k = 0; k < 8; ++k)
            h[1 + k] = (uint8_t) (W >> (56 - 8 * k));
        wire_off[i] = frame_off[i] + 9u;
    }
}

} // namespace zmqg
