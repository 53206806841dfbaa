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
//      (k_zmtp_compact, k_zmtp_next_walk; normally only the last is unlinked);
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
// counts, off_wg[nwg] = m), and the links (round 4: in this kernel, no launch
// of their own): candidate k is unlinked when its frame does not end at
// candidate k+1 (the last one never does).  k+1 is the next entry of the same
// list, or the first entry of the next non-empty list (found from the
// counts), so no other workgroup's output of this launch is needed.  Per list: nb[k] =
// the first unlinked index >= k in k's list (or none), first_w[w] = the first
// unlinked index of list w (or none), wid[k] = w.
__global__ __launch_bounds__(kZmtpThreads) void k_zmtp_compact(const uint8_t *b, uint64_t n, const uint64_t *cand_wg,
                                                               const uint64_t *count_wg, const uint64_t *off_wg,
                                                               uint32_t nwg, uint64_t *cand,
                                                               uint64_t *nb, uint64_t *first_w, uint32_t *wid)
{
    __shared__ unsigned long long sh[kZmtpThreads / 64];
    const uint32_t w = blockIdx.x, c = (uint32_t) count_wg[w], tid = threadIdx.x;
    const uint32_t lane = tid & 63u, wv = tid >> 6;
    const uint64_t o = off_wg[w];
    const uint64_t *const list = cand_wg + (size_t) w * kZmtpWgCap;
    // the first entry of the next non-empty list: the workgroup looks at the
    // next 256 lists' counts at once (further only behind a 4 MiB gap)
    __shared__ uint32_t sh_nx[kZmtpThreads / 64];
    uint64_t after = kZmtpNone;
    for (uint32_t w0 = w + 1; c > 0 && w0 < nwg; w0 += kZmtpThreads) {
        const uint32_t q = w0 + tid;
        const unsigned long long nz = __ballot(q < nwg && count_wg[q] != 0);
        __syncthreads();
        if (lane == 0)
            sh_nx[wv] = nz ? w0 + 64u * wv + (uint32_t) __builtin_ctzll(nz) : nwg;
        __syncthreads();
        uint32_t f = nwg;
        for (uint32_t k = 0; k < kZmtpThreads / 64; ++k)
            f = sh_nx[k] < f ? sh_nx[k] : f;
        if (f < nwg) {
            after = cand_wg[(size_t) f * kZmtpWgCap];
            break;
        }
    }
    unsigned long long carry = kZmtpNone; // the minimum over the later chunks
    for (int j = (int) ((c + kZmtpThreads - 1) / kZmtpThreads) - 1; j >= 0; --j) {
        const uint32_t k = (uint32_t) j * kZmtpThreads + tid;
        unsigned long long u = kZmtpNone;
        if (k < c) {
            const uint64_t p = list[k];
            cand[o + k] = p;
            wid[o + k] = w;
            const uint64_t next = k + 1 < c ? list[k + 1] : after;
            uint32_t hdr;
            uint64_t size;
            zmtp_header(b, n, p, hdr, size);
            u = next != p + hdr + size ? o + k : kZmtpNone;
        }
        // suffix minimum within the chunk, then the later chunks'
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const unsigned long long x = __shfl_down(u, d);
            if (lane + d < 64u && x < u)
                u = x;
        }
        __syncthreads();
        if (lane == 0)
            sh[wv] = u;
        __syncthreads();
        for (uint32_t q = wv + 1; q < kZmtpThreads / 64; ++q)
            u = sh[q] < u ? sh[q] : u;
        u = carry < u ? carry : u;
        if (k < c)
            nb[o + k] = u;
        // the chunk's minimum: wave 0's lane 0 value with the later waves' and chunks'
        unsigned long long lo = carry;
        for (uint32_t q = 0; q < kZmtpThreads / 64; ++q)
            lo = sh[q] < lo ? sh[q] : lo;
        carry = lo;
    }
    if (tid == 0)
        first_w[w] = carry;
}

// first_w -> its suffix minimum over the lists, in place (one workgroup of T
// threads, each a contiguous run of entries): the first unlinked candidate in
// lists >= w.
constexpr uint32_t kZmtpNextThreads = 1024;
template <uint32_t T>
__device__ void zmtp_suffix_min(uint64_t *first_w, uint64_t count)
{
    // (wave shuffles, one LDS exchange between the waves)
    __shared__ unsigned long long sh[T / 64];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint64_t per = (count + T - 1) / T;
    const uint64_t r0 = threadIdx.x * per < count ? threadIdx.x * per : count;
    const uint64_t r1 = r0 + per < count ? r0 + per : count;
    unsigned long long x = kZmtpNone;
    for (uint64_t s = r0; s < r1; ++s)
        x = first_w[s] < x ? first_w[s] : x;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const unsigned long long y = __shfl_down(x, d);
        if (lane + d < 64u && y < x)
            x = y;
    }
    if (lane == 0)
        sh[wv] = x;
    __syncthreads();
    unsigned long long later = kZmtpNone; // the later waves' minimum
    for (uint32_t q = wv + 1; q < T / 64; ++q)
        later = sh[q] < later ? sh[q] : later;
    const unsigned long long nx = __shfl_down(x, 1);
    unsigned long long c = lane < 63u ? (nx < later ? nx : later) : later; // minimum over the later threads
    for (uint64_t s = r1; s-- > r0;) {
        const unsigned long long v = first_w[s];
        c = v < c ? v : c;
        first_w[s] = c;
    }
}

// Exclusive sum of v[0..n) into o[0..n] (o[n] = total) by one workgroup of
// 1024 threads, each a contiguous run: the workgroups' candidate counts.
constexpr uint32_t kZmtpScan1 = 1024;
__global__ __launch_bounds__(kZmtpScan1) void k_zmtp_exsum(const uint64_t *v, uint64_t n, uint64_t *o)
{
    // (wave shuffles, one LDS exchange between the waves)
    __shared__ unsigned long long sh[kZmtpScan1 / 64];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint64_t per = (n + kZmtpScan1 - 1) / kZmtpScan1;
    const uint64_t r0 = threadIdx.x * per < n ? threadIdx.x * per : n, r1 = r0 + per < n ? r0 + per : n;
    unsigned long long t = 0;
    for (uint64_t i = r0; i < r1; ++i)
        t += v[i];
    unsigned long long x = t;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const unsigned long long y = __shfl_up(x, d);
        if ((int) lane >= d)
            x += y;
    }
    if (lane == 63)
        sh[wv] = x;
    __syncthreads();
    unsigned long long acc = x - t, tot = 0;
    for (uint32_t q = 0; q < kZmtpScan1 / 64; ++q) {
        acc += q < wv ? sh[q] : 0ull;
        tot += sh[q];
    }
    for (uint64_t i = r0; i < r1; ++i) {
        const unsigned long long y = v[i];
        o[i] = acc;
        acc += y;
    }
    if (threadIdx.x == 0)
        o[n] = tot;
}

// Parse state written by k_zmtp_walk (device).  It begins with the call's
// result (zmqg_zmtp_result's layout), which the decode's frame kernel copies
// to the caller's result (FrameCtl::res_src).
struct ZmtpWalk {
    unsigned long long frames;    // frames returned (chain + an extra last one)
    unsigned long long consumed;  // bytes of the buffer those frames cover
    unsigned long long out_bytes; // payload bytes of the returned frames (k_zmtp_frames adds them up)
    int32_t error;                // 0 or EMSGSIZE
    uint32_t pad;
    unsigned long long runs;      // linked runs on the chain
    uint32_t extra;               // 1: the last frame is a complete non-MESSAGE frame at `extra_off`
    unsigned long long extra_off;
};
static_assert(sizeof(zmqg_zmtp_result) == 32 && offsetof(ZmtpWalk, runs) == 32, "the result prefix");

// Thread 0 walks the chain (see the file comment).  run[2r], run[2r+1]: the
// first and last candidate of run r; runpre[r]: frames before run r.  The
// next unlinked candidate >= cur is nb[cur], or (none left in cur's list
// wid[cur]) first_w[wid[cur] + 1], already a suffix minimum over the lists.
__device__ void zmtp_walk(const uint8_t *b, uint64_t n, int64_t max_msg, uint64_t max_frames, const uint64_t *cand,
                          const uint64_t *m_p, const uint64_t *nb, const uint64_t *first_w, const uint32_t *wid,
                          uint64_t nwg, uint64_t *run, uint64_t *runpre, ZmtpWalk *out)
{
    const uint64_t m = *m_p;
    uint64_t frames = 0, runs = 0, q = 0;
    bool full = false;
    if (m > 0 && cand[0] == 0 && max_frames > 0) {
        uint64_t cur = 0;
        for (;;) {
            uint64_t last = nb[cur];
            if (last == kZmtpNone) {
                const uint64_t wn = (uint64_t) wid[cur] + 1u;
                last = wn < nwg ? first_w[wn] : kZmtpNone;
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

// first_w's suffix minimum over the lists, then thread 0 walks.
__global__ __launch_bounds__(kZmtpNextThreads) void k_zmtp_next_walk(const uint8_t *b, uint64_t n, int64_t max_msg,
                                                                     uint64_t max_frames, const uint64_t *cand,
                                                                     const uint64_t *m_p, const uint64_t *nb,
                                                                     uint64_t *first_w, const uint32_t *wid,
                                                                     uint64_t nwg, uint64_t *run, uint64_t *runpre,
                                                                     ZmtpWalk *out)
{
    zmtp_suffix_min<kZmtpNextThreads>(first_w, nwg);
    __threadfence_block();
    __syncthreads();
    if (threadIdx.x == 0)
        zmtp_walk(b, n, max_msg, max_frames, cand, m_p, nb, first_w, wid, nwg, run, runpre, out);
}

// Frame descriptors from the runs (a persistent grid over the candidates).  Entries [frames, max_frames) get an empty frame
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
