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

// Chunk (k, thread) = stream bytes [t0 + 16 (256 k + thread), +16) of the tile
// t0 = 16 KiB x tile, k = 0..3: consecutive lanes read consecutive chunks
// (coalesced), each with the 16 bytes before it (a header) and the 8 after (a
// signature's tail), so the signature and header tests run on registers.
constexpr uint32_t kZmtpRounds = kZmtpWgBytes / 16u / kZmtpThreads; // 4
__device__ __forceinline__ void zmtp_scan_load(const uint8_t *b, uint64_t n, uint64_t tile,
                                               uint32_t (&w)[kZmtpRounds][10])
{
    const uint64_t wg0 = tile * kZmtpWgBytes;
#pragma unroll
    for (uint32_t k = 0; k < kZmtpRounds; ++k) {
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

// One tile's candidates from its registers: written in (k, thread) order,
// which is stream order, after one block scan of the four rounds' counts
// packed in 16-bit fields (a tile holds at most kZmtpWgCap = 2048 of them).
__device__ __forceinline__ void zmtp_scan_tile(uint64_t n, int64_t max_msg, uint64_t tile,
                                               const uint32_t (&w)[kZmtpRounds][10], uint64_t *cand_wg,
                                               uint64_t *count_wg, uint16_t *count16)
{
    constexpr uint32_t R = kZmtpRounds;
    static_assert(R == 4, "four 16-bit count fields");
    const uint64_t wg0 = tile * kZmtpWgBytes;
    uint64_t *const dst0 = cand_wg + (size_t) tile * kZmtpWgCap;
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
    if (threadIdx.x == 0) {
        count_wg[tile] = base_out;
        count16[tile] = (uint16_t) base_out; // (<= kZmtpWgCap = 2048)
    }
}

// Candidate scan, one workgroup per tile.
__global__ __launch_bounds__(kZmtpThreads) void k_zmtp_scan(const uint8_t *b, uint64_t n, int64_t max_msg,
                                                            uint64_t *cand_wg, uint64_t *count_wg,
                                                            uint16_t *count16)
{
    uint32_t w[kZmtpRounds][10];
    zmtp_scan_load(b, n, blockIdx.x, w);
    zmtp_scan_tile(n, max_msg, blockIdx.x, w, cand_wg, count_wg, count16);
}

// The same as a persistent grid: each workgroup takes tiles blockIdx.x,
// + gridDim.x, ..., the next tile's loads in flight while it tests the
// current one.
__global__ __launch_bounds__(kZmtpThreads) void k_zmtp_scan_p(const uint8_t *b, uint64_t n, int64_t max_msg,
                                                              uint64_t nwg, uint64_t *cand_wg, uint64_t *count_wg,
                                                              uint16_t *count16)
{
    uint32_t wa[kZmtpRounds][10], wb[kZmtpRounds][10];
    uint64_t t = blockIdx.x;
    if (t >= nwg)
        return;
    zmtp_scan_load(b, n, t, wa);
    for (;;) {
        const uint64_t tn = t + gridDim.x;
        if (tn < nwg)
            zmtp_scan_load(b, n, tn, wb);
        zmtp_scan_tile(n, max_msg, t, wa, cand_wg, count_wg, count16);
        if (tn >= nwg)
            break;
        __syncthreads(); // (the block scan's LDS is reused)
        t = tn;
        const uint64_t tn2 = t + gridDim.x;
        if (tn2 < nwg)
            zmtp_scan_load(b, n, tn2, wa);
        zmtp_scan_tile(n, max_msg, t, wb, cand_wg, count_wg, count16);
        if (tn2 >= nwg)
            break;
        __syncthreads();
        t = tn2;
    }
}

// A candidate's header (it passed the scan's tests: header and body lie inside
// [0, n)): its nine bytes loaded at once, not the flags byte first; returns
// the flags byte.
__device__ __forceinline__ uint32_t zmtp_cand_header(const uint8_t *b, uint64_t n, uint64_t p, uint32_t &hdr,
                                                     uint64_t &size)
{
    if (p + 9 <= n) {
        uint32_t x[9];
#pragma unroll
        for (int k = 0; k < 9; ++k)
            x[k] = b[p + k];
        if (x[0] & kZmtpLarge) {
            uint64_t v = 0;
#pragma unroll
            for (int k = 1; k <= 8; ++k)
                v = (v << 8) | x[k];
            hdr = 9;
            size = v;
        } else {
            hdr = 2;
            size = x[1];
        }
        return x[0];
    }
    zmtp_header(b, n, p, hdr, size);
    return b[p];
}

// Tile lists -> the sorted candidate array, and the links (round 4: in this
// kernel, no launch of their own): candidate k is unlinked when its frame
// does not end at candidate k+1 (the last one never does).  k+1 is the next
// entry of the same list, or the first entry of the next non-empty list
// (found from the counts), so no other list's output of this launch is
// needed.  Per list: nb[k] = the first unlinked index >= k in k's list (or
// none), first_w[w] = the first unlinked index of list w (or none), wid[k] = w;
// per candidate also its frame (cdesc[k] = body offset | body length << 32,
// cflag[k] = the flags byte), so the walk and the descriptors read no header.
// One wave per list, four lists a workgroup (round 6: a workgroup per list
// kept 4,266 workgroups of mostly idle lanes in flight for the config-2
// stream -- ~16 candidates a list -- behind four barriers each; 12.3 us).
// The list's place in the array: with count16, the sum of the counts before
// it, taken here (round 6: the separate one-workgroup sum kernel cost ~5 us
// of launch and dependent latency): the workgroup sums the counts before its
// first list (a few 16-byte loads per thread, L2-resident), each wave adds
// the lists of its workgroup before its own, and the wave of the last list
// writes the candidate count to off_wg[nwg]; without count16 (large streams),
// off_wg holds the exclusive sum already.
// Latency: every load that depends on nothing else (the list's count and
// first 65 entries, the next 64 lists' counts, the counts to sum) goes out
// first; the next list's first entry and the headers are the second and
// last round of dependent loads (round 5 had seven).
constexpr uint32_t kZmtpCompactLists = kZmtpThreads / 64; // lists per workgroup
__global__ __launch_bounds__(kZmtpThreads) void k_zmtp_compact(const uint8_t *b, uint64_t n, const uint64_t *cand_wg,
                                                               const uint64_t *count_wg, const uint16_t *count16,
                                                               uint64_t *off_wg, uint32_t nwg, uint64_t *cand,
                                                               uint64_t *cdesc, uint8_t *cflag, uint64_t *nb,
                                                               uint64_t *first_w, uint32_t *wid)
{
    __shared__ uint32_t sh_o[kZmtpThreads / 64];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
    const uint32_t w0 = blockIdx.x * kZmtpCompactLists, w = w0 + wv;
    const bool live = w < nwg; // (the wave of a list past the end only helps with the sum)
    const uint32_t wl = live ? w : nwg - 1;
    const uint64_t *const list = cand_wg + (size_t) wl * kZmtpWgCap;
    // round 1 of loads
    const uint32_t c = live ? (uint32_t) count_wg[wl] : 0u;
    const uint64_t p0 = list[lane], p1 = list[lane + 1]; // chunk 0 (entries past c unused)
    uint32_t q = w + 1 + lane;
    bool nz = q < nwg && count_wg[q] != 0;
    uint64_t o;
    if (count16) {
        // the lists before w0 (summed by the whole workgroup) and this
        // wave's predecessors in the workgroup, w0 .. w - 1 (by the wave)
        uint32_t pb = lane < wv && w0 + lane < nwg ? count16[w0 + lane] : 0u;
        uint32_t s = 0;
        const uint32_t w8 = w0 & ~7u;
        for (uint32_t i = tid * 8u; i < w8; i += kZmtpThreads * 8u) {
            const uint4 v = *(const uint4 *) (count16 + i);
            s += (v.x & 0xffffu) + (v.x >> 16) + (v.y & 0xffffu) + (v.y >> 16) + (v.z & 0xffffu) + (v.z >> 16) +
                 (v.w & 0xffffu) + (v.w >> 16);
        }
        if (tid < (w0 & 7u))
            s += count16[w8 + tid];
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            s += __shfl_xor(s, d);
            pb += __shfl_xor(pb, d);
        }
        if (lane == 0)
            sh_o[wv] = s;
        __syncthreads();
        o = pb;
#pragma unroll
        for (uint32_t k = 0; k < kZmtpThreads / 64; ++k)
            o += sh_o[k];
        if (live && w + 1 == nwg && lane == 0)
            off_wg[nwg] = o + c;
    } else {
        o = live ? off_wg[wl] : 0;
    }
    if (!live)
        return;
    // the first entry of the next non-empty list (further than the next 64
    // lists only behind a 1 MiB gap)
    uint64_t after = kZmtpNone;
    for (uint32_t ws = w + 1; c > 0 && ws < nwg;) {
        const unsigned long long bal = __ballot(nz);
        if (bal) {
            after = cand_wg[(size_t) (ws + (uint32_t) __builtin_ctzll(bal)) * kZmtpWgCap];
            break;
        }
        ws += 64u;
        q = ws + lane;
        nz = q < nwg && count_wg[q] != 0;
    }
    unsigned long long carry = kZmtpNone; // the minimum over the later chunks
    for (int j = (int) ((c + 63u) / 64u) - 1; j >= 0; --j) {
        const uint32_t k = (uint32_t) j * 64u + lane;
        unsigned long long u = kZmtpNone;
        if (k < c) {
            const uint64_t p = j == 0 ? p0 : list[k];
            const uint64_t next = k + 1 < c ? (j == 0 ? p1 : list[k + 1]) : after;
            uint32_t hdr;
            uint64_t size;
            const uint32_t fl = zmtp_cand_header(b, n, p, hdr, size);
            cand[o + k] = p;
            wid[o + k] = w;
            cdesc[o + k] = (p + hdr) | (size << 32); // (in_bytes < 2^31: both fit)
            cflag[o + k] = (uint8_t) fl;
            u = next != p + hdr + size ? o + k : kZmtpNone;
        }
        // suffix minimum within the chunk, then the later chunks'
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const unsigned long long x = __shfl_down(u, d);
            if (lane + d < 64u && x < u)
                u = x;
        }
        u = carry < u ? carry : u;
        if (k < c)
            nb[o + k] = u;
        carry = __shfl(u, 0); // the chunk's minimum with the later chunks'
    }
    if (lane == 0)
        first_w[w] = carry;
}

// first_w -> its suffix minimum over the lists, in place (one workgroup of T
// threads, each a contiguous run of entries): the first unlinked candidate in
// lists >= w.
constexpr uint32_t kZmtpNextThreads = 1024;
template <uint32_t T>
__device__ void zmtp_suffix_min(uint64_t *first_w, uint64_t count)
{
    // (wave shuffles, one LDS exchange between the waves; up to 8 entries a
    // thread -- 8,192 lists -- read once, all loads at once, into registers)
    constexpr uint32_t R = 8;
    __shared__ unsigned long long sh[T / 64];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint64_t per = (count + T - 1) / T;
    const uint64_t r0 = threadIdx.x * per < count ? threadIdx.x * per : count;
    const uint64_t r1 = r0 + per < count ? r0 + per : count;
    const bool regs = per <= R;
    unsigned long long v[R];
    unsigned long long x = kZmtpNone;
    if (regs) {
#pragma unroll
        for (uint32_t i = 0; i < R; ++i)
            v[i] = r0 + i < r1 ? first_w[r0 + i] : kZmtpNone;
#pragma unroll
        for (uint32_t i = 0; i < R; ++i)
            x = v[i] < x ? v[i] : x;
    } else {
        for (uint64_t s = r0; s < r1; ++s)
            x = first_w[s] < x ? first_w[s] : x;
    }
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
    if (regs) {
#pragma unroll
        for (int i = (int) R - 1; i >= 0; --i)
            if (r0 + i < r1) {
                c = v[i] < c ? v[i] : c;
                first_w[r0 + i] = c;
            }
    } else {
        for (uint64_t s = r1; s-- > r0;) {
            const unsigned long long e = first_w[s];
            c = e < c ? e : c;
            first_w[s] = c;
        }
    }
}

// Streams up to this many 16 KiB lists (128 MiB) take their offsets inside
// k_zmtp_compact; longer ones from a hipCUB scan of the counts.
constexpr uint32_t kZmtpInlineSumLists = 8192;

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
// wid[cur]) first_w[wid[cur] + 1], already a suffix minimum over the lists;
// a frame's end comes from cdesc.  pre: what the walk reads first (m, cand[0],
// nb[0], wid[0], cdesc[m - 1]), loaded before the suffix minimum's barrier;
// the clean stream's walk is then one more load (first_w[1]).
struct ZmtpWalkPre {
    uint64_t m, cand0, nb0, dlast;
    uint32_t wid0;
};
__device__ void zmtp_walk(const uint8_t *b, uint64_t n, int64_t max_msg, uint64_t max_frames, const uint64_t *cand,
                          const uint64_t *cdesc, const ZmtpWalkPre &pre, const uint64_t *nb, const uint64_t *first_w,
                          const uint32_t *wid, uint64_t nwg, uint64_t *run, uint64_t *runpre, ZmtpWalk *out)
{
    const uint64_t m = pre.m;
    uint64_t frames = 0, runs = 0, q = 0;
    bool full = false;
    if (m > 0 && pre.cand0 == 0 && max_frames > 0) {
        uint64_t cur = 0;
        for (;;) {
            uint64_t last = cur ? nb[cur] : pre.nb0;
            if (last == kZmtpNone) {
                const uint64_t wn = (uint64_t) (cur ? wid[cur] : pre.wid0) + 1u;
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
            const uint64_t d = last == m - 1 ? pre.dlast : cdesc[last];
            q = (d & 0xffffffffull) + (d >> 32); // the frame's end
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
                                                                     const uint64_t *cdesc, const uint64_t *m_p,
                                                                     const uint64_t *nb, uint64_t *first_w,
                                                                     const uint32_t *wid, uint64_t nwg, uint64_t *run,
                                                                     uint64_t *runpre, ZmtpWalk *out)
{
    ZmtpWalkPre pre{};
    if (threadIdx.x == 0) {
        // (index 0 is read even when there are no candidates: the arrays
        // always hold at least 1,024 entries, and m = 0 ignores them)
        pre.m = *m_p;
        pre.cand0 = cand[0];
        pre.nb0 = nb[0];
        pre.wid0 = wid[0];
        pre.dlast = pre.m ? cdesc[pre.m - 1] : 0;
    }
    zmtp_suffix_min<kZmtpNextThreads>(first_w, nwg);
    __threadfence_block();
    __syncthreads();
    if (threadIdx.x == 0)
        zmtp_walk(b, n, max_msg, max_frames, cand, cdesc, pre, nb, first_w, wid, nwg, run, runpre, out);
}

// Frame descriptors from the runs (a persistent grid over the candidates).  Entries [frames, max_frames) get an empty frame
// (offset 0, length 0: the decode reports it malformed and writes nothing
// else), so the decode can run over max_frames without the frame count
// reaching the host.
__device__ __forceinline__ void zmtp_frames_body(const uint8_t *b, uint64_t n, const uint64_t *cdesc,
                                                 const uint8_t *cflag, uint64_t m, const uint64_t *run, const uint64_t *runpre, const ZmtpWalk *walk,
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
        const uint64_t d = cdesc[k]; // (loaded before the runs are searched)
        const uint8_t fl = cflag[k];
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
        const uint64_t body = d & 0xffffffffull, size = d >> 32;
        f_off[j] = body;
        f_len[j] = (uint32_t) size;
        f_flags[j] = fl;
        out_off[j] = body; // the payload at its body's offset (see zmqg_decode_zmtp)
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

__global__ __launch_bounds__(kZmtpThreads) void k_zmtp_frames(const uint8_t *b, uint64_t n, const uint64_t *cdesc,
                                                              const uint8_t *cflag, const uint64_t *m_p,
                                                              const uint64_t *run,
                                                              const uint64_t *runpre, const ZmtpWalk *walk,
                                                              uint64_t max_frames, uint64_t *f_off, uint32_t *f_len,
                                                              uint8_t *f_flags, uint32_t *sid_fill, uint32_t sid,
                                                              uint64_t *out_off, unsigned long long *out_bytes)
{
    zmtp_frames_body(b, n, cdesc, cflag, *m_p, run, runpre, walk, max_frames, f_off, f_len, f_flags, sid_fill, sid, out_off,
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
