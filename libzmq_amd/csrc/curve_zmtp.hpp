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
// walking byte by byte:
//   1. candidates: every offset p whose header and body lie inside the
//      buffer, whose size passes maxmsgsize, and whose body starts with
//      "\x07MESSAGE" -- a superset of the true MESSAGE frame starts (a
//      peer can plant the signature inside a body), in offset order, less
//      the shadow a LARGE header's size field casts (k_zmtp_scan);
//   2. links: candidate k is linked when the frame at cand[k] ends exactly
//      at cand[k+1]; the unlinked ones are listed (normally just the last);
//   3. one thread walks the chain from offset 0 over whole linked runs,
//      jumping only at unlinked candidates (a binary search for the next
//      frame's offset among the candidates), and records the runs;
//   4. one thread per candidate turns the runs into frame descriptors.
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

// Candidate scan, one thread per 16 aligned bytes: every 0x07 byte q that
// starts "\x07MESSAGE" is a body start; the frame starts it can belong to
// are q-9 (LARGE header) and q-2 (short header).  A LARGE frame's size field
// ends "<b7> <b8>" right before its body, so whenever <b7> has no LARGE bit
// q-2 also reads as a short header (size <b8>) with the same signature: a
// shadow inside the true frame's header.  When q-9 is a candidate, q-2 is
// therefore dropped.  (A true frame never starts inside another true frame's
// header; a planted LARGE candidate at q-9 whose header covers a true start
// at q-2 only ends the walk early: that frame is then taken as the frame
// after the chain, and the next call resumes behind it.)  Candidates are
// appended unordered; the caller sorts them.
constexpr int kZmtpScanIters = 16;  // 16-byte chunks per thread: 64 KB per workgroup
constexpr int kZmtpScanList = 1024; // candidates a workgroup gathers in LDS before one global reservation

__device__ __forceinline__ void zmtp_emit(uint64_t p, uint64_t *list, uint32_t *lcount, uint64_t *cand,
                                          unsigned long long *count)
{
    const uint32_t k = atomicAdd(lcount, 1u);
    if (k < (uint32_t) kZmtpScanList)
        list[k] = p;
    else
        cand[atomicAdd(count, 1ull)] = p; // overflow (a flood of planted signatures): one by one
}

__global__ __launch_bounds__(256) void k_zmtp_scan(const uint8_t *b, uint64_t n, int64_t max_msg, uint64_t *cand,
                                                   unsigned long long *count)
{
    // a contended global counter takes ~88 returning atomics per us, so
    // candidates are gathered per workgroup and reserved with one atomic
    __shared__ uint64_t list[kZmtpScanList];
    __shared__ uint32_t lcount;
    __shared__ unsigned long long gbase;
    if (threadIdx.x == 0)
        lcount = 0;
    __syncthreads();
    const ZmtpIsCandidate isc{b, n, max_msg};
    const uint64_t wg0 = (uint64_t) blockIdx.x * blockDim.x * 16u * kZmtpScanIters;
    for (int it = 0; it < kZmtpScanIters; ++it) {
        const uint64_t base = wg0 + ((uint64_t) it * blockDim.x + threadIdx.x) * 16u;
        if (base >= n)
            break;
        uint32_t w[4];
        if (base + 16 <= n) {
            const uint4 v = *(const uint4 *) (b + base);
            w[0] = v.x;
            w[1] = v.y;
            w[2] = v.z;
            w[3] = v.w;
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                uint32_t x = 0;
                for (int j = 0; j < 4; ++j) {
                    const uint64_t p = base + 4 * k + j;
                    x |= (uint32_t) (p < n ? b[p] : 0u) << (8 * j);
                }
                w[k] = x;
            }
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t x = w[k] ^ 0x07070707u;
            if (!((x - 0x01010101u) & ~x & 0x80808080u))
                continue; // no 0x07 byte in this word
            for (int j = 0; j < 4; ++j) {
                if (((w[k] >> (8 * j)) & 0xffu) != 0x07u)
                    continue;
                const uint64_t q = base + 4 * k + j;
                if (q + 8 > n || b[q + 1] != 'M' || b[q + 2] != 'E' || b[q + 3] != 'S' || b[q + 4] != 'S' ||
                    b[q + 5] != 'A' || b[q + 6] != 'G' || b[q + 7] != 'E')
                    continue;
                if (q >= 9 && (b[q - 9] & kZmtpLarge) && isc(q - 9))
                    zmtp_emit(q - 9, list, &lcount, cand, count);
                else if (q >= 2 && !(b[q - 2] & kZmtpLarge) && isc(q - 2))
                    zmtp_emit(q - 2, list, &lcount, cand, count);
            }
        }
    }
    __syncthreads();
    const uint32_t nl = lcount < (uint32_t) kZmtpScanList ? lcount : (uint32_t) kZmtpScanList;
    if (threadIdx.x == 0)
        gbase = nl ? atomicAdd(count, (unsigned long long) nl) : 0ull;
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < nl; k += blockDim.x)
        cand[gbase + k] = list[k];
}

// candidate k's frame does not end at candidate k+1 (the last one never does)
struct ZmtpIsUnlinked {
    const uint8_t *b;
    uint64_t n;
    const uint64_t *cand;
    const unsigned long long *m; // candidates
    __device__ bool operator()(const uint64_t &k) const
    {
        if (k + 1 >= *m)
            return true;
        uint32_t hdr;
        uint64_t size;
        zmtp_header(b, n, cand[k], hdr, size);
        return cand[k + 1] != cand[k] + hdr + size;
    }
};

// Parse state written by k_zmtp_walk (device; read back by the host).
struct ZmtpWalk {
    unsigned long long frames;   // frames returned (chain + an extra last one)
    unsigned long long consumed; // bytes of the buffer those frames cover
    unsigned long long runs;     // linked runs on the chain
    int32_t error;               // 0 or EMSGSIZE
    uint32_t extra;              // 1: the last frame is a complete non-MESSAGE frame at `extra_off`
    unsigned long long extra_off;
};

// Thread 0 walks the chain (see the file comment).  run[2r], run[2r+1]: the
// first and last candidate of run r; runpre[r]: frames before run r.
__global__ void k_zmtp_walk(const uint8_t *b, uint64_t n, int64_t max_msg, uint64_t max_frames, const uint64_t *cand,
                            const unsigned long long *m_p, const uint64_t *bad, const unsigned long long *nbad_p,
                            uint64_t *run, uint64_t *runpre, ZmtpWalk *out)
{
    if (blockIdx.x != 0 || threadIdx.x != 0)
        return;
    const uint64_t m = *m_p, nbad = *nbad_p;
    uint64_t frames = 0, runs = 0, q = 0, bi = 0;
    bool full = false;
    if (m > 0 && cand[0] == 0 && max_frames > 0) {
        uint64_t cur = 0;
        for (;;) {
            while (bi < nbad && bad[bi] < cur)
                ++bi;
            uint64_t last = bi < nbad ? bad[bi] : m - 1; // the run's last candidate
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

// Frame descriptors from the runs: one thread per candidate.
__global__ void k_zmtp_frames(const uint8_t *b, uint64_t n, const uint64_t *cand, const unsigned long long *m_p,
                              const uint64_t *run, const uint64_t *runpre, const ZmtpWalk *walk, uint64_t *f_off,
                              uint32_t *f_len, uint8_t *f_flags)
{
    const uint64_t k = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t runs = walk->runs;
    if (k == 0 && walk->extra) {
        uint32_t hdr;
        uint64_t size;
        const uint64_t q = walk->extra_off;
        zmtp_header(b, n, q, hdr, size);
        const uint64_t j = walk->frames - 1;
        f_off[j] = q + hdr;
        f_len[j] = (uint32_t) size;
        f_flags[j] = b[q];
    }
    if (k >= *m_p || runs == 0)
        return;
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
        return; // not on the chain
    const uint64_t j = runpre[lo] + (k - run[2 * lo]);
    uint32_t hdr;
    uint64_t size;
    zmtp_header(b, n, cand[k], hdr, size);
    f_off[j] = cand[k] + hdr;
    f_len[j] = (uint32_t) size;
    f_flags[j] = b[cand[k]];
}

// Payload bytes per frame (the decode output), for the offsets scan.
__global__ void k_zmtp_payload_sizes(uint64_t nf, const uint32_t *f_len, uint64_t *psize, uint32_t *sid_fill,
                                     uint32_t sid)
{
    const uint64_t j = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (j > nf)
        return;
    psize[j] = j < nf && f_len[j] >= 33u ? f_len[j] - 33u : 0u;
    if (j < nf)
        sid_fill[j] = sid;
}

// msg_t flags of a decoded frame: the ZMTP frame's MORE / COMMAND bits
// (src/v2_decoder.cpp:35-41) ORed with the plaintext's (set_flags ORs,
// src/msg.cpp:433-436); 0 for a frame that failed.
__global__ void k_zmtp_flags(uint64_t nf, const uint8_t *f_flags, const int32_t *status, uint8_t *flags_out)
{
    const uint64_t j = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nf || status[j] != 0)
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
