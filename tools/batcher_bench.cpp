// Host-to-host rates of the asynchronous path on one MI355X (config 2
// shape: 1 KiB messages), all in payload GiB/s of one direction:
//   copy      pinned hipMemcpyAsync H2D, D2H, and both at once (the PCIe
//             ceiling any staged path has)
//   zerocopy  zmqg_encode_batch / zmqg_decode_batch reading and writing
//             pinned host memory in place: coherent (zmqg_host_alloc) and
//             non-coherent pinned memory
//   batcher   curve_batcher_t end to end over 256 connections: submit copy
//             from pageable memory, launch, fence, delivery copy into
//             pageable memory (what an I/O thread pays)
// Build: see tools/batcher_bench.sh.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <vector>

#include "../libzmq_amd/host/curve_batcher.hpp"

#define HC(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)
#define CK(c)                                                            \
    do {                                                                 \
        if (!(c)) {                                                      \
            fprintf(stderr, "%s:%d check failed: %s\n", __FILE__, __LINE__, #c); \
            exit(1);                                                     \
        }                                                                \
    } while (0)

static double now()
{
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static const char client_prefix[] = "CurveZMQMESSAGEC";
static const char server_prefix[] = "CurveZMQMESSAGES";
static const size_t n = 65536, P = 1024, W = P + 33;
static const double GiB = 1073741824.0;

struct batch_t {
    uint32_t *sid, *len, *wlen;
    uint64_t *nonce, *in_off, *out_off;
    uint8_t *flags, *pay, *wire, *back, *flo;
    int32_t *st;
};

static void fill_batch(batch_t &b, uint64_t nonce0)
{
    for (size_t i = 0; i < n; ++i) {
        b.sid[i] = 0;
        b.len[i] = P;
        b.wlen[i] = W;
        b.nonce[i] = nonce0 + i;
        b.in_off[i] = i * P;
        b.out_off[i] = i * W;
        b.flags[i] = 0;
    }
}

static void alloc_batch(batch_t &b, unsigned flags)
{
    HC(hipHostMalloc((void **) &b.sid, 4 * n, flags));
    HC(hipHostMalloc((void **) &b.len, 4 * n, flags));
    HC(hipHostMalloc((void **) &b.wlen, 4 * n, flags));
    HC(hipHostMalloc((void **) &b.nonce, 8 * n, flags));
    HC(hipHostMalloc((void **) &b.in_off, 8 * n, flags));
    HC(hipHostMalloc((void **) &b.out_off, 8 * n, flags));
    HC(hipHostMalloc((void **) &b.flags, n, flags));
    HC(hipHostMalloc((void **) &b.pay, n * P, flags));
    HC(hipHostMalloc((void **) &b.wire, n * W, flags));
    HC(hipHostMalloc((void **) &b.back, n * P, flags));
    HC(hipHostMalloc((void **) &b.flo, n, flags));
    HC(hipHostMalloc((void **) &b.st, 4 * n, flags));
    for (size_t i = 0; i < n * P; ++i)
        b.pay[i] = (uint8_t) (i * 131 + (i >> 10));
}

static void zerocopy(const char *label, unsigned flags, zmqg_ctx *enc, zmqg_ctx *dec, hipStream_t s)
{
    batch_t b;
    alloc_batch(b, flags);
    static uint64_t nonce = 3;
    const int reps = 6;
    double te = 0, td = 0;
    hipEvent_t e0, e1;
    HC(hipEventCreate(&e0));
    HC(hipEventCreate(&e1));
    for (int r = 0; r <= reps; ++r) {
        fill_batch(b, nonce);
        nonce += n;
        HC(hipEventRecord(e0, s));
        CK(zmqg_encode_batch(enc, n, b.sid, b.nonce, b.flags, b.in_off, b.len, b.pay, b.out_off, b.wire, s) == 0);
        HC(hipEventRecord(e1, s));
        HC(hipEventSynchronize(e1));
        float ms;
        HC(hipEventElapsedTime(&ms, e0, e1));
        if (r)
            te += ms;
        HC(hipEventRecord(e0, s));
        CK(zmqg_decode_batch(dec, n, b.sid, b.out_off, b.wlen, b.wire, b.in_off, b.back, b.flo, b.st, s) == 0);
        HC(hipEventRecord(e1, s));
        HC(hipEventSynchronize(e1));
        HC(hipEventElapsedTime(&ms, e0, e1));
        if (r)
            td += ms;
        for (size_t i = 0; i < n; ++i)
            CK(b.st[i] == 0);
        CK(memcmp(b.back, b.pay, n * P) == 0);
    }
    printf("zerocopy %-12s encode %6.1f  decode %6.1f GiB/s\n", label, reps * n * P / GiB / (te * 1e-3),
           reps * n * P / GiB / (td * 1e-3));
}

struct sink_t : zmqg::curve_sink_t {
    uint8_t *dst;
    size_t stride;
    size_t got = 0;
    bool ok = true;
    void on_encoded(uint64_t tag, const uint8_t *wire, size_t size)
    {
        memcpy(dst + tag * stride, wire, size);
        ++got;
    }
    void on_decoded(uint64_t tag, int status, const uint8_t *payload, size_t size, uint8_t)
    {
        if (status != 0 || size != P)
            ok = false;
        else
            memcpy(dst + tag * stride, payload, size);
        ++got;
    }
};

int main()
{
    HC(hipSetDevice(0));
    hipStream_t s, s2;
    HC(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    HC(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    uint8_t precom[32];
    for (int i = 0; i < 32; ++i)
        precom[i] = (uint8_t) i;

    {   // raw pinned copies
        const size_t bytes = n * W;
        uint8_t *h, *h2, *d, *d2;
        HC(hipHostMalloc((void **) &h, bytes, hipHostMallocDefault));
        HC(hipHostMalloc((void **) &h2, bytes, hipHostMallocDefault));
        HC(hipMalloc((void **) &d, bytes));
        HC(hipMalloc((void **) &d2, bytes));
        memset(h, 1, bytes);
        memset(h2, 2, bytes);
        for (int mode = 0; mode < 3; ++mode) {
            HC(hipDeviceSynchronize());
            const double t0 = now();
            for (int r = 0; r < 8; ++r) {
                if (mode != 1)
                    HC(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s));
                if (mode != 0)
                    HC(hipMemcpyAsync(h2, d2, bytes, hipMemcpyDeviceToHost, s2));
            }
            HC(hipDeviceSynchronize());
            const double dt = now() - t0;
            printf("copy %-7s %6.1f GB/s per direction\n", mode == 0 ? "H2D" : mode == 1 ? "D2H" : "both",
                   8 * bytes / dt / 1e9);
        }
        HC(hipHostFree(h));
        HC(hipHostFree(h2));
        HC(hipFree(d));
        HC(hipFree(d2));
    }

    zmqg_ctx *enc, *dec;
    CK(zmqg_ctx_create(0, 1, &enc) == 0);
    CK(zmqg_ctx_create(0, 1, &dec) == 0);
    CK(zmqg_session_set(enc, 0, precom, (const uint8_t *) client_prefix, (const uint8_t *) server_prefix, 0, 1) == 0);
    CK(zmqg_session_set(dec, 0, precom, (const uint8_t *) server_prefix, (const uint8_t *) client_prefix, 0, 2) == 0);
    zerocopy("coherent", hipHostMallocMapped | hipHostMallocPortable, enc, dec, s);
    zerocopy("noncoherent", hipHostMallocMapped | hipHostMallocPortable | hipHostMallocNonCoherent, enc, dec, s);
    CK(zmqg_ctx_destroy(enc) == 0);
    CK(zmqg_ctx_destroy(dec) == 0);

    // batcher end to end, 256 connections on one ctx (client and server side)
    const int nc = 256;
    zmqg_ctx *ctx;
    CK(zmqg_ctx_create(0, 2 * nc, &ctx) == 0);
    std::vector<zmqg::curve_encoding_gpu_t *> cl, sv;
    for (int c = 0; c < nc; ++c) {
        cl.push_back(new zmqg::curve_encoding_gpu_t(ctx, c, client_prefix, server_prefix, false));
        sv.push_back(new zmqg::curve_encoding_gpu_t(ctx, nc + c, server_prefix, client_prefix, false));
        uint8_t k[32];
        for (int i = 0; i < 32; ++i)
            k[i] = (uint8_t) (c * 7 + i);
        memcpy(cl[c]->get_writable_precom_buffer(), k, 32);
        memcpy(sv[c]->get_writable_precom_buffer(), k, 32);
        sv[c]->set_peer_nonce(0); // the handshake's nonces are not replayed here
    }
    std::vector<uint8_t> src(n * P), wires(n * W), back(n * P);
    for (size_t i = 0; i < n * P; ++i)
        src[i] = (uint8_t) (i * 31 + 7);
    zmqg::curve_batcher_t::config_t cfg;
    cfg.slot_msgs = 8192;
    cfg.slot_bytes = 8192 * W;
    cfg.slots = 4;
    sink_t es, ds;
    es.dst = &wires[0];
    es.stride = W;
    ds.dst = &back[0];
    ds.stride = P;
    zmqg::curve_batcher_t eb(ctx, &es, cfg), db(ctx, &ds, cfg);
    CK(eb.init() == 0 && db.init() == 0);
    const int rounds = 4;
    double te = 0, td = 0;
    for (int r = 0; r <= rounds; ++r) {
        es.got = 0;
        double t0 = now();
        for (size_t i = 0; i < n; ++i) {
            CK(eb.submit_encode(cl[i % nc], &src[i * P], P, 0, i) == 0);
            if ((i & 8191) == 8191) {
                CK(eb.flush() == 0);
                CK(eb.poll() >= 0);
            }
        }
        CK(eb.drain() >= 0);
        CK(es.got == n);
        if (r)
            te += now() - t0;
        ds.got = 0;
        t0 = now();
        for (size_t i = 0; i < n; ++i) {
            CK(db.submit_decode(sv[i % nc], &wires[i * W], W, i) == 0);
            if ((i & 8191) == 8191) {
                CK(db.flush() == 0);
                CK(db.poll() >= 0);
            }
        }
        CK(db.drain() >= 0);
        CK(ds.got == n && ds.ok);
        if (r)
            td += now() - t0;
        CK(memcmp(&back[0], &src[0], n * P) == 0);
    }
    printf("batcher  256 conns    encode %6.1f  decode %6.1f GiB/s  (%.2f / %.2f Mmsg/s)\n",
           rounds * n * P / GiB / te, rounds * n * P / GiB / td, rounds * n / te / 1e6, rounds * n / td / 1e6);
    for (int c = 0; c < nc; ++c) {
        delete cl[c];
        delete sv[c];
    }
    return 0;
}
