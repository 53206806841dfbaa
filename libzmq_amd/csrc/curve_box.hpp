// curve_box.hpp -- batched handshake boxes:
// crypto_box_easy_afternm / crypto_box_open_easy_afternm with a key and a
// full 24-byte nonce per item.
//
// The CURVE handshake seals every command body with these two calls, under
// a different key/nonce per box, one box per command:
//   HELLO     crypto_box(C', S)  "CurveZMQHELLO---" || short nonce  src/curve_client_tools.hpp:45
//   WELCOME   crypto_box(S', C') "WELCOME-" || 16 random            src/curve_server.cpp:232 (client opens :92)
//   cookie    crypto_secretbox(K) "COOKIE--" || 16 random           src/curve_server.cpp:208 (opens :334)
//   INITIATE  vouch crypto_box(C, S') "VOUCH---" || 16 random      src/curve_client_tools.hpp:140
//             box crypto_box(C', S') "CurveZMQINITIATE" || short    src/curve_client_tools.hpp:177 (opens :291, :359)
//   READY     crypto_box_afternm(precom) "CurveZMQREADY---" || short src/curve_server.cpp:441 (client opens curve_client.cpp:206)
// crypto_box(pk, sk) = crypto_box_afternm(crypto_box_beforenm(pk, sk)) and
// crypto_secretbox(k) = crypto_box_afternm(k) (libsodium 1.0.18), so with
// zmqg_box_beforenm_batch these two kernels produce and open every one of
// them; the reference's NaCl-style zero-padded buffers (crypto_box_ZEROBYTES
// in, BOXZEROBYTES out) are the "easy" layouts here without the padding.
//
// Work split: handshake boxes are small (64 .. a few hundred bytes) and each
// has its own key, so one thread owns one box: HSalsa20(k, n[0:16]) for the
// subkey, then the keystream windows in order with a serial Poly1305 over
// the ciphertext (curve_device.hpp).  Open verifies the tag before it writes
// any plaintext, as libsodium does.
#pragma once

#include "curve_device.hpp"

namespace zmqg {

// Box i: key[32i..], nonce[24i..], message in[in_off[i] .. +len[i]).
// Seal writes tag(16) || ciphertext(len[i]) at out[out_off[i]].
// Open reads tag || ciphertext (len[i] >= 16 bytes) and writes len[i] - 16
// plaintext bytes at out[out_off[i]], status 0; status -1 (and the
// plaintext region zero-filled) for a short box or a tag mismatch.
template <bool OPEN>
__global__ __launch_bounds__(64) void k_box(uint32_t n, const uint8_t *__restrict__ key,
                                            const uint8_t *__restrict__ nonce, const uint64_t *__restrict__ in_off,
                                            const uint32_t *__restrict__ len, const uint8_t *__restrict__ in,
                                            const uint64_t *__restrict__ out_off, uint8_t *__restrict__ out,
                                            int32_t *__restrict__ status)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    uint32_t kw[16], nw[16];
    load_window(key + 32ull * i, 32, kw);
    load_window(nonce + 24ull * i, 24, nw);
    uint32_t sub[8];
    hsalsa20(sub, kw, nw); // XSalsa20: subkey from the first 16 nonce bytes
    const uint32_t n0 = nw[4], n1 = nw[5];
    const uint8_t *src = in + in_off[i];
    uint8_t *dst = out + out_off[i];
    const uint32_t L = len[i];
    if (OPEN && L < 16u) {
        status[i] = -1;
        return;
    }
    const uint32_t mlen = OPEN ? L - 16u : L;
    const uint8_t *ct = OPEN ? src + 16 : nullptr; // ciphertext to authenticate (open)
    uint8_t *ct_out = OPEN ? nullptr : dst + 16;   // ciphertext written (seal)

    uint32_t ks[16];
    salsa20_block(ks, sub, n0, n1, 0, 0);
    const fe r = poly_r_from_key(ks[0], ks[1], ks[2], ks[3]);
    const uint32_t s1 = r.l[1] * 5, s2 = r.l[2] * 5, s3 = r.l[3] * 5, s4 = r.l[4] * 5;
    const uint32_t spad[4] = {ks[4], ks[5], ks[6], ks[7]};
    fe h = fe_zero();
    // Keystream window w covers stream bytes [64w, 64w + 64); message byte p
    // is stream byte 32 + p, so window 0 holds message bytes 0..31 and window
    // w >= 1 bytes [64w - 32, 64w + 32) (16-byte aligned Poly1305 blocks).
    const uint32_t nwin = (mlen + 32u + 63u) / 64u;
    if (OPEN) {
        // authenticate first: Poly1305 over the ciphertext in 64-byte steps
        for (uint32_t p = 0; p < mlen; p += 64u) {
            const int nv = (int) (mlen - p < 64u ? mlen - p : 64u);
            uint32_t c[16];
            load_window(ct + p, nv, c);
            poly_absorb64(h, r, s1, s2, s3, s4, c, nv);
        }
        uint32_t tag[4], got[16];
        poly_finish(h, spad, tag);
        load_window(src, 16, got);
        if ((tag[0] ^ got[0]) | (tag[1] ^ got[1]) | (tag[2] ^ got[2]) | (tag[3] ^ got[3])) {
            for (uint32_t b = 0; b < mlen; ++b)
                dst[b] = 0;
            status[i] = -1;
            return;
        }
    }
    for (uint32_t w = 0; w < nwin; ++w) {
        const uint32_t p0 = w == 0 ? 0u : 64u * w - 32u; // first message byte of the window
        const uint32_t cap = w == 0 ? 32u : 64u;
        const int nv = (int) (mlen - p0 < cap ? mlen - p0 : cap);
        if (w > 0)
            salsa20_block(ks, sub, n0, n1, w, 0);
        uint32_t x[16], y[16];
        load_window(OPEN ? ct + p0 : src + p0, nv, x);
#pragma unroll
        for (int k = 0; k < 16; ++k)
            y[k] = x[k] ^ (w == 0 ? (k < 8 ? ks[8 + k] : 0u) : ks[k]);
        mask_tail(y, nv);
        store_window(OPEN ? dst + p0 : ct_out + p0, nv, y);
        if (!OPEN)
            poly_absorb64(h, r, s1, s2, s3, s4, y, nv);
    }
    if (!OPEN) {
        uint32_t tag[16] = {0};
        poly_finish(h, spad, tag);
        store_window(dst, 16, tag);
    }
    if (status)
        status[i] = 0;
}

} // namespace zmqg
