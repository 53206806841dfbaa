// curve_encoding_gpu.cpp -- see curve_encoding_gpu.hpp.
#include "curve_encoding_gpu.hpp"

#include <errno.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

namespace zmqg
{
namespace
{
struct thread_state_t
{
    zmqg_ctx *ctx;
    bool failed;
    uint32_t next, limit;
    std::vector<uint32_t> free_sids;
    thread_state_t () : ctx (NULL), failed (false), next (0), limit (0) {}
    ~thread_state_t ()
    {
        if (ctx)
            zmqg_ctx_destroy (ctx);
    }
};
thread_local thread_state_t tls_state;
}

uint32_t session_limit ()
{
    const char *e = getenv ("ZMQG_THREAD_SESSIONS");
    const long v = e ? atol (e) : 0;
    return v > 0 && v <= (1L << 24) ? (uint32_t) v : (uint32_t) thread_sessions;
}

zmqg_ctx *thread_ctx ()
{
    thread_state_t &t = tls_state;
    if (!t.ctx && !t.failed) {
        const char *d = getenv ("ZMQG_DEVICE");
        t.limit = session_limit ();
        if (zmqg_ctx_create (d ? atoi (d) : 0, t.limit, &t.ctx) != 0) {
            t.ctx = NULL;
            t.failed = true;
        }
    }
    return t.ctx;
}

int acquire_session (uint32_t *sid_)
{
    thread_state_t &t = tls_state;
    if (!thread_ctx ()) {
        errno = EIO;
        return -1;
    }
    if (!t.free_sids.empty ()) {
        *sid_ = t.free_sids.back ();
        t.free_sids.pop_back ();
        return 0;
    }
    if (t.next == t.limit) {
        errno = ENOMEM;
        return -1;
    }
    *sid_ = t.next++;
    return 0;
}

void release_session (uint32_t sid_)
{
    tls_state.free_sids.push_back (sid_);
}

curve_encoding_gpu_t::curve_encoding_gpu_t (zmqg_ctx *ctx_,
                                            uint32_t sid_,
                                            const char *encode_nonce_prefix_,
                                            const char *decode_nonce_prefix_,
                                            bool downgrade_sub_) :
    _ctx (ctx_),
    _sid (sid_),
    _cn_nonce (1), // src/curve_mechanism_base.cpp:20-21
    _installed (false),
    _downgrade_sub (downgrade_sub_),
    _peer (1), // src/curve_mechanism_base.cpp:21
    _peer_state (peer_synced)
{
    memcpy (_encode_nonce_prefix, encode_nonce_prefix_, 16);
    memcpy (_decode_nonce_prefix, decode_nonce_prefix_, 16);
    memset (_cn_precom, 0, sizeof _cn_precom);
    memset (_installed_precom, 0, sizeof _installed_precom);
}

int curve_encoding_gpu_t::sync_session ()
{
    if (_installed
        && memcmp (_installed_precom, _cn_precom, sizeof _cn_precom) == 0)
        return 0;
    //  the reference's _cn_peer_nonce starts at 1 (curve_mechanism_base.cpp:21)
    uint64_t peer = 1;
    if (_installed) {
        uint64_t *p;
        if (host_peer (&p) != 0)
            return -1;
        peer = *p;
    }
    if (zmqg_session_set (_ctx, _sid, _cn_precom, _encode_nonce_prefix,
                          _decode_nonce_prefix, _downgrade_sub ? 1 : 0, peer)
        != 0)
        return -1;
    memcpy (_installed_precom, _cn_precom, sizeof _cn_precom);
    _installed = true;
    _peer = peer;
    _peer_state = peer_synced;
    return 0;
}

int curve_encoding_gpu_t::host_peer (uint64_t **peer_)
{
    if (_peer_state == peer_device_ahead) {
        if (zmqg_session_get_peer_nonce (_ctx, _sid, &_peer) != 0)
            return -1;
        _peer_state = peer_synced;
    }
    *peer_ = &_peer;
    return 0;
}

int curve_encoding_gpu_t::device_peer ()
{
    if (_peer_state == peer_host_ahead) {
        if (zmqg_session_set_peer_nonce (_ctx, _sid, _peer) != 0)
            return -1;
        _peer_state = peer_synced;
    }
    return 0;
}

int32_t curve_encoding_gpu_t::frame_verdict (const uint8_t *wire_,
                                             size_t size_,
                                             uint64_t *peer_)
{
    if (size_ <= 1 || size_ <= wire_[0])
        return ZMQG_ERR_MALFORMED_UNSPECIFIED; //  src/mechanism_base.cpp:16-22
    if (size_ < 8 || memcmp (wire_, "\x07MESSAGE", 8) != 0)
        return ZMQG_ERR_UNEXPECTED_COMMAND; //  src/curve_mechanism_base.cpp:85-90
    if (size_ < 33)
        return ZMQG_ERR_MALFORMED_MESSAGE; //  :92-96
    uint64_t nonce = 0;
    for (int k = 0; k < 8; ++k)
        nonce = nonce << 8 | wire_[8 + k]; //  get_uint64: big-endian
    if (nonce <= *peer_)
        return ZMQG_ERR_INVALID_SEQUENCE; //  :99-104
    *peer_ = nonce; //  :105, before the MAC
    return 0;
}

void curve_encoding_gpu_t::set_peer_nonce (nonce_t peer_nonce_)
{
    if (sync_session () == 0
        && zmqg_session_set_peer_nonce (_ctx, _sid, peer_nonce_) == 0) {
        _peer = peer_nonce_;
        _peer_state = peer_synced;
    }
}

curve_encoding_gpu_t::nonce_t curve_encoding_gpu_t::get_peer_nonce () const
{
    if (_peer_state == peer_host_ahead)
        return _peer;
    uint64_t p = 0;
    zmqg_session_get_peer_nonce (_ctx, _sid, &p);
    return p;
}

int curve_encoding_gpu_t::encode_msg (const uint8_t *in_,
                                      size_t len_,
                                      uint8_t flags_,
                                      uint8_t *out_)
{
    if (len_ > 0xffffffffu) {
        errno = EINVAL;
        return -1;
    }
    if (sync_session () != 0) {
        errno = EIO;
        return -1;
    }
    const nonce_t nonce = get_and_inc_nonce (); // src/curve_mechanism_base.cpp:114-116
    const int rc =
      zmqg_encode_msg (_ctx, _sid, nonce, flags_, in_, (uint32_t) len_, out_);
    if (rc != 0) {
        errno = -rc;
        return -1;
    }
    return 0;
}

int curve_encoding_gpu_t::decode_msg (const uint8_t *in_,
                                      size_t wire_len_,
                                      uint8_t *out_,
                                      uint8_t *flags_out_,
                                      int *error_event_code_)
{
    if (wire_len_ > 0xffffffffu) {
        errno = EINVAL;
        return -1;
    }
    if (sync_session () != 0 || device_peer () != 0) {
        errno = EIO;
        return -1;
    }
    //  the host copy follows the device's through the same rule
    uint64_t peer = _peer;
    if (_peer_state == peer_synced)
        frame_verdict (in_, wire_len_, &peer);
    int32_t status = 0;
    const int rc = zmqg_decode_msg (_ctx, _sid, in_, (uint32_t) wire_len_, out_,
                                    flags_out_, &status);
    if (rc != 0) {
        errno = -rc;
        _peer_state = peer_device_ahead;
        return -1;
    }
    _peer = peer;
    if (status != 0) {
        //  src/curve_mechanism_base.cpp:84-108, 277-281
        if (error_event_code_)
            *error_event_code_ = status;
        errno = EPROTO;
        return -1;
    }
    return 0;
}

int curve_encoding_gpu_t::encode (msg_buf_t *msg_)
{
    std::vector<uint8_t> wire (wire_size (msg_->flags, msg_->size ()));
    if (encode_msg (msg_->data (), msg_->size (), msg_->flags, &wire[0]) != 0)
        return -1;
    msg_->bytes.swap (wire);
    msg_->flags = 0; // the boxed message is a fresh msg_t
    return 0;
}

int curve_encoding_gpu_t::decode (msg_buf_t *msg_, int *error_event_code_)
{
    const size_t w = msg_->size ();
    uint8_t fl = 0;
    //  decoded in place: the payload lands at the front of the wire bytes
    if (decode_msg (msg_->data (), w, msg_->data (), &fl, error_event_code_)
        != 0)
        return -1;
    msg_->bytes.resize (w - 33);
    msg_->flags |= fl; // msg_t::set_flags ORs (src/msg.cpp:433-436)
    return 0;
}

int curve_encoding_gpu_t::encode_many (curve_encoding_gpu_t *const *enc_,
                                       msg_buf_t *const *msgs_,
                                       size_t n_)
{
    if (n_ == 0)
        return 0;
    zmqg_ctx *ctx = enc_[0]->_ctx;
    std::vector<uint32_t> sid (n_), len (n_);
    std::vector<uint64_t> nonce (n_), in_off (n_), out_off (n_);
    std::vector<uint8_t> flags (n_);
    uint64_t in_bytes = 0, out_bytes = 0;
    for (size_t i = 0; i < n_; ++i) {
        curve_encoding_gpu_t *e = enc_[i];
        if (e->_ctx != ctx || msgs_[i]->size () > 0xffffffffu) {
            errno = EINVAL;
            return -1;
        }
        if (e->sync_session () != 0) {
            errno = EIO;
            return -1;
        }
        sid[i] = e->_sid;
        nonce[i] = e->get_and_inc_nonce (); // src/curve_mechanism_base.cpp:114-116
        flags[i] = msgs_[i]->flags;
        len[i] = (uint32_t) msgs_[i]->size ();
        in_off[i] = in_bytes;
        in_bytes += len[i];
        out_off[i] = out_bytes;
        out_bytes +=
          zmqg_wire_size (flags[i], e->_downgrade_sub ? 1 : 0, len[i]);
    }
    std::vector<uint8_t> in (in_bytes ? in_bytes : 1), out (out_bytes);
    for (size_t i = 0; i < n_; ++i)
        if (len[i])
            memcpy (&in[in_off[i]], msgs_[i]->data (), len[i]);
    const int rc =
      zmqg_encode_host (ctx, n_, &sid[0], &nonce[0], &flags[0], &in_off[0],
                        &len[0], &in[0], in_bytes, &out_off[0], &out[0],
                        out_bytes);
    if (rc != 0) {
        errno = -rc;
        return -1;
    }
    for (size_t i = 0; i < n_; ++i) {
        const uint64_t end = i + 1 < n_ ? out_off[i + 1] : out_bytes;
        msgs_[i]->bytes.assign (out.begin () + out_off[i], out.begin () + end);
        msgs_[i]->flags = 0; // the boxed message is a fresh msg_t
    }
    return 0;
}

int curve_encoding_gpu_t::decode_many (curve_encoding_gpu_t *const *dec_,
                                       msg_buf_t *const *msgs_,
                                       size_t n_,
                                       int32_t *status_out_)
{
    if (n_ == 0)
        return 0;
    zmqg_ctx *ctx = dec_[0]->_ctx;
    std::vector<uint32_t> sid (n_), wire_len (n_);
    std::vector<uint64_t> in_off (n_), out_off (n_);
    uint64_t in_bytes = 0, out_bytes = 0;
    for (size_t i = 0; i < n_; ++i) {
        curve_encoding_gpu_t *d = dec_[i];
        if (d->_ctx != ctx || msgs_[i]->size () > 0xffffffffu) {
            errno = EINVAL;
            return -1;
        }
        if (d->sync_session () != 0 || d->device_peer () != 0) {
            errno = EIO;
            return -1;
        }
        d->_peer_state = peer_device_ahead; //  the call advances the device's
        sid[i] = d->_sid;
        wire_len[i] = (uint32_t) msgs_[i]->size ();
        in_off[i] = in_bytes;
        in_bytes += wire_len[i];
        out_off[i] = out_bytes;
        out_bytes += wire_len[i] >= 33 ? wire_len[i] - 33 : 0;
    }
    std::vector<uint8_t> in (in_bytes ? in_bytes : 1),
      out (out_bytes ? out_bytes : 1), flags (n_);
    for (size_t i = 0; i < n_; ++i)
        if (wire_len[i])
            memcpy (&in[in_off[i]], msgs_[i]->data (), wire_len[i]);
    const int rc = zmqg_decode_host (ctx, n_, &sid[0], &in_off[0],
                                     &wire_len[0], &in[0], in_bytes,
                                     &out_off[0], &out[0], out_bytes,
                                     &flags[0], status_out_);
    if (rc != 0) {
        errno = -rc;
        return -1;
    }
    for (size_t i = 0; i < n_; ++i) {
        if (status_out_[i] != 0)
            continue; // the reference leaves a failed message undecrypted
        const uint64_t plen = wire_len[i] - 33;
        msgs_[i]->bytes.assign (out.begin () + out_off[i],
                                out.begin () + out_off[i] + plen);
        msgs_[i]->flags |= flags[i]; // msg_t::set_flags ORs (src/msg.cpp:433-436)
    }
    return 0;
}
}
