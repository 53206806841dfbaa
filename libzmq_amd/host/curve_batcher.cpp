// curve_batcher.cpp -- see curve_batcher.hpp.
#include "curve_batcher.hpp"

#include <errno.h>
#include <string.h>
#include <time.h>

namespace zmqg
{
namespace
{
size_t align256 (size_t x)
{
    return (x + 255) & ~(size_t) 255;
}

//  largest wire growth over the payload: "\x07MESSAGE" + nonce + tag + the
//  flags byte + up to 10 bytes of a downgraded SUBSCRIBE/CANCEL prefix
//  (src/curve_mechanism_base.cpp:113-128, 169)
const size_t max_wire_growth = 8 + 8 + 16 + 1 + 10;

uint64_t mono_ns ()
{
    timespec t;
    clock_gettime (CLOCK_MONOTONIC, &t);
    return static_cast<uint64_t> (t.tv_sec) * 1000000000u + t.tv_nsec;
}
}

curve_batcher_t::curve_batcher_t (zmqg_ctx *ctx_,
                                  curve_sink_t *sink_,
                                  const config_t &config_,
                                  void *stream_) :
    _ctx (ctx_),
    _sink (sink_),
    _config (config_),
    _stream (stream_),
    _out_cap (0)
{
    _open[0] = _open[1] = NULL;
    _stats.batch_ns = _stats.fence_ns = _stats.launches = 0;
}

curve_batcher_t::~curve_batcher_t ()
{
    //  nothing may still be reading or writing a slot when it is freed
    wait_idle ();
    for (size_t i = 0; i < _slots.size (); ++i)
        if (_slots[i].base)
            zmqg_host_free (_ctx, _slots[i].base);
}

int curve_batcher_t::init ()
{
    if (!_ctx || !_sink || _config.slots < 2 || _config.slot_msgs == 0
        || _config.slot_bytes == 0 || !_slots.empty ()) {
        errno = EINVAL;
        return -1;
    }
    if (!_stream && zmqg_ctx_stream (_ctx, &_stream) != 0) {
        errno = EINVAL;
        return -1;
    }
    const size_t m = _config.slot_msgs;
    _out_cap = _config.slot_bytes + max_wire_growth * m;
    const size_t o_sid = 0, o_nonce = align256 (o_sid + 4 * m),
                 o_flags = align256 (o_nonce + 8 * m),
                 o_in_off = align256 (o_flags + m),
                 o_len = align256 (o_in_off + 8 * m),
                 o_out_off = align256 (o_len + 4 * m),
                 o_flags_out = align256 (o_out_off + 8 * m),
                 o_status = align256 (o_flags_out + m),
                 o_verdict = align256 (o_status + 4 * m),
                 o_in = align256 (o_verdict + 4 * m),
                 o_out = align256 (o_in + _config.slot_bytes),
                 total = align256 (o_out + _out_cap);
    _slots.resize (_config.slots);
    for (size_t i = 0; i < _slots.size (); ++i) {
        slot_t &s = _slots[i];
        void *p = NULL;
        const int rc = zmqg_host_alloc (_ctx, total, &p);
        if (rc != 0) {
            errno = -rc;
            return -1;
        }
        uint8_t *b = static_cast<uint8_t *> (p);
        s.base = b;
        s.sid = reinterpret_cast<uint32_t *> (b + o_sid);
        s.nonce = reinterpret_cast<uint64_t *> (b + o_nonce);
        s.flags = b + o_flags;
        s.in_off = reinterpret_cast<uint64_t *> (b + o_in_off);
        s.len = reinterpret_cast<uint32_t *> (b + o_len);
        s.out_off = reinterpret_cast<uint64_t *> (b + o_out_off);
        s.flags_out = b + o_flags_out;
        s.status = reinterpret_cast<int32_t *> (b + o_status);
        s.verdict = reinterpret_cast<int32_t *> (b + o_verdict);
        s.in = b + o_in;
        s.out = b + o_out;
        s.tags.resize (m);
        s.kind = encode_kind;
        s.n = s.in_used = s.out_used = 0;
        s.fence = 0;
        _free.push_back (&s);
    }
    return 0;
}

int curve_batcher_t::wait_oldest ()
{
    slot_t *s = _flight.front ();
    const int rc = zmqg_fence_wait (_ctx, s->fence);
    if (rc != 0) {
        errno = -rc;
        return -1;
    }
    _flight.pop_front ();
    return deliver (s);
}

//  Make _open[kind_] a slot with room for one more message of the given
//  input / output bytes, launching the current one when it is full.
int curve_batcher_t::open_slot (kind_t kind_, size_t in_need_, size_t out_need_)
{
    if (in_need_ > _config.slot_bytes || out_need_ > _out_cap) {
        errno = EMSGSIZE;
        return -1;
    }
    slot_t *s = _open[kind_];
    if (s
        && (s->n == _config.slot_msgs
            || s->in_used + in_need_ > _config.slot_bytes
            || s->out_used + out_need_ > _out_cap)) {
        _open[kind_] = NULL;
        if (launch (s) != 0)
            return -1;
        s = NULL;
    }
    if (!s) {
        while (_free.empty ()) {
            if (_flight.empty ()) {
                errno = EAGAIN;
                return -1;
            }
            if (wait_oldest () < 0)
                return -1;
        }
        s = _free.back ();
        _free.pop_back ();
        s->kind = kind_;
        s->n = s->in_used = s->out_used = 0;
        s->max_len = 0;
        _open[kind_] = s;
    }
    return 0;
}

int curve_batcher_t::submit_encode (curve_encoding_gpu_t *conn_,
                                    const uint8_t *data_,
                                    size_t size_,
                                    uint8_t msg_flags_,
                                    uint64_t tag_)
{
    if (_slots.empty () || !conn_ || conn_->_ctx != _ctx
        || (size_ && !data_) || size_ > 0xffffffffu) {
        errno = EINVAL;
        return -1;
    }
    if (conn_->sync_session () != 0) {
        errno = EIO;
        return -1;
    }
    const size_t wire = static_cast<size_t> (
      zmqg_wire_size (msg_flags_, conn_->_downgrade_sub ? 1 : 0, size_));
    if (open_slot (encode_kind, size_, wire) != 0)
        return -1;
    slot_t *s = _open[encode_kind];
    const size_t i = s->n++;
    s->sid[i] = conn_->_sid;
    s->nonce[i] = conn_->get_and_inc_nonce (); // src/curve_mechanism_base.cpp:114-116
    s->flags[i] = msg_flags_;
    s->in_off[i] = s->in_used;
    s->len[i] = static_cast<uint32_t> (size_);
    s->out_off[i] = s->out_used;
    s->tags[i] = tag_;
    if (size_ > s->max_len)
        s->max_len = size_;
    if (size_)
        memcpy (s->in + s->in_used, data_, size_);
    s->in_used += size_;
    s->out_used += wire;
    return 0;
}

int curve_batcher_t::submit_decode (curve_encoding_gpu_t *conn_,
                                    const uint8_t *wire_,
                                    size_t size_,
                                    uint64_t tag_)
{
    if (_slots.empty () || !conn_ || conn_->_ctx != _ctx
        || (size_ && !wire_) || size_ > 0xffffffffu) {
        errno = EINVAL;
        return -1;
    }
    if (conn_->sync_session () != 0) {
        errno = EIO;
        return -1;
    }
    uint64_t *peer = NULL;
    if (_config.replay_host && _config.verify_first
        && conn_->host_peer (&peer) != 0) {
        errno = EIO;
        return -1;
    }
    if (!peer && conn_->device_peer () != 0) {
        errno = EIO;
        return -1;
    }
    //  decoded in place: each payload byte is left over its own ciphertext
    //  byte, at wire offset 33 of the frame, so a decode slot needs no output
    //  area (the reference decrypts into message + 16 instead,
    //  src/curve_mechanism_base.cpp:222-228, and then moves the payload)
    if (open_slot (decode_kind, size_, 0) != 0)
        return -1;
    slot_t *s = _open[decode_kind];
    const size_t i = s->n++;
    s->sid[i] = conn_->_sid;
    s->in_off[i] = s->in_used;
    s->len[i] = static_cast<uint32_t> (size_);
    s->out_off[i] = s->in_used + 33;
    s->tags[i] = tag_;
    if (peer) {
        //  the connection's frames reach this call in receive order
        s->verdict[i] =
          curve_encoding_gpu_t::frame_verdict (wire_, size_, peer);
        if (s->verdict[i] == 0)
            conn_->_peer_state = curve_encoding_gpu_t::peer_host_ahead;
    } else
        conn_->_peer_state = curve_encoding_gpu_t::peer_device_ahead;
    if (size_ > s->max_len)
        s->max_len = size_;
    if (size_)
        memcpy (s->in + s->in_used, wire_, size_);
    s->in_used += size_;
    return 0;
}

int curve_batcher_t::launch (slot_t *s)
{
    int rc;
    const uint64_t t0 = mono_ns ();
    //  the slot's longest frame bounds the batch: a slot of small messages
    //  (every stream within the frame kernel's 4.5 KiB) skips the
    //  large-frame launches
    zmqg_batch_opts o;
    memset (&o, 0, sizeof o);
    o.size = sizeof o;
    o.max_len = s->max_len ? s->max_len : 1;
    if (s->kind == encode_kind)
        rc = zmqg_encode_batch_ex (_ctx, s->n, s->sid, s->nonce, s->flags,
                                   s->in_off, s->len, s->in, s->out_off,
                                   s->out, &o, _stream);
    else {
        //  the slot is host memory the I/O thread can read while the batch
        //  runs: verify before any plaintext reaches it, as libsodium's open
        //  does (src/curve_mechanism_base.cpp:226-228)
        o.flags = _config.verify_first ? ZMQG_OPT_VERIFY_FIRST : 0;
        if (_config.verify_first && _config.replay_host) {
            o.flags |= ZMQG_OPT_REPLAY_HOST;
            o.verdict_in = s->verdict;
        }
        o.out_bytes = s->in_used;
        rc = zmqg_decode_batch_ex (_ctx, s->n, s->sid, s->in_off, s->len,
                                   s->in, s->out_off, s->in, s->flags_out,
                                   s->status, &o, _stream);
    }
    const uint64_t t1 = mono_ns ();
    uint64_t fence = 0;
    if (rc == 0)
        rc = _config.notify_fd >= 0
               ? zmqg_fence_record_notify (_ctx, _stream, _config.notify_fd,
                                           &fence)
               : zmqg_fence_record (_ctx, _stream, &fence);
    if (rc != 0) {
        //  The slot's messages are lost with the device, but kernels of the
        //  batch may have been queued and still read or write the slot: it
        //  goes back to the free list only once the stream is known to have
        //  passed them (its own fence, or a plain one recorded now); when
        //  that cannot be known the slot leaves the rotation.
        if (fence == 0 && zmqg_fence_record (_ctx, _stream, &fence) != 0)
            fence = 0;
        if (fence != 0 && zmqg_fence_wait (_ctx, fence) == 0)
            _free.push_back (s);
        s->n = 0;
        errno = -rc;
        return -1;
    }
    s->fence = fence;
    _flight.push_back (s);
    _stats.batch_ns += t1 - t0;
    _stats.fence_ns += mono_ns () - t1;
    ++_stats.launches;
    return 0;
}

int curve_batcher_t::deliver (slot_t *s)
{
    const int n = static_cast<int> (s->n);
    if (s->kind == encode_kind) {
        for (size_t i = 0; i < s->n; ++i) {
            const uint64_t end = i + 1 < s->n ? s->out_off[i + 1] : s->out_used;
            _sink->on_encoded (s->tags[i], s->out + s->out_off[i],
                               static_cast<size_t> (end - s->out_off[i]));
        }
    } else {
        for (size_t i = 0; i < s->n; ++i) {
            if (s->status[i] == 0)
                _sink->on_decoded (s->tags[i], 0, s->in + s->out_off[i],
                                   s->len[i] - 33u, s->flags_out[i]);
            else
                _sink->on_decoded (s->tags[i], s->status[i], NULL, 0, 0);
        }
    }
    s->n = 0;
    _free.push_back (s);
    return n;
}

int curve_batcher_t::flush ()
{
    //  decode first: received frames usually gate the replies encoded next
    const kind_t order[2] = {decode_kind, encode_kind};
    for (int k = 0; k < 2; ++k) {
        slot_t *s = _open[order[k]];
        if (s && s->n) {
            _open[order[k]] = NULL;
            if (launch (s) != 0)
                return -1;
        }
    }
    return 0;
}

int curve_batcher_t::poll ()
{
    int delivered = 0;
    while (!_flight.empty ()) {
        const int rc = zmqg_fence_query (_ctx, _flight.front ()->fence);
        if (rc < 0) {
            errno = -rc;
            return -1;
        }
        if (rc == 0)
            break;
        slot_t *s = _flight.front ();
        _flight.pop_front ();
        delivered += deliver (s);
    }
    return delivered;
}

int curve_batcher_t::drain ()
{
    if (flush () != 0)
        return -1;
    int delivered = 0;
    while (!_flight.empty ()) {
        const int rc = wait_oldest ();
        if (rc < 0)
            return -1;
        delivered += rc;
    }
    return delivered;
}

int curve_batcher_t::wait_idle ()
{
    int rc = 0;
    for (size_t i = 0; i < _flight.size (); ++i) {
        const int r = zmqg_fence_wait (_ctx, _flight[i]->fence);
        if (r != 0 && rc == 0) {
            errno = -r;
            rc = -1;
        }
    }
    return rc;
}

size_t curve_batcher_t::queued () const
{
    size_t n = 0;
    for (int k = 0; k < 2; ++k)
        if (_open[k])
            n += _open[k]->n;
    return n;
}

size_t curve_batcher_t::in_flight () const
{
    size_t n = 0;
    for (size_t i = 0; i < _flight.size (); ++i)
        n += _flight[i]->n;
    return n;
}
}
