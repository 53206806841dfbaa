// curve_engine_hook.cpp -- see curve_engine_hook.hpp.
#include "curve_engine_hook.hpp"

#include <errno.h>

namespace zmqg
{
curve_io_hook_t::curve_io_hook_t (zmqg_ctx *ctx_,
                                  const curve_batcher_t::config_t &config_,
                                  void *stream_) :
    _batcher (ctx_, this, config_, stream_)
{
}

int curve_io_hook_t::init ()
{
    return _batcher.init ();
}

int curve_io_hook_t::iteration ()
{
    if (_batcher.flush () != 0)
        return -1;
    return _batcher.poll ();
}

int curve_io_hook_t::drain ()
{
    return _batcher.drain ();
}

size_t curve_io_hook_t::outstanding () const
{
    return _batcher.queued () + _batcher.in_flight ();
}

//  The tag of every submission is its link: the batcher delivers each
//  connection's results in submission order, so appending keeps the order.
void curve_io_hook_t::on_encoded (uint64_t tag_,
                                  const uint8_t *wire_,
                                  size_t size_)
{
    curve_engine_link_t *l = reinterpret_cast<curve_engine_link_t *> (tag_);
    if (!_links.count (l))
        return;
    --l->_send_pending;
    l->_encoded.push_back (std::vector<uint8_t> (wire_, wire_ + size_));
}

void curve_io_hook_t::on_decoded (uint64_t tag_,
                                  int status_,
                                  const uint8_t *payload_,
                                  size_t size_,
                                  uint8_t flags_)
{
    curve_engine_link_t *l = reinterpret_cast<curve_engine_link_t *> (tag_);
    if (!_links.count (l))
        return;
    --l->_recv_pending;
    if (l->_failed)
        return; //  after a failure nothing more reaches the session
    if (status_ != 0) {
        //  curve_mechanism_base_t::decode returned -1 with this
        //  error_event_code: the engine's protocol-error path.  Messages
        //  decoded before it stay queued: the reference had pushed them to
        //  the session already.
        l->_failed = status_;
        return;
    }
    msg_buf_t m;
    m.bytes.assign (payload_, payload_ + size_);
    m.flags = flags_;
    l->_decoded.push_back (m);
}

curve_engine_link_t::curve_engine_link_t (curve_io_hook_t *hook_,
                                          curve_encoding_gpu_t *codec_) :
    _hook (hook_),
    _codec (codec_),
    _send_pending (0),
    _recv_pending (0),
    _failed (0)
{
    _hook->_links.insert (this);
}

curve_engine_link_t::~curve_engine_link_t ()
{
    _hook->_links.erase (this);
}

int curve_engine_link_t::submit_send (const uint8_t *data_,
                                      size_t size_,
                                      uint8_t msg_flags_)
{
    if (_failed) {
        errno = EPIPE;
        return -1;
    }
    if (_hook->_batcher.submit_encode (_codec, data_, size_, msg_flags_,
                                       reinterpret_cast<uint64_t> (this))
        != 0)
        return -1;
    ++_send_pending;
    return 0;
}

bool curve_engine_link_t::next_encoded (std::vector<uint8_t> &wire_)
{
    if (_encoded.empty ())
        return false;
    wire_.swap (_encoded.front ());
    _encoded.pop_front ();
    return true;
}

int curve_engine_link_t::submit_received (const uint8_t *wire_, size_t size_)
{
    if (_failed) {
        errno = EPIPE;
        return -1;
    }
    if (_hook->_batcher.submit_decode (_codec, wire_, size_,
                                       reinterpret_cast<uint64_t> (this))
        != 0)
        return -1;
    ++_recv_pending;
    return 0;
}

bool curve_engine_link_t::next_decoded (msg_buf_t &msg_)
{
    if (_decoded.empty ())
        return false;
    msg_.bytes.swap (_decoded.front ().bytes);
    msg_.flags = _decoded.front ().flags;
    _decoded.pop_front ();
    return true;
}
}
