// curve_engine_hook.cpp -- see curve_engine_hook.hpp.
#include "curve_engine_hook.hpp"

#include <errno.h>
#include <string.h>
#include <sys/eventfd.h>
#include <unistd.h>

namespace zmqg
{
void result_fifo_t::push (const uint8_t *data_, size_t size_, uint8_t flags_)
{
    if (_tail + size_ > _buf.size ()) {
        if (_head > 0) {
            //  (the records before _head are gone: slide the rest down)
            memmove (&_buf[0], &_buf[0] + _head, _tail - _head);
            _tail -= _head;
            _head = 0;
        }
        if (_tail + size_ > _buf.size ()) {
            size_t cap = _buf.size () ? _buf.size () * 2 : 64u << 10;
            while (cap < _tail + size_)
                cap *= 2;
            _buf.resize (cap);
        }
    }
    if (size_)
        memcpy (&_buf[0] + _tail, data_, size_);
    _tail += size_;
    _recs.push_back (std::make_pair (size_, flags_));
}

void result_fifo_t::pop ()
{
    _head += _recs.front ().first;
    _recs.pop_front ();
    if (_recs.empty ())
        _head = _tail = 0;
}

namespace
{
//  the hook's wake-up descriptor, as the mailbox's signaler makes its own
//  (src/signaler.cpp: eventfd, non-blocking, close-on-exec)
int make_eventfd ()
{
    return eventfd (0, EFD_NONBLOCK | EFD_CLOEXEC);
}

curve_batcher_t::config_t with_fd (curve_batcher_t::config_t config_, int fd_)
{
    config_.notify_fd = fd_;
    return config_;
}
}

curve_io_hook_t::curve_io_hook_t (zmqg_ctx *ctx_,
                                  const curve_batcher_t::config_t &config_,
                                  void *stream_) :
    _ctx (ctx_),
    _fd (make_eventfd ()),
    _batcher (ctx_, this, with_fd (config_, _fd), stream_),
    _next_id (0)
{
}

curve_io_hook_t::~curve_io_hook_t ()
{
    //  the slots' notifications write _fd: it stays open until they ran (and
    //  open for good when the ctx cannot tell: a stream that never reaches
    //  them must not write into a descriptor number reused by then)
    _batcher.wait_idle ();
    if (_ctx && zmqg_notify_quiesce (_ctx) != 0)
        return;
    if (_fd >= 0)
        close (_fd);
}

int curve_io_hook_t::init ()
{
    if (_fd < 0)
        return -1; //  errno from eventfd
    return _batcher.init ();
}

int curve_io_hook_t::in_event ()
{
    //  clear the counter first: a batch finishing after this read writes
    //  it again, so no completion is lost between the read and the poll
    uint64_t v;
    while (read (_fd, &v, sizeof v) < 0 && errno == EINTR)
        ;
    const int n = _batcher.poll ();
    if (n < 0)
        return -1;
    resume ();
    return n;
}

int curve_io_hook_t::timer_event ()
{
    const int rc = _batcher.flush ();
    resume ();
    return rc;
}

int curve_io_hook_t::iteration ()
{
    if (_batcher.flush () != 0)
        return -1;
    const int n = _batcher.poll ();
    if (n < 0)
        return -1;
    resume ();
    return n;
}

int curve_io_hook_t::drain ()
{
    const int n = _batcher.drain ();
    if (n < 0)
        return -1;
    resume ();
    return n;
}

size_t curve_io_hook_t::outstanding () const
{
    return _batcher.queued () + _batcher.in_flight ();
}

curve_engine_link_t *curve_io_hook_t::find (uint64_t id_) const
{
    const std::map<uint64_t, curve_engine_link_t *>::const_iterator it =
      _links.find (id_);
    return it == _links.end () ? NULL : it->second;
}

void curve_io_hook_t::resume ()
{
    //  a callback may submit (a back-pressure wait then delivers more and
    //  marks more links), close links, or open new ones: every link is
    //  looked up by id at its turn
    while (!_out_ready.empty () || !_in_ready.empty ()) {
        std::vector<uint64_t> in, out;
        in.swap (_in_ready);
        out.swap (_out_ready);
        for (size_t i = 0; i < in.size (); ++i) {
            curve_engine_link_t *l = find (in[i]);
            if (l && l->_events)
                l->_events->decoded_ready ();
        }
        for (size_t i = 0; i < out.size (); ++i) {
            curve_engine_link_t *l = find (out[i]);
            if (l && l->_events)
                l->_events->encoded_ready ();
        }
    }
}

//  The tag of every submission is its link's id: the batcher delivers each
//  connection's results in submission order, so appending keeps the order.
void curve_io_hook_t::on_encoded (uint64_t tag_,
                                  const uint8_t *wire_,
                                  size_t size_)
{
    curve_engine_link_t *l = find (tag_);
    if (!l)
        return; //  closed while in flight
    --l->_send_pending;
    const bool first = l->_encoded.empty ();
    l->_encoded.push (wire_, size_, 0);
    if (first)
        _out_ready.push_back (tag_);
}

void curve_io_hook_t::on_decoded (uint64_t tag_,
                                  int status_,
                                  const uint8_t *payload_,
                                  size_t size_,
                                  uint8_t flags_)
{
    curve_engine_link_t *l = find (tag_);
    if (!l)
        return;
    --l->_recv_pending;
    if (l->_failed)
        return; //  after a failure nothing more reaches the session
    const bool first = l->_decoded.empty ();
    if (status_ != 0) {
        //  curve_mechanism_base_t::decode returned -1 with this
        //  error_event_code: the engine's protocol-error path.  Messages
        //  decoded before it stay queued: the reference had pushed them to
        //  the session already.
        l->_failed = status_;
        _in_ready.push_back (tag_);
        return;
    }
    l->_decoded.push (payload_, size_, flags_);
    if (first)
        _in_ready.push_back (tag_);
}

curve_engine_link_t::curve_engine_link_t (curve_io_hook_t *hook_,
                                          curve_encoding_gpu_t *codec_,
                                          curve_link_events_t *events_) :
    _hook (hook_),
    _codec (codec_),
    _events (events_),
    _id (++hook_->_next_id),
    _send_pending (0),
    _recv_pending (0),
    _failed (0)
{
    _hook->_links[_id] = this;
}

curve_engine_link_t::~curve_engine_link_t ()
{
    _hook->_links.erase (_id);
}

int curve_engine_link_t::submit_send (const uint8_t *data_,
                                      size_t size_,
                                      uint8_t msg_flags_)
{
    if (_failed) {
        errno = EPIPE;
        return -1;
    }
    //  counted before the submit: a back-pressure wait inside it may deliver
    //  this very message
    ++_send_pending;
    if (_hook->_batcher.submit_encode (_codec, data_, size_, msg_flags_, _id)
        != 0) {
        --_send_pending;
        return -1;
    }
    return 0;
}

bool curve_engine_link_t::next_encoded (std::vector<uint8_t> &wire_)
{
    if (_encoded.empty ())
        return false;
    wire_.assign (_encoded.front_data (),
                  _encoded.front_data () + _encoded.front_size ());
    _encoded.pop ();
    return true;
}

bool curve_engine_link_t::peek_encoded (const uint8_t **wire_,
                                        size_t *size_) const
{
    if (_encoded.empty ())
        return false;
    *wire_ = _encoded.front_data ();
    *size_ = _encoded.front_size ();
    return true;
}

int curve_engine_link_t::submit_received (const uint8_t *wire_, size_t size_)
{
    if (_failed) {
        errno = EPIPE;
        return -1;
    }
    ++_recv_pending;
    if (_hook->_batcher.submit_decode (_codec, wire_, size_, _id) != 0) {
        --_recv_pending;
        return -1;
    }
    return 0;
}

bool curve_engine_link_t::next_decoded (msg_buf_t &msg_)
{
    if (_decoded.empty ())
        return false;
    msg_.bytes.assign (_decoded.front_data (),
                       _decoded.front_data () + _decoded.front_size ());
    msg_.flags = _decoded.front_flags ();
    _decoded.pop ();
    return true;
}

bool curve_engine_link_t::peek_decoded (const uint8_t **payload_,
                                        size_t *size_,
                                        uint8_t *flags_) const
{
    if (_decoded.empty ())
        return false;
    *payload_ = _decoded.front_data ();
    *size_ = _decoded.front_size ();
    *flags_ = _decoded.front_flags ();
    return true;
}
}
