// Test double of libzmq's zmq::msg_t for tests/host/test_zmq_binding.cpp.
//
// NOT the reference's msg_t: the reference's src/msg.cpp includes its
// cmake-generated platform.hpp, and a reference build from stand-ins for
// generated headers is not made here.  This class
// restates, in a few lines each, the parts of msg_t the binding
// (libzmq_amd/host/zmq_curve_encoding.hpp) calls, with the reference's
// semantics:
//   init_size  src/msg.cpp:62-94   size <= max_vsm_size (33, src/msg.hpp:
//                                  154-156) inline ("VSM"), else one malloc
//                                  of header + size ("LMSG"); flags 0
//   move       src/msg.cpp:305-324 close this, take src's state, re-init src
//   shrink     src/msg.cpp:404-425 size = new_size (<= size)
//   set_flags  src/msg.cpp:433-436 flags |= f
//   flags / data / size
// plus is_vsm() for the test's own checks.
#ifndef ZMQG_TEST_MSG_MODEL_HPP
#define ZMQG_TEST_MSG_MODEL_HPP

#include <assert.h>
#include <errno.h>
#include <stddef.h>
#include <stdlib.h>
#include <string.h>

namespace zmq
{
class msg_t
{
  public:
    enum
    {
        more = 1,
        command = 2,
        subscribe = 12,
        cancel = 16,
        max_vsm_size = 33
    };

    msg_t () : _lmsg (NULL), _size (0), _flags (0), _vsm (true) {}
    ~msg_t () { close (); }

    int init ()
    {
        close ();
        _vsm = true;
        _size = 0;
        _flags = 0;
        return 0;
    }
    int init_size (size_t size_)
    {
        close ();
        _flags = 0;
        _size = size_;
        _vsm = size_ <= max_vsm_size;
        if (!_vsm) {
            _lmsg = static_cast<unsigned char *> (malloc (size_));
            if (!_lmsg) {
                errno = ENOMEM;
                return -1;
            }
        }
        return 0;
    }
    int close ()
    {
        if (!_vsm)
            free (_lmsg);
        _lmsg = NULL;
        _vsm = true;
        _size = 0;
        return 0;
    }
    int move (msg_t &src_)
    {
        close ();
        _vsm = src_._vsm;
        _size = src_._size;
        _flags = src_._flags;
        if (_vsm)
            memcpy (_inline, src_._inline, sizeof _inline);
        else
            _lmsg = src_._lmsg;
        src_._lmsg = NULL;
        src_._vsm = true;
        src_.init ();
        return 0;
    }
    void shrink (size_t new_size_)
    {
        assert (new_size_ <= _size);
        _size = new_size_;
    }
    void set_flags (unsigned char flags_) { _flags |= flags_; }
    unsigned char flags () const { return _flags; }
    void *data () { return _vsm ? _inline : _lmsg; }
    size_t size () const { return _size; }
    bool is_vsm () const { return _vsm; }

  private:
    unsigned char _inline[max_vsm_size];
    unsigned char *_lmsg;
    size_t _size;
    unsigned char _flags;
    bool _vsm;

    msg_t (const msg_t &);
    msg_t &operator= (const msg_t &);
};
}

#endif
