"""The reference-side binding.

libzmq_amd/host/zmq_curve_encoding.hpp is the zmq::curve_encoding_t that
src/curve_mechanism_base.hpp includes under ZMQ_USE_ZMQG_CURVE.  Here it is
compiled to an object against the reference's own headers -- msg.hpp
(msg_t::init_size/move/shrink/set_flags/data/size/flags,
src/msg.hpp:62-190), err.hpp (errno_assert), macros.hpp
(ZMQ_NON_COPYABLE_NOR_MOVABLE), include/zmq.h and src/zmq_draft.h, in the
order src/precompiled.hpp includes the public ones -- together with a
translation unit that uses the class the way curve_mechanism_base_t and the
handshake do (src/curve_mechanism_base.cpp:38-52, src/curve_client_tools.hpp:
105, src/curve_server.cpp:382-383).  Object only: the reference's msg.cpp
includes its cmake-generated platform.hpp, so msg_t's definitions are not
linked here; the adapter underneath is linked and run
against the device by tests/host/test_curve_encoding_gpu.cpp.

Reads /root/reference at test time, so CPU-only (skipped where it is absent,
e.g. on the GPU box)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"

USE = r"""
#include "../include/zmq.h"
#include "zmq_draft.h"
#include "zmq_curve_encoding.hpp"

//  what curve_mechanism_base_t (src/curve_mechanism_base.cpp:38-52) and the
//  handshake (src/curve_client_tools.hpp:105, src/curve_server.cpp:382-383,
//  src/curve_client.cpp:206) call on the codec
int mechanism_use (zmq::curve_encoding_t *c_, zmq::msg_t *msg_)
{
    int error_event_code = 0;
    memset (c_->get_writable_precom_buffer (), 0, 32);
    const zmq::curve_encoding_t::nonce_t n = c_->get_and_inc_nonce ();
    c_->set_peer_nonce (n + 1);
    int rc = c_->encode (msg_);
    rc |= c_->decode (msg_, &error_event_code);
    return rc + error_event_code + (c_->get_precom_buffer () != NULL);
}

zmq::curve_encoding_t *make_client_codec (bool downgrade_sub_)
{
    //  src/curve_client.cpp:22-23
    return new zmq::curve_encoding_t ("CurveZMQMESSAGEC", "CurveZMQMESSAGES",
                                      downgrade_sub_);
}

void drop_codec (zmq::curve_encoding_t *c_)
{
    delete c_;
}
"""

# symbols the object must take from the reference's msg_t and from the adapter
NEEDED = [
    "zmq::msg_t::init_size(unsigned long)",
    "zmq::msg_t::move(zmq::msg_t&)",
    "zmq::msg_t::shrink(unsigned long)",
    "zmq::msg_t::set_flags(unsigned char)",
    "zmq::msg_t::data()",
    "zmq::msg_t::size() const",
    "zmq::msg_t::flags() const",
    "zmqg::curve_encoding_gpu_t::encode_msg(unsigned char const*, unsigned long, unsigned char, unsigned char*)",
    "zmqg::curve_encoding_gpu_t::decode_msg(unsigned char const*, unsigned long, unsigned char*, unsigned char*, int*)",
    "zmqg::acquire_session(unsigned int*)",
    "zmqg::release_session(unsigned int)",
    "zmqg::thread_ctx()",
]


@pytest.mark.skipif(not os.path.exists(os.path.join(REF, "src", "msg.hpp")),
                    reason="reference sources not present")
def test_binding_compiles_against_reference_msg_t(tmp_path):
    src = tmp_path / "use_binding.cpp"
    src.write_text(USE)
    obj = tmp_path / "use_binding.o"
    cmd = ["g++", "-std=c++11", "-O2", "-Wall", "-Werror", "-c", "-o", str(obj), str(src),
           "-I" + os.path.join(REF, "src"), "-I" + os.path.join(REF, "include"),
           "-I" + os.path.join(ROOT, "libzmq_amd", "host")]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    syms = subprocess.run(["nm", "-C", "--undefined-only", str(obj)], capture_output=True, text=True,
                          check=True).stdout
    missing = [s for s in NEEDED if s not in syms]
    assert not missing, (missing, syms)


@pytest.mark.skipif(not os.path.exists(os.path.join(REF, "src", "msg.cpp")),
                    reason="reference sources not present")
def test_binding_links_reference_msg_t():
    """SURVEY a10 on the reference's own msg_t: tests/host/build_ref_binding.sh
    compiles src/msg.cpp, metadata.cpp and err.cpp where they lie (test-only
    platform.hpp) and links them with the drop-in codec and
    tests/host/test_zmq_binding.cpp; the executable's msg_t is the reference's
    (run on the GPU by tests/test_host_adapter.py)."""
    r = subprocess.run(["sh", os.path.join(ROOT, "tests", "host", "build_ref_binding.sh")], capture_output=True,
                       text=True)
    assert r.returncode == 0, r.stderr + r.stdout
    exe = os.path.join(ROOT, "tests", "host", "_ref", "test_zmq_binding_ref")
    syms = subprocess.run(["nm", "-C", "--defined-only", exe], capture_output=True, text=True, check=True).stdout
    for s in ("zmq::msg_t::init_size(unsigned long)", "zmq::msg_t::move(zmq::msg_t&)",
              "zmq::msg_t::shrink(unsigned long)", "zmq::msg_t::set_flags(unsigned char)",
              "zmq::msg_t::init_external_storage(", "zmq::metadata_t::drop_ref()"):
        assert s in syms, s
