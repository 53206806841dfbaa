"""CPU-side checks of the drop-in boundary: the C-ABI library loads and
exports every function include/zmqg_curve.h declares (no GPU calls), and the
host-only helpers agree with the oracle."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "zmqg_curve.h")
LIB = os.path.join(ROOT, "libzmq_amd", "libzmqg_curve.so")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(zmqg_[a-z_0-9]+)\s*\(", text)))


def test_header_declares_expected_entry_points():
    names = declared_functions()
    for required in ["zmqg_ctx_create", "zmqg_ctx_destroy", "zmqg_session_set", "zmqg_encode_batch",
                     "zmqg_decode_batch", "zmqg_encode_host", "zmqg_decode_host", "zmqg_wire_size"]:
        assert required in names


def test_library_exports_every_declared_symbol():
    assert os.path.exists(LIB), "build first: make -C libzmq_amd/csrc"
    out = subprocess.check_output(["nm", "-D", "--defined-only", LIB]).decode()
    exported = set(l.split()[-1] for l in out.splitlines() if l.strip())
    missing = [n for n in declared_functions() if n not in exported]
    assert not missing, missing


def test_library_loads_and_reports_abi_version():
    lib = ctypes.CDLL(LIB)
    assert lib.zmqg_abi_version() == 5


def test_header_compiles_as_c():
    src = '#include "zmqg_curve.h"\nint main(void){return zmqg_abi_version()==ZMQG_CURVE_ABI_VERSION?0:1;}\n'
    r = subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-fsyntax-only", "-I", os.path.join(ROOT, "include"),
                        "-x", "c", "-"], input=src.encode(), capture_output=True)
    assert r.returncode == 0, r.stderr.decode()


@pytest.mark.parametrize("flags,down,plen", [(0, 0, 0), (1, 0, 1024), (12, 0, 5), (12, 1, 5), (16, 0, 0),
                                             (16, 1, 3), (13, 0, 7), (4, 0, 9), (0x80 | 1, 0, 2)])
def test_wire_size_matches_oracle(flags, down, plen):
    from libzmq_amd import curve
    from oracle import oracle as O
    assert curve.wire_size(flags, down, plen) == O.wire_size(flags, down, plen)


def test_status_codes_match_zmq_h():
    text = open(HEADER).read()
    codes = dict(re.findall(r"#define (ZMQG_ERR_[A-Z_]+) (0x[0-9a-f]+)", text))
    assert int(codes["ZMQG_ERR_UNEXPECTED_COMMAND"], 16) == 0x10000001
    assert int(codes["ZMQG_ERR_INVALID_SEQUENCE"], 16) == 0x10000002
    assert int(codes["ZMQG_ERR_MALFORMED_UNSPECIFIED"], 16) == 0x10000011
    assert int(codes["ZMQG_ERR_MALFORMED_MESSAGE"], 16) == 0x10000012
    assert int(codes["ZMQG_ERR_CRYPTOGRAPHIC"], 16) == 0x11000001
