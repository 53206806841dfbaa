"""The C++ curve_encoding_t mirror (libzmq_amd/host) over the C ABI: it
compiles and links against the product library here; on a GPU it runs the
round trips of the reference's unittests/unittest_curve_encoding.cpp plus the
error paths and the batched forms (tests/host/test_curve_encoding_gpu.cpp)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_DIR = os.path.join(ROOT, "libzmq_amd")


def build_adapter_test(out_dir):
    exe = os.path.join(out_dir, "test_curve_encoding_gpu")
    cmd = ["g++", "-O2", "-std=c++11", "-Wall", "-Werror", "-o", exe,
           os.path.join(ROOT, "tests", "host", "test_curve_encoding_gpu.cpp"),
           os.path.join(ROOT, "libzmq_amd", "host", "curve_encoding_gpu.cpp"),
           "-L" + LIB_DIR, "-lzmqg_curve", "-Wl,-rpath," + LIB_DIR,
           "-L/opt/rocm/lib", "-Wl,-rpath-link,/opt/rocm/lib"]
    subprocess.check_call(cmd)
    return exe


def test_adapter_compiles_and_links(tmp_path):
    exe = build_adapter_test(str(tmp_path))
    assert os.path.exists(exe)


@pytest.mark.gpu
def test_adapter_roundtrips_on_gpu(tmp_path):
    exe = build_adapter_test(str(tmp_path))
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr + r.stdout
    assert r.stdout.strip() == "OK 7"
