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
    assert r.stdout.strip() == "OK 8"


def build_batcher_test(out_dir):
    exe = os.path.join(out_dir, "test_curve_batcher")
    cmd = ["g++", "-O2", "-std=c++11", "-Wall", "-Werror", "-o", exe,
           os.path.join(ROOT, "tests", "host", "test_curve_batcher.cpp"),
           os.path.join(ROOT, "libzmq_amd", "host", "curve_batcher.cpp"),
           os.path.join(ROOT, "libzmq_amd", "host", "curve_encoding_gpu.cpp"),
           "-L" + LIB_DIR, "-lzmqg_curve", "-Wl,-rpath," + LIB_DIR,
           "-L/opt/rocm/lib", "-Wl,-rpath-link,/opt/rocm/lib"]
    subprocess.check_call(cmd)
    return exe


def build_engine_hook_test(out_dir):
    exe = os.path.join(out_dir, "test_engine_hook")
    cmd = ["g++", "-O2", "-std=c++11", "-Wall", "-Werror", "-o", exe,
           os.path.join(ROOT, "tests", "host", "test_engine_hook.cpp"),
           os.path.join(ROOT, "libzmq_amd", "host", "curve_engine_hook.cpp"),
           os.path.join(ROOT, "libzmq_amd", "host", "curve_batcher.cpp"),
           os.path.join(ROOT, "libzmq_amd", "host", "curve_encoding_gpu.cpp"),
           "-L" + LIB_DIR, "-lzmqg_curve", "-Wl,-rpath," + LIB_DIR,
           "-L/opt/rocm/lib", "-Wl,-rpath-link,/opt/rocm/lib", "-lpthread"]
    subprocess.check_call(cmd)
    return exe


def test_engine_hook_compiles_and_links(tmp_path):
    assert os.path.exists(build_engine_hook_test(str(tmp_path)))


@pytest.mark.gpu
def test_engine_hook_drives_batcher_like_the_engine(tmp_path):
    """SURVEY 8f row 1, engine side: curve_io_hook_t / curve_engine_link_t
    driven by two I/O threads that sleep in epoll_wait with no timeout
    (src/epoll.cpp:140-179) over real non-blocking socketpairs, woken only by
    the sockets and the hooks' eventfds (batch completion), engines resumed
    through restart_output / restart_input (src/stream_engine_base.cpp:
    383-390, 400-442); 16 connections, a tampered frame failing only its own
    connection, a link closed with messages in flight; a 60 s watchdog
    bounds the run."""
    exe = build_engine_hook_test(str(tmp_path))
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr + r.stdout
    assert r.stdout.startswith("OK 4800 "), r.stdout
    print(r.stdout.strip())


def test_batcher_compiles_and_links(tmp_path):
    assert os.path.exists(build_batcher_test(str(tmp_path)))


def _read_batcher_records(path):
    import numpy as np
    raw = open(path, "rb").read()
    n_conn, n_msgs = np.frombuffer(raw[:8], np.uint32)
    p = 8
    precoms = [raw[p + 32 * c:p + 32 * (c + 1)] for c in range(n_conn)]
    p += 32 * n_conn
    downgrade = list(raw[p:p + n_conn])
    p += n_conn
    recs = []
    for _ in range(n_msgs):
        conn, flags, plen, wlen = np.frombuffer(raw[p:p + 16], np.uint32)
        p += 16
        payload = raw[p:p + plen]
        p += plen
        wire = raw[p:p + wlen]
        p += wlen
        recs.append((int(conn), int(flags), payload, wire))
    assert p == len(raw)
    return precoms, downgrade, recs


@pytest.mark.gpu
def test_batcher_matches_per_message_path_and_oracle(tmp_path):
    """The async batcher on a GPU (its own checks against the n = 1 path),
    then every frame it encoded against the CPU oracle, one by one."""
    import numpy as np
    from oracle import oracle as O
    exe = build_batcher_test(str(tmp_path))
    dump = os.path.join(str(tmp_path), "records.bin")
    r = subprocess.run([exe, dump], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr + r.stdout
    assert r.stdout.startswith("OK ")
    precoms, downgrade, recs = _read_batcher_records(dump)
    sessions = np.concatenate([O.make_sessions([p], downgrade_sub=bool(d)) for p, d in zip(precoms, downgrade)])
    checked = 0
    for conn, flags, payload, wire in recs:
        nonce = int.from_bytes(wire[8:16], "big")
        inp = np.frombuffer(payload, np.uint8) if payload else np.zeros(1, np.uint8)
        ref = O.encode_batch(sessions, [conn], [nonce], [flags], [0], [len(payload)], inp, [0], len(wire))
        assert O.wire_size(flags, downgrade[conn], len(payload)) == len(wire)
        assert ref.tobytes() == wire
        checked += 1
    assert checked == len(recs) > 1000


def build_binding_test(out_dir):
    """zmq_curve_encoding.hpp (the drop-in zmq::curve_encoding_t) over the
    msg_t test double of tests/host/msg_model (see its header)."""
    exe = os.path.join(out_dir, "test_zmq_binding")
    cmd = ["g++", "-O2", "-std=c++11", "-Wall", "-Werror", "-o", exe,
           "-I" + os.path.join(ROOT, "tests", "host", "msg_model"),
           "-I" + os.path.join(ROOT, "libzmq_amd", "host"),
           os.path.join(ROOT, "tests", "host", "test_zmq_binding.cpp"),
           os.path.join(ROOT, "libzmq_amd", "host", "curve_encoding_gpu.cpp"),
           "-L" + LIB_DIR, "-lzmqg_curve", "-Wl,-rpath," + LIB_DIR,
           "-L/opt/rocm/lib", "-Wl,-rpath-link,/opt/rocm/lib"]
    subprocess.check_call(cmd)
    return exe


def test_binding_compiles_and_links(tmp_path):
    assert os.path.exists(build_binding_test(str(tmp_path)))


@pytest.mark.gpu
def test_binding_runs_on_msg_t(tmp_path):
    """the four unittest_curve_encoding.cpp round trips on msg_t
    objects (VSM / LMSG split, move, shrink, set_flags OR), subscribe, a
    tampered box, and a connection without a session slot (no abort)."""
    exe = build_binding_test(str(tmp_path))
    env = dict(os.environ, ZMQG_THREAD_SESSIONS="4")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr + r.stdout
    assert r.stdout.strip() == "OK 14"


@pytest.mark.gpu
def test_binding_runs_on_reference_msg_t():
    """SURVEY a10 on the REFERENCE's msg_t (src/msg.cpp:62-94 init_size,
    305-324 move, 404-436 shrink / set_flags, 108-129 external storage),
    prebuilt by tests/host/build_ref_binding.sh in the build step (the
    reference is not on the GPU box): the same round trips as above plus
    decode in place on zero-copy msg_t slices of a shared receive buffer
    (src/v2_decoder.cpp:88-113)."""
    exe = os.path.join(ROOT, "tests", "host", "_ref", "test_zmq_binding_ref")
    if not os.path.exists(exe):
        pytest.skip("tests/host/_ref/test_zmq_binding_ref not built (needs the reference sources at build time)")
    env = dict(os.environ, ZMQG_THREAD_SESSIONS="4")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr + r.stdout
    assert r.stdout.strip() == "OK 15"
