"""Config 1's plumbing (BASELINE.json configs[0]): CURVE PUSH/PULL over
tcp://127.0.0.1 between two builds of the reference libzmq -- the stock one
(libsodium codec) and the one with INTEGRATION.md section 2 applied
(tests/host/libzmq_zmqg.patch: curve_encoding_t swapped for the GPU codec,
the stream engine, I/O threads, handshake and sockets untouched).  Built by
tests/host/build_libzmq.sh (run by __graft_entry__.build()); the test
program is tests/host/test_curve_interop.cpp, shaped like the reference's
perf/local_thr.cpp / perf/remote_thr.cpp with CURVE set up as
tests/test_security_curve.cpp does.

Each run sends 100,000 messages (1 KiB, plus 0 B, 33 B, 64 B and 64 KiB ones
and three-part MORE messages) with ZMTP heartbeats every 5 ms on both
sides (PING/PONG through the codec, src/zmtp_engine.cpp:463, 479); the
receiver checks every part byte for byte, its size and its MORE flag, then
acknowledges over a second CURVE connection the other way.  This is
interop evidence between the two codecs on real sockets, not an oracle pin.

CPU: the stock pair (checks the harness).  GPU: GPU-codec server with a
stock client, the reverse, and GPU on both sides.  PUB/SUB runs the SUB's
SUBSCRIBE / CANCEL commands across the two codecs in both directions."""
import os
import socket
import subprocess
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "host", "_ref", "libzmq")
N = 100000


def _exe(kind):
    p = os.path.join(BIN, "interop_" + kind)
    if not os.path.exists(p):
        pytest.skip("interop build absent (tests/host/build_libzmq.sh needs /root/reference and libsodium)")
    return p


def _ports():
    socks = []
    for _ in range(2):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        socks.append(s)
    ports = [s.getsockname()[1] for s in socks]
    for s in socks:
        s.close()
    return ports


def run_pair(server_kind, client_kind, n=N, seed=11, heartbeat_ms=5):
    """PULL (CURVE server) built as server_kind, PUSH (CURVE client) as
    client_kind; returns the receiver's line: OK n parts msgs/s MB/s."""
    srv, cli = _exe(server_kind), _exe(client_kind)
    p, q = _ports()
    ep, ack = f"tcp://127.0.0.1:{p}", f"tcp://127.0.0.1:{q}"
    args = [ep, ack, str(n), str(seed), str(heartbeat_ms)]
    pull = subprocess.Popen([srv, "pull"] + args, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    try:
        assert pull.stdout.readline().strip() == "READY"
        push = subprocess.run([cli, "push"] + args, capture_output=True, text=True, timeout=240)
        out, err = pull.communicate(timeout=60)
    finally:
        if pull.poll() is None:
            pull.kill()
            pull.wait()
    assert push.returncode == 0, push.stderr + push.stdout
    assert push.stdout.strip() == f"SENT {n} ACKED"
    assert pull.returncode == 0, err + out
    line = out.strip().splitlines()[-1]
    f = line.split()
    assert f[0] == "OK" and int(f[1]) == n, line
    return {"server": server_kind, "client": client_kind, "messages": n, "parts": int(f[2]),
            "msgs_per_s": float(f[3]), "MB_per_s": float(f[4])}


def _env(**kv):
    e = dict(os.environ)
    e.update(kv)
    return e


def run_pubsub(pub_kind, sub_kind, seed=5, heartbeat_ms=5, pub_zmtp30=False):
    """PUB (CURVE server) as pub_kind, SUB (CURVE client) as sub_kind: the
    SUB's SUBSCRIBE / CANCEL commands cross the two codecs; returns the SUB's
    counts (received, alpha, beta, gamma).  pub_zmtp30: the PUB announces
    ZMTP 3.0 (tests/host/libzmq_test_switches.patch), so the SUB takes
    handshake_v3_0 (src/zmtp_engine.cpp:383-393) and its CURVE mechanism
    encodes subscriptions with downgrade_sub (src/curve_mechanism_base.cpp:
    118-158); the SUB's stderr then carries the patch's trace line, which
    the result reports as "downgraded"."""
    pub, sub = _exe(pub_kind), _exe(sub_kind)
    p, q = _ports()
    args = [f"tcp://127.0.0.1:{p}", f"tcp://127.0.0.1:{q}", "-", str(seed), str(heartbeat_ms)]
    pub_env = _env(ZMQG_TEST_ZMTP30="1") if pub_zmtp30 else None
    pp = subprocess.Popen([pub, "pub"] + args, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                          env=pub_env)
    try:
        assert pp.stdout.readline().strip() == "READY"
        s = subprocess.run([sub, "sub"] + args, capture_output=True, text=True, timeout=120,
                           env=_env(ZMQG_TEST_ZMTP30_TRACE="1"))
        out, err = pp.communicate(timeout=60)
    finally:
        if pp.poll() is None:
            pp.kill()
            pp.wait()
    assert s.returncode == 0, s.stderr + s.stdout
    assert pp.returncode == 0, err + out
    f = s.stdout.strip().split()
    assert f[0] == "OK", s.stdout
    return {"pub": pub_kind, "sub": sub_kind, "received": int(f[1]), "alpha": int(f[2]), "beta": int(f[3]),
            "gamma": int(f[4]), "downgraded": "handshake_v3_0" in s.stderr}


def test_stock_pubsub_subscribe_cancel():
    r = run_pubsub("stock", "stock")
    assert not r["downgraded"]
    print(r)


def test_stock_pubsub_downgraded_subscriptions():
    """The harness for the ZMTP 3.0 cases on the CPU: a stock PUB announcing
    3.0, a stock SUB that takes handshake_v3_0 and sends its subscriptions
    downgraded -- the filter still applies exactly."""
    r = run_pubsub("stock", "stock", pub_zmtp30=True)
    assert r["downgraded"], r
    print(r)


def test_stock_pair_delivers_everything():
    r = run_pair("stock", "stock")
    print(r)


@pytest.mark.gpu
@pytest.mark.parametrize("server,client", [("zmqg", "stock"), ("stock", "zmqg"), ("zmqg", "zmqg")])
def test_gpu_codec_interoperates_with_stock(server, client):
    """Every message arrives byte-exact across the two codecs, in both
    directions of the CURVE roles, with heartbeats on."""
    t0 = time.time()
    r = run_pair(server, client)
    r["wall_s"] = time.time() - t0
    print(r)


@pytest.mark.gpu
@pytest.mark.parametrize("pub,sub", [("stock", "zmqg"), ("zmqg", "stock")])
def test_gpu_codec_subscribe_cancel_interop(pub, sub):
    """SUBSCRIBE / CANCEL commands (msg_t::subscribe / cancel,
    src/curve_mechanism_base.cpp:118-164) encoded by one codec and decoded by
    the other: the PUB applies exactly the SUB's subscriptions -- nothing
    outside them arrives, beta stops after its cancel, gamma starts after its
    subscription.  Interop evidence for the command layouts the golden
    vectors restate (tests/golden/make_golden.py), not an oracle pin."""
    print(run_pubsub(pub, sub))


# --- the batched codec inside the engine ---------

@pytest.mark.gpu
@pytest.mark.parametrize("server,client", [("zmqgb", "stock"), ("stock", "zmqgb"), ("zmqgb", "zmqgb"),
                                           ("zmqgb", "zmqg")])
def test_gpu_batched_codec_interoperates(server, client):
    """The stream engine with the I/O thread's batched GPU codec
    (tests/host/libzmq_zmqg_batched.patch): every message of config 1's
    plan arrives byte-exact, MORE flags included, with heartbeats every 5 ms
    (PING / PONG submitted in order with the messages), both CURVE roles,
    against the stock codec and the per-message GPU codec."""
    t0 = time.time()
    r = run_pair(server, client)
    r["wall_s"] = time.time() - t0
    print(r)


@pytest.mark.gpu
@pytest.mark.parametrize("pub,sub", [("stock", "zmqgb"), ("zmqgb", "stock")])
def test_gpu_batched_subscribe_cancel_interop(pub, sub):
    """SUBSCRIBE / CANCEL through the batched codec in both directions: the
    PUB applies exactly the SUB's subscriptions."""
    r = run_pubsub(pub, sub)
    assert not r["downgraded"]
    print(r)


@pytest.mark.gpu
@pytest.mark.parametrize("pub,sub", [("stock", "zmqg"), ("zmqg", "stock"), ("stock", "zmqgb"),
                                     ("zmqgb", "stock")])
def test_gpu_downgraded_subscriptions_interop(pub, sub):
    """A ZMTP 3.0 PUB (test switch): the SUB runs handshake_v3_0 and its
    CURVE codec encodes SUBSCRIBE / CANCEL with downgrade_sub -- as a
    message whose first byte is 1 / 0 (src/curve_mechanism_base.cpp:118-158)
    -- which the PUB's codec decodes and src/xpub.cpp applies.  With the GPU
    codec on the SUB side the device writes the downgraded layout and the
    stock PUB's libsodium opens it; with the GPU codec on the PUB side it
    opens the stock SUB's.  The filter applies exactly as in the 3.1 cases:
    the downgrade_sub layout crosses the reference codec both ways."""
    r = run_pubsub(pub, sub, pub_zmtp30=True)
    assert r["downgraded"], r
    print(r)
