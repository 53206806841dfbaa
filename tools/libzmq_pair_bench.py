"""CURVE PUSH/PULL message rate of the libzmq builds of tests/host/build_libzmq.sh
(config 1 over tcp://127.0.0.1, the plan of tests/host/test_curve_interop.cpp:
1 KiB messages plus the 0 B / 33 B / 64 B / 64 KiB and three-part ones, every
byte checked, heartbeats every 5 ms), pairings run back to back on one box.

    python tools/libzmq_pair_bench.py [--reps R] [--messages N] [--pairs stock:stock,zmqgb:zmqgb]

Prints one JSON object: per pairing the receiver's msg/s of every repetition,
their median, and (INTEROP_THREAD_CPU) the CPU seconds of each thread over the
timed window on both sides.  bench.py's host_paths.libzmq_pairs calls run()."""
import argparse
import json
import os
import socket
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "host", "_ref", "libzmq")


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


def _cpu(text):
    out = {}
    for line in text.splitlines():
        f = line.split()
        if len(f) >= 6 and f[0] == "cpu":   # cpu <thread name> <s> of <wall> s
            out[" ".join(f[1:-4])] = float(f[-4])
    return out


def _stats(text):
    return [line for line in text.splitlines() if line.startswith("zmqg engine:")]


def run_pair(server, client, n=100000, seed=11, heartbeat_ms=5, timeout=240):
    """One run: PULL (CURVE server) built as `server`, PUSH (CURVE client) as
    `client`.  Returns msgs_per_s, MB_per_s and the per-thread CPU split."""
    srv, cli = os.path.join(BIN, "interop_" + server), os.path.join(BIN, "interop_" + client)
    p, q = _ports()
    args = [f"tcp://127.0.0.1:{p}", f"tcp://127.0.0.1:{q}", str(n), str(seed), str(heartbeat_ms)]
    env = dict(os.environ, INTEROP_THREAD_CPU="1", ZMQG_ENGINE_STATS="1")
    pull = subprocess.Popen([srv, "pull"] + args, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env)
    try:
        if pull.stdout.readline().strip() != "READY":
            raise RuntimeError("receiver did not start")
        push = subprocess.run([cli, "push"] + args, capture_output=True, text=True, timeout=timeout, env=env)
        out, err = pull.communicate(timeout=60)
    finally:
        if pull.poll() is None:
            pull.kill()
            pull.wait()
    if push.returncode != 0 or pull.returncode != 0:
        raise RuntimeError(f"{server}/{client}: push rc {push.returncode} {push.stderr[-300:]} "
                           f"pull rc {pull.returncode} {err[-300:]}")
    f = out.strip().splitlines()[-1].split()
    if f[0] != "OK" or int(f[1]) != n:
        raise RuntimeError(f"{server}/{client}: {out[-200:]}")
    return {"msgs_per_s": float(f[3]), "MB_per_s": float(f[4]), "cpu_receiver": _cpu(err),
            "cpu_sender": _cpu(push.stderr),
            "engine_receiver": _stats(err), "engine_sender": _stats(push.stderr)}


def run(pairs=(("stock", "stock"), ("zmqgb", "zmqgb")), reps=5, n=100000):
    res = {}
    for rep in range(reps):
        for s, c in pairs:   # interleaved, so a slow phase of the box hits every pairing
            r = run_pair(s, c, n)
            e = res.setdefault(f"{s}/{c}", {"server": s, "client": c, "messages": n, "msgs_per_s": [],
                                             "cpu": []})
            e["msgs_per_s"].append(r["msgs_per_s"])
            e["cpu"].append({"receiver": r["cpu_receiver"], "sender": r["cpu_sender"],
                             "engine_receiver": r["engine_receiver"], "engine_sender": r["engine_sender"]})
    for e in res.values():
        e["median_msgs_per_s"] = statistics.median(e["msgs_per_s"])
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--messages", type=int, default=100000)
    ap.add_argument("--pairs", default="stock:stock,zmqgb:zmqgb,zmqgb:stock,stock:zmqgb")
    a = ap.parse_args()
    pairs = [tuple(p.split(":")) for p in a.pairs.split(",")]
    print(json.dumps(run(pairs, a.reps, a.messages)))
    sys.stdout.flush()


if __name__ == "__main__":
    main()
