"""bench.py --gpus 2 on the GPU box: the launcher starts two ranks (torchrun,
127.0.0.1), each rank runs the config-2 step on its GPU -- ranks share a
device when the box has fewer GPUs than ranks -- config 5 splits one batch
over the ranks with shard.partition (strong scaling, sum over ranks), and
rank 0 prints exactly one line, with n_gpus = the distinct devices used
(1 on a one-GPU box, with shared_devices) and max-over-ranks timing.
The multi-process path the driver's 8-GPU scaling run takes, on real
kernels rather than the gloo tests' CPU stand-ins."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_config2_and_strong_config5():
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "2", "--warmup", "1",
                        "--no-cpu-baseline", "--no-host-staged", "--configs", "5"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith('{"metric"')]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    # n_gpus counts distinct devices: two ranks on a one-GPU box must not
    # claim two GPUs
    import torch
    ndev = torch.cuda.device_count()
    assert d["ranks"] == 2 and d["n_gpus"] == min(2, ndev) and d["shared_devices"] == (ndev < 2)
    assert d["steps"] == 2 and d["scaling"] == "weak"
    assert d["config"]["parallelism"].startswith("frame-sharded x2")
    assert d["value"] > 0 and d["msgs_per_s"] > 0
    c5 = d["configs"]["config5"]
    assert c5["scaling"] == "strong" and c5["frames_per_gpu"] == 512 and c5["value"] > 0


def _rank_device(rank, world, port, seed, n, S, q):
    """One rank of the sharded decode on the device: its slice's session
    maxima from zmqg_session_max_batch, all_gather over gloo, the exclusive
    max-scan as the sessions' starting peer nonces, the slice decoded by the
    frame kernels (ranks share the GPU when the box has one)."""
    import numpy as np
    import torch
    import torch.distributed as dist

    from libzmq_amd import curve as C
    from libzmq_amd import shard
    from tests.test_multigpu import _batch

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda", rank % torch.cuda.device_count())
        torch.cuda.set_device(dev)
        B = _batch(seed, n, S)
        lo, hi = shard.partition(shard.stream_blocks(B["wls"]), world)[rank]
        t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a).view(dt).copy()).to(dev)
        wire = t(B["inp"], np.uint8)
        sid, in_off, wl = t(B["sid"][lo:hi], np.int32), t(B["in_off"][lo:hi], np.int64), t(B["wls"][lo:hi], np.int32)
        pout = t(B["pout"][lo:hi], np.int64)
        rng = np.random.default_rng(seed)
        precoms = [rng.integers(0, 256, 32, dtype=np.uint8).tobytes() for _ in range(S)]
        dec = C.CurveContext(dev.index, S)
        for s in range(S):
            dec.session_set(s, precoms[s], C.SERVER_PREFIX, C.CLIENT_PREFIX, False, 2)
        mine = shard.session_max_device(dec, sid, in_off, wl, wire, S)
        allmax = shard.gather_session_max(mine)
        peer = shard.peer_prefix(allmax, np.full(S, 2, np.uint64), rank)
        for s in range(S):
            dec.set_peer_nonce(s, int(peer[s]))
        out = torch.zeros(B["psize"], dtype=torch.uint8, device=dev)
        fl = torch.zeros(hi - lo, dtype=torch.uint8, device=dev)
        st = torch.zeros(hi - lo, dtype=torch.int32, device=dev)
        dec.decode_batch(sid, in_off, wl, wire, pout, out, fl, st)
        torch.cuda.synchronize(dev)
        o = out.cpu().numpy()
        payload = b"".join(o[int(B["pout"][i]):int(B["pout"][i]) + int(B["plen"][i])].tobytes()
                           for i in range(lo, hi) if int(st[i - lo]) == 0)
        res = [None] * world
        dist.all_gather_object(res, dict(rank=rank, lo=lo, hi=hi, st=st.cpu().numpy().tolist(),
                                         fl=fl.cpu().numpy().tolist(), payload=payload,
                                         peer_after=[dec.get_peer_nonce(s) for s in range(S)]))
        if rank == 0:
            q.put(res)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("S", [1, 3])
def test_sharded_decode_world2_on_device(S):
    """SURVEY §8e on real kernels: two ranks (processes) each decode their
    slice of one adversarial batch (replays across the cut, tampering) on the
    GPU, exchanging only per-session nonce maxima; the union equals the
    oracle's sequential decode of the whole batch, and each session's final
    peer nonce on the last rank equals the sequential one."""
    import socket

    import numpy as np
    import torch.multiprocessing as mp

    from oracle import oracle as O
    from tests.test_multigpu import _batch

    seed, n, world = 31 + S, 400, 2
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank_device, args=(r, world, port, seed, n, S, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=200)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    B = _batch(seed, n, S)
    peer = np.full(S, 2, np.uint64)
    rpl, rfl, rst = O.decode_batch(B["dec"], peer, B["sid"], B["in_off"], B["wls"], B["inp"], B["pout"], B["psize"])
    res.sort(key=lambda d: d["rank"])
    assert res[0]["lo"] == 0 and res[-1]["hi"] == len(B["sid"]) and res[0]["hi"] == res[1]["lo"]
    st = np.concatenate([np.array(d["st"], np.int32) for d in res])
    fl = np.concatenate([np.array(d["fl"], np.uint8) for d in res])
    assert np.array_equal(st, rst)
    assert (rst[res[1]["lo"]:] == 0x10000002).any()  # a replay across the cut, rejected on rank 1
    assert np.array_equal(fl, rfl)
    ref = b"".join(rpl[int(B["pout"][i]):int(B["pout"][i]) + int(B["plen"][i])].tobytes()
                   for i in range(len(B["sid"])) if rst[i] == 0)
    assert b"".join(d["payload"] for d in res) == ref
    assert res[1]["peer_after"] == [int(x) for x in peer]
