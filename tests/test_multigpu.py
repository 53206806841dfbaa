"""Multi-rank path on CPU: world_size 2 over gloo.

Each rank takes a contiguous, block-balanced slice of one batch
(libzmq_amd.shard.partition), exchanges only its per-session maxima of
header-valid nonces (all_gather), starts its sessions from the exclusive
max-scan over ranks, and decodes its slice -- here with the CPU oracle in
place of the GPU (the kernels are covered by the -m gpu tests; this covers
the sharding logic and the collective).  The gathered result must equal a
single-rank sequential decode of the whole batch, bit for bit, replays that
straddle the rank boundary included.
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from libzmq_amd import shard
from oracle import oracle as O
from tests.helpers import pack, random_batch, wire_layout

ERR_INVALID_SEQUENCE = 0x10000002  # ZMQ_PROTOCOL_ERROR_ZMTP_INVALID_SEQUENCE, include/zmq.h:427


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batch(seed, n, S):
    """An adversarial decode batch over S sessions: the wire frames of a
    random encode, with replays of earlier frames and tampered copies mixed
    in (so some replays land on the other rank's side of the split)."""
    rng = np.random.default_rng(seed)
    precoms = [rng.integers(0, 256, 32, dtype=np.uint8).tobytes() for _ in range(S)]
    b = random_batch(rng, n, [0, 17, 64, 300, 1500], S)
    out_off, wl, total = wire_layout(b["flags"], b["lens"], [False] * S, b["sid"])
    enc = O.make_sessions(precoms)
    wire = O.encode_batch(enc, b["sid"], b["nonce"], b["flags"], b["in_off"], b["lens"], b["inp"], out_off, total)
    frames = [wire[int(out_off[i]):int(out_off[i]) + int(wl[i])].tobytes() for i in range(n)]
    stream, sids = [], []
    for i in range(n):
        stream.append(frames[i])
        sids.append(int(b["sid"][i]))
        r = rng.random()
        if r < 0.12:
            j = int(rng.integers(0, n))  # an earlier or a later frame of any session
            stream.append(frames[j])
            sids.append(int(b["sid"][j]))
        elif r < 0.16:
            f = bytearray(frames[i])
            f[-1] ^= 0x10
            stream.append(bytes(f))
            sids.append(int(b["sid"][i]))
    inp, in_off = pack(stream)
    wls = np.array([len(f) for f in stream], np.uint32)
    plen = np.maximum(wls.astype(np.int64) - 33, 0)
    _, pout = pack([b"\0" * int(p) for p in plen])
    psize = int(pout[-1]) + int(plen[-1]) + 1
    dec = np.concatenate([O.make_sessions([p], dec_prefix=O.CLIENT_PREFIX) for p in precoms])
    return dict(dec=dec, sid=np.array(sids, np.uint32), in_off=in_off, wls=wls, inp=inp, pout=pout, psize=psize,
                plen=plen, S=S)


def _rank_main(rank, world, port, seed, n, S, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        B = _batch(seed, n, S)
        N = len(B["sid"])
        lo, hi = shard.partition(shard.stream_blocks(B["wls"]), world)[rank]
        # per-session maxima of this slice's header-valid nonces -> all ranks
        vn = shard.header_nonces(B["inp"], B["in_off"][lo:hi], B["wls"][lo:hi])
        mine = shard.session_max(B["sid"][lo:hi], vn, S)
        allmax = shard.gather_session_max(mine)
        peer0 = np.full(S, 2, np.uint64)
        peer = shard.peer_prefix(allmax, peer0, rank)
        # decode this slice (the oracle stands in for the device)
        pl, fl, st = O.decode_batch(B["dec"], peer, B["sid"][lo:hi], B["in_off"][lo:hi], B["wls"][lo:hi], B["inp"],
                                    B["pout"][lo:hi], B["psize"])
        # the new peer nonces: max over ranks
        newpeer = allmax.max(axis=0)
        newpeer = np.maximum(newpeer, peer0)
        spans = [(int(B["pout"][i]), int(B["plen"][i])) for i in range(lo, hi)]
        payload = b"".join(pl[o:o + ln].tobytes() for o, ln in spans)
        t = shard.max_over_ranks(float(rank + 1))
        out = [None] * world
        dist.all_gather_object(out, dict(rank=rank, lo=lo, hi=hi, st=st.tolist(), fl=fl.tolist(), payload=payload,
                                         peer=peer.tolist(), newpeer=newpeer.tolist(), t=t, N=N))
        if rank == 0:
            q.put(out)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("S", [1, 3])
def test_sharded_decode_world2_equals_sequential(S):
    seed, n, world = 11 + S, 240, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, seed, n, S, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=240)
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
    assert (rst == ERR_INVALID_SEQUENCE).any()
    # a replay whose original sits on rank 0 is rejected on rank 1
    lo1 = res[1]["lo"]
    assert (rst[lo1:] == ERR_INVALID_SEQUENCE).any()
    assert np.array_equal(fl, rfl)
    payload = b"".join(d["payload"] for d in res)
    ref = b"".join(rpl[int(B["pout"][i]):int(B["pout"][i]) + int(B["plen"][i])].tobytes() for i in range(len(B["sid"])))
    assert payload == ref
    assert res[0]["newpeer"] == res[1]["newpeer"] == [int(x) for x in peer]
    assert res[0]["t"] == res[1]["t"] == 2.0  # max over ranks


def test_partition_balances_salsa20_blocks():
    rng = np.random.default_rng(5)
    sizes = rng.choice([64 + 33, 1024 + 33, 65536 + 33], 5000)
    w = shard.stream_blocks(sizes)
    for world in (1, 2, 4, 8):
        parts = shard.partition(w, world)
        assert parts[0][0] == 0 and parts[-1][1] == len(w)
        assert all(parts[r][1] == parts[r + 1][0] for r in range(world - 1))
        loads = [int(w[a:b].sum()) for a, b in parts]
        ideal = int(w.sum()) / world  # every cut lies within half a frame of its target
        assert all(abs(x - ideal) <= int(w.max()) for x in loads)


def test_header_nonces_follow_check_validity():
    good = b"\x07MESSAGE" + (1234).to_bytes(8, "big") + bytes(16) + b"\x00"
    frames = [good, good[:32], b"\x08MESSAGE" + good[8:], good + b"xyz", b"\x40" + good[1:]]
    inp, off = pack(frames)
    wl = np.array([len(f) for f in frames], np.uint32)
    v = shard.header_nonces(inp, off, wl)
    assert list(v) == [1234, 0, 0, 1234, 0]


def test_header_nonces_vectorised_matches_rule():
    """shard.header_nonces (vectorised) against the header rule written as a
    per-frame loop: size >= 33, size > data[0] (mechanism_base.cpp:14-25),
    "\\x07MESSAGE" prefix (curve_mechanism_base.cpp:85-90), BE nonce."""
    rng = np.random.default_rng(11)
    frames = []
    for _ in range(400):
        f = bytearray(rng.integers(0, 256, int(rng.integers(0, 90)), dtype=np.uint8).tobytes())
        if len(f) >= 8 and rng.random() < 0.7:
            f[:8] = b"\x07MESSAGE"
        frames.append(bytes(f))
    inp, in_off = pack(frames)
    wl = np.array([len(f) for f in frames], np.int64)
    got = shard.header_nonces(inp, in_off, wl)
    exp = [0 if len(f) < 33 or len(f) <= f[0] or f[:8] != b"\x07MESSAGE" else int.from_bytes(f[8:16], "big")
           for f in frames]
    assert np.array_equal(got, np.array(exp, np.uint64))
    assert (got != 0).sum() > 50
