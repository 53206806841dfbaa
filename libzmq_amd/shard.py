"""Multi-GPU sharding of CURVE MESSAGE batches.

The path shards by frame: every frame is an independent AEAD under its own
nonce, so encode needs no exchange at all.  The only cross-frame state is a
session's replay counter on decode (_cn_peer_nonce,
src/curve_mechanism_base.cpp:98-106): a frame passes iff its nonce exceeds
the peer nonce, which is the maximum of the session's value before the batch
and every earlier header-valid nonce of the session in batch order.  When a
session's frames span ranks, rank r must start from

    peer_r[s] = max(peer_before[s], max header-valid nonce of s on ranks < r)

-- an exclusive max-scan over ranks of one small per-session vector, the only
collective of the path (all_gather of sessions x 8 bytes).  When every
session lives on one rank (the bench's layout: each rank owns its sessions)
the prefix is the identity and there is no collective at all.

Batches are split into contiguous frame ranges balanced by Salsa20 block
count (the VALU work), so mixed sizes land evenly.  The timing aggregate of
a run is the maximum over ranks.
"""
import numpy as np

MESSAGE_HDR = b"\x07MESSAGE"  # src/curve_mechanism_base.cpp:85-90


def stream_blocks(stream_len):
    """Salsa20 blocks (64 keystream bytes) per frame for stream lengths 32 + plaintext."""
    return (np.asarray(stream_len, np.int64) + 63) // 64


def partition(weights, world):
    """Contiguous frame ranges [(start, end)] per rank with about equal total weight."""
    w = np.asarray(weights, np.int64)
    n = len(w)
    if world < 1:
        raise ValueError("world must be >= 1")
    c = np.cumsum(w)
    total = int(c[-1]) if n else 0
    bounds = [0]
    for r in range(1, world):
        target = total * r / world
        if total:
            # the frame crossing the target goes to whichever side keeps the
            # cut nearer the target
            k = min(int(np.searchsorted(c, target, side="left")), n - 1)
            below = int(c[k - 1]) if k > 0 else 0
            b = k + 1 if int(c[k]) - target <= target - below else k
        else:
            b = (n * r) // world
        bounds.append(min(max(b, bounds[-1]), n))
    bounds.append(n)
    return [(bounds[r], bounds[r + 1]) for r in range(world)]


def header_nonces(wire, in_off, wire_len):
    """Header-valid nonce of each wire frame (0 where the header fails), the
    value the replay rule compares: check_basic_command_structure
    (src/mechanism_base.cpp:14-25), "\\x07MESSAGE" and size >= 33
    (src/curve_mechanism_base.cpp:80-97), nonce = big-endian bytes 8..15.
    Host arrays, vectorised (a gather of 16 bytes per frame); on the device
    the same values come from CurveContext.session_max_batch /
    decode_batch(session_max_out=...) (include/zmqg_curve.h)."""
    buf = np.asarray(wire, np.uint8)
    off = np.asarray(in_off, np.int64)
    wl = np.asarray(wire_len, np.int64)
    out = np.zeros(len(off), np.uint64)
    if len(off) == 0:
        return out
    ok = wl >= 33
    idx = np.minimum(off[:, None] + np.arange(16)[None, :], max(len(buf) - 1, 0))
    h = buf[idx]  # [n, 16]; rows of frames shorter than 33 bytes are ignored below
    ok &= wl > h[:, 0]
    ok &= (h[:, :8] == np.frombuffer(MESSAGE_HDR, np.uint8)[None, :]).all(axis=1)
    be = h[:, 8:16].astype(np.uint64)
    v = np.zeros(len(off), np.uint64)
    for k in range(8):  # big-endian bytes 8..15
        v = (v << np.uint64(8)) | be[:, k]
    out[ok] = v[ok]
    return out


def session_max_device(ctx, sid, in_off, wire_len, wire, n_sessions, stream=None):
    """Per-session maxima of header-valid nonces computed on the device
    (zmqg_session_max_batch): device tensors in, a host uint64 vector out."""
    import torch
    m = torch.zeros(n_sessions, dtype=torch.int64, device=wire.device)
    ctx.session_max_batch(sid, in_off, wire_len, wire, m, stream)
    torch.cuda.synchronize(wire.device)
    return m.cpu().numpy().view(np.uint64)


def session_max(sid, nonces, n_sessions):
    """Per-session maximum of header-valid nonces (0 for sessions without frames)."""
    m = np.zeros(n_sessions, np.uint64)
    np.maximum.at(m, np.asarray(sid, np.int64), np.asarray(nonces, np.uint64))
    return m


def peer_prefix(all_session_max, peer_before, rank):
    """Starting peer nonce per session for `rank` from the [world, sessions]
    matrix of per-rank session maxima (the exclusive max-scan over ranks)."""
    m = np.asarray(all_session_max, np.uint64)
    p = np.asarray(peer_before, np.uint64).copy()
    if rank > 0:
        p = np.maximum(p, m[:rank].max(axis=0))
    return p


def gather_session_max(local_max, group=None):
    """all_gather of the per-session maxima (torch.distributed, gloo or RCCL):
    returns the [world, sessions] matrix every rank needs for peer_prefix."""
    import torch
    import torch.distributed as dist

    t = torch.from_numpy(np.ascontiguousarray(local_max).view(np.int64).copy())
    if dist.get_backend(group) == "nccl":
        t = t.cuda()
    parts = [torch.zeros_like(t) for _ in range(dist.get_world_size(group))]
    dist.all_gather(parts, t, group=group)
    return np.stack([p.cpu().numpy().view(np.uint64) for p in parts])


def max_over_ranks(value, group=None):
    """The run's aggregate time: the slowest rank (float, all ranks get it)."""
    import torch
    import torch.distributed as dist

    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())
