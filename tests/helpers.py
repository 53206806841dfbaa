"""Shared batch builders for the parity tests (test infrastructure)."""
import numpy as np

from oracle import oracle as O


def pack(chunks, rng=None, max_gap=0, base_gap=0):
    """Concatenate byte arrays with optional random gaps (to vary alignment).
    Returns (buffer, offsets)."""
    offs = []
    pos = base_gap
    for c in chunks:
        if rng is not None and max_gap:
            pos += int(rng.integers(0, max_gap + 1))
        offs.append(pos)
        pos += len(c)
    buf = np.zeros(max(pos, 1), np.uint8)
    for o, c in zip(offs, chunks):
        if len(c):
            buf[o:o + len(c)] = np.frombuffer(bytes(c), np.uint8)
    return buf, np.array(offs, np.uint64)


def random_batch(rng, n, sizes, n_sessions, flag_choices=(0, 1), nonce_start=3, max_gap=0):
    """Random frames: returns dict with payload buffer and descriptors."""
    lens = np.array([int(rng.choice(sizes)) for _ in range(n)], np.uint32)
    sid = rng.integers(0, n_sessions, n).astype(np.uint32)
    flags = np.array([int(rng.choice(flag_choices)) for _ in range(n)], np.uint8)
    payloads = [rng.integers(0, 256, int(l), dtype=np.uint8).tobytes() for l in lens]
    inp, in_off = pack(payloads, rng, max_gap)
    nonce = np.zeros(n, np.uint64)
    nxt = {}
    for i in range(n):
        s = int(sid[i])
        nonce[i] = nxt.get(s, nonce_start)
        nxt[s] = int(nonce[i]) + 1
    return dict(n=n, lens=lens, sid=sid, flags=flags, payloads=payloads, inp=inp, in_off=in_off, nonce=nonce)


def wire_layout(flags, lens, downgrade, sid, rng=None, max_gap=0):
    sizes = [O.wire_size(int(f), int(downgrade[int(s)]), int(l)) for f, l, s in zip(flags, lens, sid)]
    offs = []
    pos = 0
    for s in sizes:
        if rng is not None and max_gap:
            pos += int(rng.integers(0, max_gap + 1))
        offs.append(pos)
        pos += s
    return np.array(offs, np.uint64), np.array(sizes, np.uint32), pos
