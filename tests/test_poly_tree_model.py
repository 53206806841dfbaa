"""The parallel Poly1305 of the one-message kernel (libzmq_amd/csrc/
curve_msg.hpp, k_msg): a CPU model of its limb arithmetic -- per-lane Horner
over four 16-byte blocks with the lanes placed at the end of the smallest
power-of-two span of lanes that holds them, log2(span) shuffle levels
h_v = h_v * r^(4*2^s) + h_(v+2^s), the 26-bit-limb multiply of
curve_device.hpp's fe_mul_s with its 32-bit intermediates -- against plain
Poly1305 (RFC 8439 / libsodium 1.0.18) on random keys and block counts.

It also pins the bound the kernel relies on: every fe_mul input limb stays
below 2^27 only because each combine is carried (fe_carry); without it, the
accumulated sums grow past that and fe_mul's last fold (c * 5 in 32 bits)
wraps -- the failure the GPU test caught at a 4,096-byte frame."""
import random

import pytest

M26 = (1 << 26) - 1
P = (1 << 130) - 5


def to_fe(x):
    return [(x >> (26 * i)) & M26 for i in range(5)]


def from_fe(h):
    return sum(h[i] << (26 * i) for i in range(5))


class Wrap(Exception):
    pass


def fe_mul(h, r):
    s = [0] + [r[i] * 5 for i in range(1, 5)]
    d = [h[0] * r[0] + h[1] * s[4] + h[2] * s[3] + h[3] * s[2] + h[4] * s[1],
         h[0] * r[1] + h[1] * r[0] + h[2] * s[4] + h[3] * s[3] + h[4] * s[2],
         h[0] * r[2] + h[1] * r[1] + h[2] * r[0] + h[3] * s[4] + h[4] * s[3],
         h[0] * r[3] + h[1] * r[2] + h[2] * r[1] + h[3] * r[0] + h[4] * s[4],
         h[0] * r[4] + h[1] * r[3] + h[2] * r[2] + h[3] * r[1] + h[4] * r[0]]
    o = [0] * 5
    c = 0
    for i in range(5):
        d[i] += c
        if d[i] >= 1 << 64:
            raise Wrap("u64 product sum")
        c = d[i] >> 26
        o[i] = d[i] & M26
    if c * 5 >= 1 << 32:
        raise Wrap("c * 5")
    o[0] += c * 5
    c = o[0] >> 26
    o[0] &= M26
    o[1] += c
    return o


def fe_carry(h):
    h = list(h)
    for i in range(4):
        c = h[i] >> 26
        h[i] &= M26
        h[i + 1] += c
    c = h[4] >> 26
    h[4] &= M26
    h[0] += c * 5
    c = h[0] >> 26
    h[0] &= M26
    h[1] += c
    return h


def tree_poly(blocks, r, carry=True):
    """H = sum m_k r^(N-k) as k_msg computes it (before the final + s)."""
    n = len(blocks)
    rf = to_fe(r)
    nl = (n + 3) // 4
    pad = 4 * nl - n
    levels = 0
    while (1 << levels) < nl:
        levels += 1
    span = 1 << levels  # the lanes right-aligned in the smallest power-of-two span
    hs = []
    for lane in range(64):
        seg = lane - (span - nl)
        h = [0] * 5
        if seg >= 0 and lane < span:
            for t in range(4):
                k = 4 * seg + t - pad
                if k >= 0:
                    m = to_fe(blocks[k] & ((1 << 128) - 1))
                    m[4] += blocks[k] >> 128 << 24  # the 2^128 pad bit of a full block
                    h = fe_mul([h[i] + m[i] for i in range(5)], rf)
        hs.append(h)
    p = fe_mul(fe_mul(rf, rf), fe_mul(rf, rf))
    for s in range(levels):
        for v in range(0, 64, 2 << s):
            h = fe_mul(hs[v], p)
            h = [h[i] + hs[v + (1 << s)][i] for i in range(5)]
            hs[v] = fe_carry(h) if carry else h
        if s + 1 < levels:
            p = fe_mul(p, p)
    return from_fe(hs[0]) % P


def horner(blocks, r):
    h = 0
    for m in blocks:
        h = (h + m) * r % P
    return h


@pytest.mark.parametrize("seed", range(4))
def test_tree_equals_horner(seed):
    rnd = random.Random(seed)
    for _ in range(150):
        r = rnd.getrandbits(128) & 0x0ffffffc0ffffffc0ffffffc0fffffff
        n = rnd.choice([1, 2, 3, 4, 5, 63, 64, 65, 128, 129, 200, 249, 252, 253, 254])
        blocks = [rnd.getrandbits(128) | (1 << 128) for _ in range(n)]
        assert tree_poly(blocks, r) == horner(blocks, r)


def test_without_carry_the_fold_wraps():
    rnd = random.Random(99)
    wrapped = 0
    for _ in range(300):
        r = rnd.getrandbits(128) & 0x0ffffffc0ffffffc0ffffffc0fffffff
        blocks = [rnd.getrandbits(128) | (1 << 128) for _ in range(254)]
        try:
            tree_poly(blocks, r, carry=False)
        except Wrap:
            wrapped += 1
    assert wrapped > 0


def _dpp(vals, ctrl, rows, ident):
    """One DPP move over a wave of 64 values: row_shr:d (0x110 + d, lane u
    reads u-d of its row of 16), row_bcast:15 (0x142, lane 15 of each row to
    the next row) and row_bcast:31 (0x143, lane 31 to rows 2 and 3); lanes
    outside the row mask or without a source lane get ident."""
    out = []
    for u in range(64):
        row = u >> 4
        src = None
        if (rows >> row) & 1:
            if 0x111 <= ctrl <= 0x11f:
                d = ctrl - 0x110
                if (u & 15) >= d:
                    src = u - d
            elif ctrl == 0x142 and row > 0:
                src = 16 * row - 1
            elif ctrl == 0x143 and row > 1:
                src = 31
        out.append(vals[src] if src is not None else ident)
    return out


def prefix_poly(blocks, r):
    """H = sum m_k r^(N-k) as k_msg computes it (before + s): c = ceil(N/64)
    blocks per lane (Horner) over nl = ceil(N/c) groups, group g on lane
    nl-1-g, the first group padded by zero blocks in front; lane u's Horner
    value times x^u (x = r^c) from an inclusive DPP prefix product over the
    lanes (one on lane 0, x elsewhere; row_shr 1, 2, 4, 8, row_bcast 15, 31,
    as many levels as nl needs), then the sum over the lanes: uncarried
    32-bit row sums (checked below 2^32), the four rows added and folded."""
    n = len(blocks)
    rf = to_fe(r)
    c = (n + 63) // 64
    nl = (n + c - 1) // c
    pad = c * nl - n
    levels = 0
    while (1 << levels) < nl:
        levels += 1
    hs = []
    for u in range(64):
        h = [0] * 5
        if u < nl:
            g = nl - 1 - u
            for t in range(c):
                k = c * g + t - pad
                if k >= 0:
                    m = to_fe(blocks[k] & ((1 << 128) - 1))
                    m[4] += blocks[k] >> 128 << 24
                    h = fe_mul([h[i] + m[i] for i in range(5)], rf)
        hs.append(h)
    if levels == 0:
        return from_fe(hs[0]) % P
    r2 = fe_mul(rf, rf)
    x = [rf, r2, fe_mul(r2, rf), fe_mul(r2, r2)][c - 1]
    one = [1, 0, 0, 0, 0]
    pw = [one if u == 0 else x for u in range(64)]
    steps = [(0x111, 0xf), (0x112, 0xf), (0x114, 0xf), (0x118, 0xf), (0x142, 0xa), (0x143, 0xc)]
    for ctrl, rows in steps[:levels]:
        limbs = [_dpp([pw[u][i] for u in range(64)], ctrl, rows, 1 if i == 0 else 0) for i in range(5)]
        pw = [fe_mul(pw[u], [limbs[i][u] for i in range(5)]) for u in range(64)]
    terms = [fe_mul(hs[u], pw[u]) for u in range(64)]
    wide = [0] * 5
    for i in range(5):
        for row in range(4):
            rs = sum(terms[u][i] for u in range(16 * row, 16 * row + 16))
            assert rs < 1 << 31  # the 32-bit DPP row sums cannot wrap
            wide[i] += rs
    return from_fe(wide) % P


def test_dpp_prefix_is_the_power_of_x():
    # the DPP steps give lane u the product of lanes 0..u (x^u here)
    vals = list(range(64))
    steps = [(0x111, 0xf), (0x112, 0xf), (0x114, 0xf), (0x118, 0xf), (0x142, 0xa), (0x143, 0xc)]
    for ctrl, rows in steps:
        o = _dpp(vals, ctrl, rows, 0)
        vals = [vals[u] + o[u] for u in range(64)]
    assert vals == [u * (u + 1) // 2 for u in range(64)]


@pytest.mark.parametrize("seed", range(4))
def test_prefix_equals_horner(seed):
    rnd = random.Random(100 + seed)
    for _ in range(150):
        r = rnd.getrandbits(128) & 0x0ffffffc0ffffffc0ffffffc0fffffff
        n = rnd.choice([1, 2, 3, 4, 5, 16, 17, 31, 32, 33, 63, 64, 65, 66, 128, 129, 130, 192, 193, 200, 249,
                          252, 253, 254])
        blocks = [rnd.getrandbits(128) | (1 << 128) for _ in range(n)]
        assert prefix_poly(blocks, r) == horner(blocks, r)
