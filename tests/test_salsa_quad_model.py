"""CPU model of k_msg's quad-lane Salsa20 (libzmq_amd/csrc/curve_msg.hpp,
salsa20_quad): lane q of a quad holds column q's quarter-round
(x[5q], x[5q+4], x[5q+8], x[5q+12], indices mod 16); before each row round
the row's b, c, d come from lanes q+1, q+2, q+3 as their d, c, b (three quad
permutations), and the inverse permutations restore the column layout.  The
model checks that this equals the Salsa20 core's 20 rounds (ten double
rounds, each a column round then a row round)."""
import random

M = 0xFFFFFFFF
NEXT, HALF, PREV = [1, 2, 3, 0], [2, 3, 0, 1], [3, 0, 1, 2]  # quad_perm 0x39 / 0x4e / 0x93


def _rotl(x, n):
    return ((x << n) | (x >> (32 - n))) & M


def _qr(a, b, c, d):
    b ^= _rotl((a + d) & M, 7)
    c ^= _rotl((b + a) & M, 9)
    d ^= _rotl((c + b) & M, 13)
    a ^= _rotl((d + c) & M, 18)
    return a, b, c, d


def _salsa_rounds(x):
    x = list(x)
    for _ in range(10):
        for i, j, k, l in ((0, 4, 8, 12), (5, 9, 13, 1), (10, 14, 2, 6), (15, 3, 7, 11)):
            x[i], x[j], x[k], x[l] = _qr(x[i], x[j], x[k], x[l])
        for i, j, k, l in ((0, 1, 2, 3), (5, 6, 7, 4), (10, 11, 8, 9), (15, 12, 13, 14)):
            x[i], x[j], x[k], x[l] = _qr(x[i], x[j], x[k], x[l])
    return x


def _perm(v, p):
    return [v[p[i]] for i in range(4)]


def _quad_rounds(x):
    a = [x[(5 * q) % 16] for q in range(4)]
    b = [x[(5 * q + 4) % 16] for q in range(4)]
    c = [x[(5 * q + 8) % 16] for q in range(4)]
    d = [x[(5 * q + 12) % 16] for q in range(4)]
    for _ in range(10):
        for q in range(4):
            a[q], b[q], c[q], d[q] = _qr(a[q], b[q], c[q], d[q])
        rb, rc, rd = _perm(d, NEXT), _perm(c, HALF), _perm(b, PREV)
        for q in range(4):
            a[q], rb[q], rc[q], rd[q] = _qr(a[q], rb[q], rc[q], rd[q])
        d, c, b = _perm(rb, PREV), _perm(rc, HALF), _perm(rd, NEXT)
    out = [0] * 16
    for q in range(4):
        out[(5 * q) % 16], out[(5 * q + 4) % 16] = a[q], b[q]
        out[(5 * q + 8) % 16], out[(5 * q + 12) % 16] = c[q], d[q]
    return out


def test_quad_layout_equals_salsa20_rounds():
    rng = random.Random(7)
    for _ in range(64):
        x = [rng.getrandbits(32) for _ in range(16)]
        assert _quad_rounds(x) == _salsa_rounds(x)


def test_poly_key_words_come_from_lanes_0_to_3():
    # k_msg reads keystream words 0..7 of block 0 with readlane: word w sits
    # in lane q, register (a, b, c, d)[k] where w = 5q + 4k (mod 16)
    where = {}
    for q in range(4):
        for k, reg in enumerate("abcd"):
            where[(5 * q + 4 * k) % 16] = (q, reg)
    assert [where[w] for w in range(8)] == [(0, "a"), (1, "d"), (2, "c"), (3, "b"), (0, "b"), (1, "a"), (2, "d"),
                                            (3, "c")]
