"""CPU model of the frame kernels' DPP wave reductions
(libzmq_amd/csrc/curve_frames.hpp: wave_scan_max_u64, wave_prev_u64,
wave_max_u64, wave_max_u32): the decode replay rule's inclusive and exclusive
prefix maxima of the header-valid nonces over a wave's 64 frames, and the
wave maxima of the window counts and frame ends.  DPP semantics as in
tests/test_poly_tree_model.py: row_shr:d reads lane u-d of the row of 16,
row_bcast:15 / :31 broadcast lane 15 of each row to the next row / lane 31 to
rows 2 and 3 (row masks 0xa / 0xc), wave_shr:1 reads lane u-1; a lane with
no source, or outside the row mask, reads 0 (bound_ctrl, `old` = 0)."""
import random


def dpp(vals, ctrl, rows=0xF):
    out = []
    for u in range(64):
        row, src = u >> 4, None
        if (rows >> row) & 1:
            if 0x111 <= ctrl <= 0x11F and (u & 15) >= ctrl - 0x110:
                src = u - (ctrl - 0x110)
            elif ctrl == 0x142 and row > 0:
                src = 16 * row - 1
            elif ctrl == 0x143 and row > 1:
                src = 31
            elif ctrl == 0x138 and u > 0:
                src = u - 1
        out.append(vals[src] if src is not None else 0)
    return out


def wave_scan_max(v):
    for ctrl, rows in ((0x111, 0xF), (0x112, 0xF), (0x114, 0xF), (0x118, 0xF), (0x142, 0xA), (0x143, 0xC)):
        o = dpp(v, ctrl, rows)
        v = [max(a, b) for a, b in zip(v, o)]
    return v


def wave_max(v):
    for ctrl in (0x111, 0x112, 0x114, 0x118):
        o = dpp(v, ctrl)
        v = [max(a, b) for a, b in zip(v, o)]
    return max(v[15], v[31], v[47], v[63])


def test_scan_prev_and_max_match_the_definitions():
    rng = random.Random(5)
    for trial in range(300):
        kind = trial % 3
        if kind == 0:
            v = [rng.getrandbits(64) for _ in range(64)]
        elif kind == 1:  # nonces of a batch: increasing with replays and header failures (0)
            base = rng.getrandbits(40)
            v = [0 if rng.random() < 0.1 else base + i + rng.choice([0, 0, 0, -3, 5]) for i in range(64)]
        else:
            v = [rng.choice([0, 1, 2, 17, 72]) for _ in range(64)]
        inc = wave_scan_max(v)
        assert inc == [max(v[:u + 1]) for u in range(64)]
        assert dpp(inc, 0x138) == [0] + [max(v[:u]) for u in range(1, 64)]
        assert wave_max(v) == max(v)
