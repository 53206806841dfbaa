#!/usr/bin/env python3
"""Generates curve_salsa_asm.hpp: the Salsa20/20 core with a fixed issue
order for gfx950, as inline assembly (round-4 experiment, measured by
tools/salsa_sched.hip and in the library's frame and body kernels: no gain
at any occupancy -- every order issues at ~4 cycles per instruction,
DESIGN.md section 3.1; not in the product).

Why a fixed order.  A Salsa20 step b ^= rotl(a + d, k) is v_add_u32 (VOP2),
v_alignbit_b32 (the rotate, VOP3) and v_xor_b32 (VOP2).  Once two waves
share a SIMD, gfx950 issues VOP2 ops at about twice the rate of the VOP3
rotate (profiles/valu_rates_r02.md), and how well the two waves' streams
fill each other's gaps depends on where the rotates sit in each stream.
The compiler's order runs a quarter-round's twelve ops mostly back to back.
Here the four quarter-rounds of a half-round are four "streams" skewed by
one op against each other (slot t issues op t-j of stream j), so every
group of four consecutive ops holds one or two rotates of independent
chains; row quarter-round j only needs column quarter-rounds j and j-1 (and
the reverse for the next column round), so the skew runs through all 20
rounds without a seam.  One asm statement holds the whole sequence, so
nothing is inserted between the ops.

Hoisting.  In the frame and body kernels a lane's key and nonce are fixed
over many blocks; only the block counter (state word 8) changes.  Every op
whose inputs do not depend on word 8 is computed once by salsa20_hoist()
(plain C, scheduled by the compiler); the per-block asm starts from those
values.  Values are tracked by version, so a hoisted op that overwrites a
word never disturbs a per-block op that reads the word's earlier value.

The generator checks its output by evaluating both the hoisted and the
per-block sequences in Python against a reference Salsa20 on random inputs.

Usage: gen_salsa_asm.py OUT.hpp
"""
import random
import sys

COL = [(0, 4, 8, 12), (5, 9, 13, 1), (10, 14, 2, 6), (15, 3, 7, 11)]
ROW = [(0, 1, 2, 3), (5, 6, 7, 4), (10, 11, 8, 9), (15, 12, 13, 14)]
SIGMA = [0x61707865, 0x3320646e, 0x79622d32, 0x6b206574]
M32 = 0xffffffff


def rotl(x, k):
    return ((x << k) | (x >> (32 - k))) & M32


def ref_block(k, n0, n1, c0, c1):
    x = [SIGMA[0], k[0], k[1], k[2], k[3], SIGMA[1], n0, n1, c0, c1, SIGMA[2], k[4], k[5], k[6], k[7], SIGMA[3]]
    inp = list(x)
    for _ in range(10):
        for qr in COL + ROW:
            a, b, c, d = qr
            x[b] ^= rotl((x[a] + x[d]) & M32, 7)
            x[c] ^= rotl((x[b] + x[a]) & M32, 9)
            x[d] ^= rotl((x[c] + x[b]) & M32, 13)
            x[a] ^= rotl((x[d] + x[c]) & M32, 18)
    return [(x[i] + inp[i]) & M32 for i in range(16)]


class Op:
    """One VALU op on versioned values.  kind: add (dst = s1 + s2), rot
    (dst = rotl(s1, k)), xor (dst = s1 ^ s2).  Values are names: 'w<i>.<v>'
    for version v of state word i, 't<j>.<n>' for stream j's temp n."""
    __slots__ = ("kind", "dst", "s1", "s2", "k", "stream", "static")

    def __init__(self, kind, dst, s1, s2, k, stream):
        self.kind, self.dst, self.s1, self.s2, self.k, self.stream = kind, dst, s1, s2, k, stream
        self.static = False


def build_streams(nrounds=20):
    """The ops of the 4 streams in canonical order (half-round by half-round,
    quarter-round j = stream j), SSA-versioned."""
    ver = [0] * 16
    tcount = [0] * 4
    streams = [[] for _ in range(4)]
    canon = []
    for h in range(nrounds):
        for j in range(4):
            a, b, c, d = (COL if h % 2 == 0 else ROW)[j]
            for (tgt, p, q, k) in ((b, a, d, 7), (c, b, a, 9), (d, c, b, 13), (a, d, c, 18)):
                t0 = f"t{j}.{tcount[j]}"
                t1 = f"t{j}.{tcount[j] + 1}"
                tcount[j] += 2
                ops = [Op("add", t0, f"w{p}.{ver[p]}", f"w{q}.{ver[q]}", 0, j),
                       Op("rot", t1, t0, None, k, j)]
                old = f"w{tgt}.{ver[tgt]}"
                ver[tgt] += 1
                ops.append(Op("xor", f"w{tgt}.{ver[tgt]}", old, t1, 0, j))
                streams[j].extend(ops)
                canon.extend(ops)
    return streams, canon, ver


def classify(canon, dynamic_inputs):
    dyn = set(dynamic_inputs)
    for op in canon:
        srcs = [s for s in (op.s1, op.s2) if s is not None]
        op.static = not any(s in dyn for s in srcs)
        if not op.static:
            dyn.add(op.dst)
    return dyn


def skew_order(streams):
    n = max(len(s) for s in streams)
    out = []
    for t in range(n + len(streams)):
        for j, s in enumerate(streams):
            o = t - j
            if 0 <= o < len(s):
                out.append(s[o])
    return out


def evaluate(ops, env):
    for op in ops:
        if op.kind == "add":
            env[op.dst] = (env[op.s1] + env[op.s2]) & M32
        elif op.kind == "rot":
            env[op.dst] = rotl(env[op.s1], op.k)
        else:
            env[op.dst] = env[op.s1] ^ env[op.s2]
    return env


def init_names(k, n0, n1, c0, c1):
    x = [SIGMA[0], k[0], k[1], k[2], k[3], SIGMA[1], n0, n1, c0, c1, SIGMA[2], k[4], k[5], k[6], k[7], SIGMA[3]]
    return {f"w{i}.0": x[i] for i in range(16)}


C_INIT = ["SIGMA0", "k[0]", "k[1]", "k[2]", "k[3]", "SIGMA1", "n0", "n1", "ctr_lo", "ctr_hi", "SIGMA2",
          "k[4]", "k[5]", "k[6]", "k[7]", "SIGMA3"]


def cname(v):
    return "v_" + v.replace(".", "_")


def gen_variant(fname_hoist, fname_block, hoist, segments=1):
    """hoist=True: word 8 (ctr_lo) is the only per-block input; the rest is
    hoisted.  hoist=False: everything per block (no hoist function)."""
    streams, canon, final_ver = build_streams()
    dyn_inputs = ["w8.0"] if hoist else [f"w{i}.0" for i in range(16)]
    classify(canon, dyn_inputs)
    order = [op for op in skew_order(streams) if not op.static]
    static_ops = [op for op in canon if op.static]
    dyn_vals = {op.dst for op in order}
    # static values read by per-block ops (hoisted inputs of the asm)
    need = []
    for op in order:
        for s in (op.s1, op.s2):
            if s is not None and s not in dyn_vals and s not in need:
                need.append(s)
    hoisted = [v for v in need if v not in dyn_inputs]  # what salsa20_hoist hands over
    hs_index = {v: i for i, v in enumerate(hoisted)}
    finals = [f"w{i}.{final_ver[i]}" for i in range(16)]
    assert all(f in dyn_vals for f in finals), "every output word must be written per block"
    # register assignment inside the asm: a dynamic word version lives in its
    # word's register; a dynamic temp in its stream's temp register
    def reg(v):
        if v in dyn_vals:
            if v.startswith("w"):
                return "%[x" + v[1:v.index(".")] + "]"
            return "%[t" + v[1:v.index(".")] + "]"
        return "%[h" + str(need.index(v)) + "]"
    lines_asm = []
    for op in order:
        if op.kind == "add":
            lines_asm.append(f"v_add_u32 {reg(op.dst)}, {reg(op.s1)}, {reg(op.s2)}")
        elif op.kind == "rot":
            lines_asm.append(f"v_alignbit_b32 {reg(op.dst)}, {reg(op.s1)}, {reg(op.s1)}, {32 - op.k}")
        else:
            lines_asm.append(f"v_xor_b32 {reg(op.dst)}, {reg(op.s1)}, {reg(op.s2)}")
    # consistency: a register must not be overwritten while a later op still
    # needs its old value (within a word / temp register, versions are
    # consumed in order)
    last_use = {}
    for idx, op in enumerate(order):
        for s in (op.s1, op.s2):
            if s is not None:
                last_use[s] = idx
    live = {}
    for idx, op in enumerate(order):
        r = reg(op.dst)
        prev = live.get(r)
        if prev is not None and prev != op.s1 and last_use.get(prev, -1) > idx:
            raise AssertionError(f"register {r} clobbered while {prev} is live")
        if prev is not None and prev == op.s1 and last_use.get(prev, -1) > idx:
            raise AssertionError(f"in-place op on {prev} which is read later")
        live[r] = op.dst

    # Python check against the reference
    rnd = random.Random(1)
    for _ in range(200):
        k = [rnd.getrandbits(32) for _ in range(8)]
        n0, n1, c0, c1 = (rnd.getrandbits(32) for _ in range(4))
        env = init_names(k, n0, n1, c0, c1)
        evaluate(static_ops, env)
        env2 = {v: env[v] for v in need}
        env2.update({f"w{i}.0": env[f"w{i}.0"] for i in range(16) if f"w{i}.0" in dyn_inputs})
        # per-block part: only the hoisted values and the per-block inputs
        evaluate(order, env2)
        x0 = init_names(k, n0, n1, c0, c1)
        got = [(env2[finals[i]] + x0[f"w{i}.0"]) & M32 for i in range(16)]
        assert got == ref_block(k, n0, n1, c0, c1)

    out = []
    nvops = sum(1 for op in order)
    if hoist:
        out.append(f"// {len(static_ops)} of {len(canon)} round ops hoisted (counter-free); "
                   f"{nvops} per block; {len(hoisted)} hoisted values")
        out.append(f"struct SalsaHoist {{\n    uint32_t v[{len(hoisted)}];\n}};")
        body = [f"__device__ __forceinline__ void {fname_hoist}(SalsaHoist &hs, const uint32_t k[8], uint32_t n0, "
                "uint32_t n1, uint32_t ctr_hi)", "{"]
        for i in range(16):
            if i != 8:
                body.append(f"    const uint32_t {cname(f'w{i}.0')} = {C_INIT[i]};")
        for op in static_ops:
            if op.kind == "add":
                e = f"{cname(op.s1)} + {cname(op.s2)}"
            elif op.kind == "rot":
                e = f"__builtin_rotateleft32({cname(op.s1)}, {op.k})"
            else:
                e = f"{cname(op.s1)} ^ {cname(op.s2)}"
            body.append(f"    const uint32_t {cname(op.dst)} = {e};")
        for i, v in enumerate(hoisted):
            body.append(f"    hs.v[{i}] = {cname(v)};")
        body.append("}")
        out.append("\n".join(body))
    params = "(uint32_t out[16], const SalsaHoist &hs, const uint32_t k[8], uint32_t n0, uint32_t n1, " \
             "uint32_t ctr_lo, uint32_t ctr_hi)" if hoist else \
             "(uint32_t out[16], const uint32_t k[8], uint32_t n0, uint32_t n1, uint32_t ctr_lo, uint32_t ctr_hi)"
    body = [f"__device__ __forceinline__ void {fname_block}{params}", "{"]
    if not hoist:
        body.append("    const uint32_t init[16] = {SIGMA0, k[0], k[1], k[2], k[3], SIGMA1, n0, n1, ctr_lo, ctr_hi,"
                    " SIGMA2, k[4], k[5], k[6], k[7], SIGMA3};")
    body.append("    uint32_t " + ", ".join(f"x{i}" for i in range(16)) + ", t0, t1, t2, t3;")
    # the sequence as `segments` asm statements (registers carried across):
    # code the compiler schedules (e.g. the previous window's Poly1305) can
    # then sit at the seams instead of before or after the whole block
    nseg = max(1, segments)
    bounds = [round(i * len(order) / nseg) for i in range(nseg + 1)]
    written = set()
    for sg in range(nseg):
        chunk = list(range(bounds[sg], bounds[sg + 1]))
        regs_w, regs_r = [], []
        for idx in chunk:
            op = order[idx]
            for v in (op.s1, op.s2):
                if v is not None and v in dyn_vals:
                    r = reg(v)[2:-1]
                    if r not in regs_r:
                        regs_r.append(r)
            r = reg(op.dst)[2:-1]
            if r not in regs_w:
                regs_w.append(r)
        outs = []
        for r in [f"x{i}" for i in range(16)] + [f"t{j}" for j in range(4)]:
            if r in written and (r in regs_w or r in regs_r):
                outs.append(f'[{r}] "+v"({r})')
            elif r in regs_w:
                outs.append(f'[{r}] "=&v"({r})')
        ins = []
        used_h = set()
        for idx in chunk:
            op = order[idx]
            for v in (op.s1, op.s2):
                if v is not None and v not in dyn_vals:
                    used_h.add(need.index(v))
        for i in sorted(used_h):
            v = need[i]
            if v in dyn_inputs:  # a per-block input word (version 0)
                src = "ctr_lo" if hoist else f"init[{v[1:v.index('.')]}]"
            else:
                src = f"hs.v[{hs_index[v]}]"
            ins.append(f'[h{i}] "v"({src})')
        body.append("    asm volatile(")
        body += [f'        "{lines_asm[idx]}\\n"' for idx in chunk]
        body.append("        : " + ",\n          ".join(outs))
        body.append("        : " + ",\n          ".join(ins) + ");")
        written.update(regs_w)
    ff = ["SIGMA0", "k[0]", "k[1]", "k[2]", "k[3]", "SIGMA1", "n0", "n1", "ctr_lo", "ctr_hi", "SIGMA2", "k[4]",
          "k[5]", "k[6]", "k[7]", "SIGMA3"]
    for i in range(16):
        body.append(f"    out[{i}] = x{i} + {ff[i]};")
    body.append("}")
    out.append("\n".join(body))
    return "\n\n".join(out), len(hoisted), nvops


def main():
    path = sys.argv[1]
    parts = ["// curve_salsa_asm.hpp -- GENERATED by gen_salsa_asm.py (do not edit): the Salsa20/20\n"
             "// core in a fixed skewed issue order (see the generator's docstring).\n"
             "#pragma once\n\n#include <stdint.h>\n\nnamespace zmqg {"]
    h, nh, nv = gen_variant("salsa20_hoist", "salsa20_block_hoisted", True)
    parts.append(h)
    b, nb, nv2 = gen_variant(None, "salsa20_block_skew", False)
    parts.append(f"// no hoisting: {nv2} ops per block, every input per block\n" + b)
    seg = gen_variant(None, "salsa20_block_hoisted_seg", True, segments=5)[0]
    seg = seg[seg.index("__device__ __forceinline__ void salsa20_block_hoisted_seg"):]
    parts.append("// the hoisted block as five asm statements (Poly1305 of the previous window\n"
                 "// can be scheduled at the seams)\n" + seg)
    parts.append("} // namespace zmqg")
    with open(path, "w") as f:
        f.write("\n\n".join(parts) + "\n")
    print(f"hoisted variant: {nv} per-block ops, {nh} hoisted values; plain: {nv2} ops, {nb} inputs")


if __name__ == "__main__":
    main()
