#!/usr/bin/env python3
"""Static instruction census of one kernel in the library's device assembly
(`make -C libzmq_amd/csrc asm` -> libzmq_amd/csrc/zmqg_curve.s).

Splits the kernel into basic blocks, finds its loops (a branch back to an
earlier label of the same kernel), and counts VALU / SALU / VMEM (global
loads, stores, LDS-DMA) / LDS / branch instructions per block, and the
VALU instructions by opcode.  Prints the loop bodies and the totals outside
them, so the per-window cost of a frame kernel can be told from its fixed
per-frame part.

  isa_census.py <asm> <kernel-name-regex> [--blocks]
"""
import collections
import re
import sys


def kernel_lines(path, pat):
    rx = re.compile(pat)
    out, on = [], False
    for line in open(path):
        if not on:
            if re.match(r"^[A-Za-z_][\w.$]*:", line) and rx.search(line.split(":")[0]):
                on = True
                out.append(line.rstrip("\n"))
            continue
        if line.startswith(".Lfunc_end"):
            break
        out.append(line.rstrip("\n"))
    return out


def classify(op):
    if op.startswith("v_"):
        return "valu"
    if op.startswith(("global_load_lds", "buffer_load")) and "lds" in op:
        return "vmem_lds_dma"
    if op.startswith(("global_store", "buffer_store", "flat_store")):
        return "vmem_store"
    if op.startswith(("global_load", "buffer_load", "flat_load")):
        return "vmem_load"
    if op.startswith(("global_atomic", "flat_atomic", "buffer_atomic")):
        return "vmem_atomic"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith(("s_load", "s_buffer_load")):
        return "smem"
    if op.startswith("s_"):
        return "salu"
    return None


def main():
    path, pat = sys.argv[1], sys.argv[2]
    show = "--blocks" in sys.argv
    lines = kernel_lines(path, pat)
    if not lines:
        sys.exit(f"no kernel matching {pat}")
    blocks, order, cur = {}, [], "entry"
    blocks[cur] = {"ins": [], "succ": []}
    order.append(cur)
    for line in lines[1:]:
        m = re.match(r"^(\.LBB[\w_]+):", line)
        if m:
            cur = m.group(1)
            blocks[cur] = {"ins": [], "succ": []}
            order.append(cur)
            continue
        t = line.strip()
        if not t or t.startswith((";", ".")):
            continue
        op = t.split()[0]
        blocks[cur]["ins"].append(op)
        if op.startswith(("s_cbranch", "s_branch")):
            tgt = t.split()[-1]
            blocks[cur]["succ"].append(tgt)
    pos = {b: i for i, b in enumerate(order)}
    loops = []  # (header, latch)
    for b in order:
        for tgt in blocks[b]["succ"]:
            if tgt in pos and pos[tgt] <= pos[b]:
                loops.append((tgt, b))
    in_loop = set()
    for h, l in loops:
        for b in order[pos[h]:pos[l] + 1]:
            in_loop.add(b)

    def count(bs):
        c, ops = collections.Counter(), collections.Counter()
        for b in bs:
            for op in blocks[b]["ins"]:
                k = classify(op)
                if k:
                    c[k] += 1
                if k == "valu":
                    ops[op] += 1
        return c, ops

    print(f"kernel: {lines[0].split(':')[0][:120]}")
    print(f"blocks {len(order)}, instructions {sum(len(blocks[b]['ins']) for b in order)}")
    for h, l in loops:
        c, ops = count(order[pos[h]:pos[l] + 1])
        print(f"loop {h} .. {l} ({pos[l] - pos[h] + 1} blocks): " + ", ".join(f"{k} {v}" for k, v in sorted(c.items())))
        print("   valu by opcode: " + ", ".join(f"{o} {n}" for o, n in ops.most_common(12)))
    c, ops = count([b for b in order if b not in in_loop])
    print("outside the loops: " + ", ".join(f"{k} {v}" for k, v in sorted(c.items())))
    print("   valu by opcode: " + ", ".join(f"{o} {n}" for o, n in ops.most_common(16)))
    if show:
        for b in order:
            c, _ = count([b])
            print(f"  {'L' if b in in_loop else ' '} {b:40s} " + ", ".join(f"{k} {v}" for k, v in sorted(c.items())))


if __name__ == "__main__":
    main()
