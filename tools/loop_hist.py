#!/usr/bin/env python3
"""Instruction histogram of the innermost loops of a kernel in hipcc -S output:
basic blocks between a loop header label and the backward branch to it."""
import collections
import re
import sys

lines = open(sys.argv[1]).read().split('\n')
key = sys.argv[2]
start = next(i for i, l in enumerate(lines) if re.match(r'^(_Z\S+):', l) and key in l)
end = next(i for i in range(start + 1, len(lines)) if '.Lfunc_end' in lines[i])
body = lines[start:end]
labels = {m.group(1): i for i, l in enumerate(body) for m in [re.match(r'^(\.LBB\S+):', l)] if m}
loops = []
for i, l in enumerate(body):
    m = re.search(r's_cbranch_\w+\s+(\.LBB\S+)|s_branch\s+(\.LBB\S+)', l)
    if m:
        tgt = m.group(1) or m.group(2)
        if tgt in labels and labels[tgt] < i:
            loops.append((labels[tgt], i))
for a, b in loops:
    ops = collections.Counter()
    for l in body[a:b + 1]:
        l = l.strip()
        if not l or l.startswith(('.', ';')) or re.match(r'^\S+:', l):
            continue
        ops[l.split()[0]] += 1
    tot = sum(ops.values())
    valu = sum(c for o, c in ops.items() if o.startswith('v_'))
    print(f'loop lines {a}-{b}: {tot} instrs, {valu} VALU')
    print('   ', ', '.join(f'{o}:{c}' for o, c in ops.most_common(45)))
