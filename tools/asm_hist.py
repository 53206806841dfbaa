#!/usr/bin/env python3
"""Static instruction histogram per kernel of a hipcc -S output."""
import collections
import re
import sys

lines = open(sys.argv[1]).read().split('\n')
keys = sys.argv[2:] or ['body', 'head']
starts = [(i, m.group(1)) for i, l in enumerate(lines) for m in [re.match(r'^(_Z\S+):\s*(;.*)?$', l)] if m]
for i, name in starts:
    if not any(k in name for k in keys):
        continue
    j = i + 1
    while j < len(lines) and not lines[j].startswith('\t.section') and '.Lfunc_end' not in lines[j]:
        j += 1
    ops = collections.Counter()
    for l in lines[i + 1:j]:
        l = l.strip()
        if not l or l.startswith(('.', ';')) or re.match(r'^\S+:', l):
            continue
        ops[l.split()[0]] += 1
    print(name[:60], 'static instrs', sum(ops.values()))
    print('   ', ', '.join(f'{o}:{c}' for o, c in ops.most_common(40)))
