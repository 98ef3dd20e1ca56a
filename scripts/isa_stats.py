#!/usr/bin/env python3
"""Instruction mix of one kernel in a hipcc -save-temps .s file."""
import collections
import re
import sys

path, pat = sys.argv[1], sys.argv[2]
s = open(path).read()
for m in re.finditer(r'^(\S*' + pat + r'\S*):\s*;', s, re.M):
    start = m.end()
    end = s.find('.Lfunc_end', start)
    body = s[start:end]
    lines = [l.strip() for l in body.splitlines()]
    ins = [l for l in lines if l and not l.startswith(('.', ';', '//')) and not l.endswith(':')]
    c = collections.Counter(l.split()[0] for l in ins)
    print(m.group(1), 'instructions:', len(ins))
    mem = {k: v for k, v in c.items() if any(t in k for t in ('load', 'store', 'waitcnt', 'scratch', 'ds_', 'branch', 'swappc', 'atomic'))}
    print(' memory/control:', dict(sorted(mem.items(), key=lambda kv: -kv[1])))
    print(' top:', c.most_common(20))
