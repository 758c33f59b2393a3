#!/usr/bin/env python3
"""Static instruction mix of kernels in a gfx950 .s file: tools/isa_mix.py file.s [substr ...]"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
pats = sys.argv[2:]
for m in re.finditer(r'^(_Z\w+):\s*(;.*)?$', s, re.M):
    n = m.group(1)
    if pats and not any(p in n for p in pats):
        continue
    j = s.find('.Lfunc_end', m.end())
    if j < 0:
        continue
    ops = collections.Counter()
    for line in s[m.end():j].split('\n'):
        line = line.strip()
        if not line or line.startswith(('.', ';', '//')) or line.endswith(':'):
            continue
        ops[line.split()[0]] += 1
    tot = sum(ops.values())
    if tot < 20:
        continue
    print(n[:70], 'static instrs', tot)
    print('   ', ops.most_common(30))
