#!/usr/bin/env python3
"""Instruction histogram of one kernel in a hipcc -S (gfx950) listing:
python tools/isa_hist.py listing.s <substring of the mangled kernel name> [top]"""
import re
import sys
from collections import Counter

path, key = sys.argv[1], sys.argv[2]
top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if re.match(r"^\S+:", l) and key in l and not l.startswith("."))
end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
c = Counter()
for l in lines[start:end]:
    l = l.strip()
    if not l or l.startswith((".", ";")) or l.endswith(":"):
        continue
    c[l.split()[0]] += 1
print(lines[start].split(":")[0], "total", sum(c.values()))
for k, v in c.most_common(top):
    print(f"{v:6d} {k}")
for l in lines[end:end + 80]:
    if any(t in l for t in (".vgpr_count", ".sgpr_count", "NumVgprs", "ScratchSize", "Occupancy", "; NumVGPRsForWavesPerEU")):
        print(l.strip())
