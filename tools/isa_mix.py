#!/usr/bin/env python3
"""Instruction mix of one kernel in the gfx950 assembly (make -C sift-parallel-optimization_amd/csrc asm).

    python tools/isa_mix.py <substring of the mangled kernel name> [asm file]
"""
import collections
import re
import sys

pat = sys.argv[1]
path = sys.argv[2] if len(sys.argv) > 2 else "sift-parallel-optimization_amd/lib/gdp-gfx950.s"
s = open(path).read()
m = re.search(r"^(_Z\S*" + re.escape(pat) + r"\S*):", s, re.M)
body = s[m.end():s.index(".Lfunc_end", m.end())].split("\n")
c = collections.Counter()
for line in body:
    line = line.strip()
    if not line or line.startswith((".", ";")) or line.endswith(":"):
        continue
    c[line.split()[0]] += 1
print(m.group(1), "total", sum(c.values()))
for k, v in c.most_common(45):
    print(f"{v:6d} {k}")
