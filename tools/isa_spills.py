#!/usr/bin/env python3
"""Scratch (spill) stores and reloads of one kernel in a hipcc -S listing, by the size and depth of
the innermost loop around them: usage isa_spills.py file.s mangled_kernel_symbol [--print]"""
import re
import sys
from collections import Counter

src = open(sys.argv[1]).read().split("\n")
sym = sys.argv[2]
st = next(i for i, l in enumerate(src) if l.startswith(sym + ":"))
en = next(i for i in range(st, len(src)) if src[i].startswith(".Lfunc_end"))
body = src[st:en]
labels = {m.group(1): i for i, l in enumerate(body) for m in [re.match(r"^(\.LBB\w+):", l)] if m}
loops = []
for i, l in enumerate(body):
    m = re.match(r"\s+s_(?:cbranch_\w+|branch)\s+(\.LBB\w+)", l)
    if m and m.group(1) in labels and labels[m.group(1)] <= i:
        loops.append((labels[m.group(1)], i))


def inner(i):
    inl = [(a, b) for a, b in loops if a <= i <= b]
    return (min((b - a for a, b in inl), default=0), len(inl))


for kind in ("scratch_store", "scratch_load"):
    ops = [i for i, l in enumerate(body) if l.strip().startswith(kind)]
    print(kind, len(ops), "by (innermost loop lines, loop depth):", sorted(Counter(inner(i) for i in ops).items()))
    if "--print" in sys.argv:
        for i in ops:
            print("   ", i, body[i].strip()[:80], inner(i))
