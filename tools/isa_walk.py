#!/usr/bin/env python3
"""Innermost loops of one kernel in a hipcc -S listing that contain a given instruction, with
their instruction census (used to read the shadow walk loops).
usage: isa_walk.py file.s mangled_kernel_symbol [marker-instruction] [--print]"""
import re
import sys

src = open(sys.argv[1]).read().split("\n")
sym = sys.argv[2]
marker = sys.argv[3] if len(sys.argv) > 3 and not sys.argv[3].startswith("--") else "global_load_dwordx4"
start = next(i for i, l in enumerate(src) if l.startswith(sym + ":"))
end = next(i for i in range(start, len(src)) if src[i].startswith(".Lfunc_end"))
body = src[start:end]
labels = {}
for i, l in enumerate(body):
    m = re.match(r"^(\.LBB\w+):", l)
    if m:
        labels[m.group(1)] = i
loops = []
for i, l in enumerate(body):
    m = re.match(r"\s+s_(?:cbranch_\w+|branch)\s+(\.LBB\w+)", l)
    if m and m.group(1) in labels and labels[m.group(1)] <= i:
        loops.append((labels[m.group(1)], i))


def census(lines):
    c = {"valu": 0, "salu": 0, "smem": 0, "vmem": 0, "lds": 0, "scratch": 0}
    for l in lines:
        s = l.strip()
        if not s or s.startswith(";") or s.startswith(".") or s.endswith(":"):
            continue
        op = s.split()[0]
        if op.startswith("scratch_"):
            c["scratch"] += 1
        elif op.startswith("s_load") or op.startswith("s_buffer"):
            c["smem"] += 1
        elif op.startswith(("global_", "buffer_", "flat_")):
            c["vmem"] += 1
        elif op.startswith("ds_"):
            c["lds"] += 1
        elif op.startswith("v_"):
            c["valu"] += 1
        elif op.startswith("s_"):
            c["salu"] += 1
    return c


for a, b in sorted(set(loops)):
    lines = body[a:b + 1]
    if any(marker in l for l in lines):
        print(f"loop lines {start + a + 1}-{start + b + 1} ({b - a} lines): {census(lines)}")
        if "--print" in sys.argv:
            print("\n".join(lines))
