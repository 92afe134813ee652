#!/usr/bin/env python3
"""Per-loop instruction census of one kernel in a hipcc -S listing (spills, VALU, SALU, loads).
usage: isa_loops.py file.s kernel_substring"""
import re, sys
from collections import Counter
src = open(sys.argv[1]).read().split("\n")
pat = sys.argv[2]
start = next(i for i, l in enumerate(src) if re.match(r"^_Z\w*" + pat + r"\w*:", l))
end = next(i for i in range(start, len(src)) if src[i].startswith(".Lfunc_end"))
body = src[start:end]
# block -> loop depth from the "; Loop Header: Depth=N" / "in Loop: Header=... Depth=N" comments
depth, cur = {}, 0
stats = Counter()
for l in body:
    m = re.match(r"^(\.LBB\w+|; %bb\.\d+):.*?(?:Depth=(\d+))?\s*$", l)
    if m:
        cur = int(m.group(2) or 0)
        continue
    s = l.strip()
    if not s or s.startswith(";") or s.startswith("."):
        continue
    op = s.split()[0]
    cls = ("scratch" if op.startswith("scratch_") else "vlane" if op in ("v_readlane_b32", "v_writelane_b32") else
           "smem" if op.startswith("s_load") or op.startswith("s_buffer") else "vmem" if op.startswith(("global_", "buffer_")) else
           "lds" if op.startswith("ds_") else "valu" if op.startswith("v_") else "salu" if op.startswith("s_") else "other")
    stats[(cur, cls)] += 1
for d in sorted({k[0] for k in stats}):
    print(f"depth {d}: " + "  ".join(f"{c}={stats[(d, c)]}" for c in ("valu", "salu", "smem", "vmem", "lds", "scratch", "vlane")))
