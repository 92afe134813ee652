#!/usr/bin/env python3
"""Register / spill metadata of the kernels in a hipcc -S listing (the amdhsa.kernels YAML):
usage: isa_meta.py file.s [name-substring]"""
import re
import sys

text = open(sys.argv[1]).read()
want = sys.argv[2] if len(sys.argv) > 2 else ""
meta = text[text.find("amdhsa.kernels:"):]
# one YAML mapping per kernel: entries start with "  - " at the kernels list's indentation
for block in re.split(r"\n  - ", meta)[1:]:
    fields = dict(re.findall(r"^\s+\.(\w+):\s+(\S+)$", block, flags=re.M))
    name = fields.get("name", "?")
    if want not in name:
        continue
    print(name, {k: fields.get(k) for k in ("vgpr_count", "vgpr_spill_count", "sgpr_count", "sgpr_spill_count",
                                            "private_segment_fixed_size", "group_segment_fixed_size")})
