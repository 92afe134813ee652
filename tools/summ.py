#!/usr/bin/env python3
"""Summarise bench JSON lines in gpurun_out/<tag>/*.log: value, per-kernel times and the
shadow walk's traversal counts (development tool)."""
import glob
import json
import os
import sys

for tag in sys.argv[1:]:
    for f in sorted(glob.glob(f"gpurun_out/{tag}/*.log")):
        for line in open(f, errors="replace"):
            if line.startswith("{") and '"metric"' in line:
                d = json.loads(line)
                k = d["config"].get("kernels_rank0", {})
                r = d.get("roofline") or {}
                tf = d["config"].get("tree_frame", {})
                print(f"{os.path.basename(f):28s} {d['value']:10.1f} {d['unit']} step={d['ms_per_step']}ms "
                      f"trace={k.get('trace_ms')} sort={k.get('sort_ms')} shadow={k.get('shadow_ms')} "
                      f"rot={tf.get('rotated')} steps={r.get('wave_steps')} lrounds={r.get('leaf_rounds')} "
                      f"boxes={r.get('box_tests')} tris={r.get('tri_tests')} frac={r.get('frac')} "
                      f"cpu={(d.get('cpu_baseline') or {}).get('value')}")
