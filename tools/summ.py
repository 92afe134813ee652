#!/usr/bin/env python3
"""Summarise bench JSON lines in gpurun_out/<tag>/*.log: value and per-kernel times."""
import glob, json, os, sys
for tag in sys.argv[1:]:
    for f in sorted(glob.glob(f"gpurun_out/{tag}/*.log")):
        for line in open(f, errors="replace"):
            if line.startswith("{") and '"metric"' in line:
                d = json.loads(line)
                k = d["config"].get("kernels_rank0", {})
                print(f"{os.path.basename(f):24s} {d['value']:10.2f} {d['unit']}  shadow={k.get('shadow_ms')} "
                      f"trace={k.get('trace_ms')} occ={d['config'].get('shadow_occ')}")
