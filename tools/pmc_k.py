#!/usr/bin/env python3
"""Per-kernel PMC counter values (summed over dispatches / number of dispatches) from rocprofv3
csv counter files: pmc_k.py <kernel-substring> file_or_dir..."""
import csv
import glob
import os
import sys

pat = sys.argv[1]
for arg in sys.argv[2:]:
    files = glob.glob(os.path.join(arg, "**", "*counter_collection.csv"), recursive=True) if os.path.isdir(arg) else [arg] * arg.endswith(".csv")
    for f in files:
        vals, disp = {}, set()
        for r in csv.DictReader(open(f)):
            if pat in r["Kernel_Name"]:
                vals[r["Counter_Name"]] = vals.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
                disp.add(r["Dispatch_Id"])
        n = max(1, len(disp))
        print(f, f"dispatches={len(disp)}")
        for k in sorted(vals):
            print(f"  {k:24s} {vals[k] / n:.4e}")
