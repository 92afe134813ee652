#!/usr/bin/env python3
"""Sum rocprofv3 counter_collection CSVs per (kernel, counter): pmc_table.py dir [dir...]"""
import csv, sys, collections
for d in [a for a in sys.argv[1:] if not a.endswith(".log")]:
    tot = collections.defaultdict(float)
    n = collections.Counter()
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:40]
        tot[(k, r["Counter_Name"])] += float(r["Counter_Value"])
        n[(k, r["Counter_Name"])] += 1
    print("==", d)
    for (k, c), v in sorted(tot.items()):
        if "k_shadow" in k:
            print(f"  {k:40s} {c:22s} {v:14.4g}  (x{n[(k, c)]})")
