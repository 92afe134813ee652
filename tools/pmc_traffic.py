#!/usr/bin/env python3
"""profiles/pmc_traffic.json from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over bench.py.

usage: pmc_traffic.py <fetch_dir> <write_dir> <key> [kernel-substring]
Per launch of the kernel (default k_shadow): bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024.
FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE counts 128-B fabric read requests at
64 B, hence the factor 2 (MI355X_MICROARCH.md, HBM section).  Both derive from the L2's
memory-side request counters, which also count Infinity-Cache hits: this is L2-miss traffic
(MALL + HBM), an upper bound on HBM bytes.
"""
import csv, json, os, sys


def per_launch(d, counter, kern):
    vals = []
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        if kern in r["Kernel_Name"] and r["Counter_Name"] == counter:
            vals.append(float(r["Counter_Value"]))
    if not vals:
        raise SystemExit(f"no {counter} rows for {kern} in {d}")
    return sum(vals) / len(vals), len(vals)


def main():
    fdir, wdir, key = sys.argv[1:4]
    kern = sys.argv[4] if len(sys.argv) > 4 else "k_shadow"
    f, nf = per_launch(fdir, "FETCH_SIZE", kern)
    w, nw = per_launch(wdir, "WRITE_SIZE", kern)
    out_path = os.path.join(os.path.dirname(__file__), "..", "profiles", "pmc_traffic.json")
    data = json.load(open(out_path)) if os.path.exists(out_path) else {}
    data[key] = {"kernel": kern, "hbm_bytes_per_launch": int(2 * f * 1024 + w * 1024),
                 "fetch_size_kib": f, "write_size_kib": w, "launches": [nf, nw],
                 "source": [os.path.relpath(fdir), os.path.relpath(wdir)],
                 "formula": "2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 FETCH_SIZE halving; L2->fabric, "
                            "Infinity-Cache hits included)"}
    json.dump(data, open(out_path, "w"), indent=1)
    print(key, data[key])


if __name__ == "__main__":
    main()
