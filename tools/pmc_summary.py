#!/usr/bin/env python3
"""profiles/pmc_k_shadow.json from rocprofv3 --pmc passes over `bench.py --steps 1` (one k_shadow
launch per pass; gpu_round.sh steps pmcf / pmcw / pmcv).

usage: pmc_summary.py <key> <fetch_dir> <write_dir> <sq_dir> [ta_dir] [kernel-substring]
Per launch of the kernel (default k_shadow):
  hbm_bytes_per_launch = 2 * FETCH_SIZE + WRITE_SIZE (KiB -> bytes; on gfx950 FETCH_SIZE counts
  128-B fabric read requests at 64 B, hence the 2: MI355X_MICROARCH.md, HBM section).  Both come
  from the L2's memory-side request counters, which include Infinity-Cache hits: L2-miss traffic,
  an upper bound on HBM bytes.
  sq_*: the SQ counters of the sq pass (SQ_INSTS_VALU = wave-level VALU instructions issued).
  *_frame: the same summed over the pass's launches per frame (PMC_FRAMES, default 1): a frame
  rendered in several chunks launches the kernel once per chunk, with chunks of unequal size.
  ta_busy_frac (optional ta pass, gpu_round.sh pmcta): TA_TA_BUSY_sum / (256 CUs x GRBM_GUI_ACTIVE / 8
  XCDs), the share of the kernel's cycles the texture-address units (vector-memory address
  path, one per CU) were busy; td_busy_frac likewise for TD_TD_BUSY_sum.
kernel_src_sha ties the entry to the k_shadow sources it measured (bench.py shadow_src_sha).
"""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def rows(d):
    for dirpath, _, files in os.walk(d):
        for f in files:
            if f.endswith("counter_collection.csv"):
                yield from csv.DictReader(open(os.path.join(dirpath, f)))


def per_launch(d, kern):
    acc = {}
    for r in rows(d):
        if kern in r["Kernel_Name"]:
            acc.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    if not acc:
        raise SystemExit(f"no {kern} rows in {d}")
    return {k: sum(v) / len(v) for k, v in acc.items()}, max(len(v) for v in acc.values())


def per_frame(d, kern, frames):
    """the kernel's counters summed over every launch of the pass, per rendered frame (a frame
    split into chunks launches the kernel once per chunk, and the chunks differ in size)"""
    acc = {}
    for r in rows(d):
        if kern in r["Kernel_Name"]:
            acc[r["Counter_Name"]] = acc.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return {k: v / frames for k, v in acc.items()}


def main():
    key, fdir, wdir, sdir = sys.argv[1:5]
    rest = sys.argv[5:]
    tdir = rest.pop(0) if rest and os.path.isdir(rest[0]) else None
    kern = rest[0] if rest else "k_shadow"
    import bench
    f, nf = per_launch(fdir, kern)
    w, nw = per_launch(wdir, kern)
    sq, ns = per_launch(sdir, kern)
    frames = int(os.environ.get("PMC_FRAMES", "1"))  # gpu_round.sh pmc* passes: bench.py --steps 1 --warmup 0
    ff, wf, sf = per_frame(fdir, kern, frames), per_frame(wdir, kern, frames), per_frame(sdir, kern, frames)
    out_path = os.path.join(ROOT, "profiles", "pmc_k_shadow.json")
    data = json.load(open(out_path)) if os.path.exists(out_path) else {}
    e = {"kernel": kern, "kernel_src_sha": bench.shadow_src_sha(),
         "hbm_bytes_per_launch": int(2 * f["FETCH_SIZE"] * 1024 + w["WRITE_SIZE"] * 1024),
         "fetch_size_kib": f["FETCH_SIZE"], "write_size_kib": w["WRITE_SIZE"], "launches": [nf, nw, ns],
         "hbm_bytes_per_frame": int(2 * ff["FETCH_SIZE"] * 1024 + wf["WRITE_SIZE"] * 1024),
         "sq_insts_valu_frame": sf["SQ_INSTS_VALU"], "frames": frames,
         "source": [os.path.relpath(x, ROOT) for x in (fdir, wdir, sdir)],
         "formula": "2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 FETCH_SIZE halving; L2->fabric, "
                    "Infinity-Cache hits included)"}
    for k, v in sq.items():
        e[k.lower()] = v
    if "SQ_ACTIVE_INST_VALU2" in sf:  # dual-issue quad-cycles (bench.py roofline issue_slots)
        e["sq_active_inst_valu2_frame"] = sf["SQ_ACTIVE_INST_VALU2"]
    if tdir:
        ta, nt = per_launch(tdir, kern)
        cyc = ta["GRBM_GUI_ACTIVE"] / 8.0  # summed over the 8 XCDs
        e["ta_busy_frac"] = round(ta["TA_TA_BUSY_sum"] / (256 * cyc), 4)
        e["td_busy_frac"] = round(ta["TD_TD_BUSY_sum"] / (256 * cyc), 4)
        e["tcp_cache_accesses"] = ta["TCP_TOTAL_CACHE_ACCESSES_sum"]
        e["source"].append(os.path.relpath(tdir, ROOT))
        e["launches"].append(nt)
    data[key] = e
    with open(out_path, "w") as fh:
        json.dump(data, fh, indent=1)
    print(key, e)


if __name__ == "__main__":
    main()
