#!/usr/bin/env python3
"""Multi-seed statistical goldens from the compiled reference ("colour under
counter RNG vs seeded reference: per-channel image means within 1 % and 8x8-box-filtered relL1
<= 3 %").  Runs HERE only (the GPU box has no /root/reference); outputs are committed under
tests/golden/seeds/:

  <name>.npz      mean_rgb (H,W,3 f32: the average of the S seeded reference frames),
                  z (H,W f32, RNG-independent), seed_means (S,3 f64: each frame's channel means),
                  seeds (S,)
  manifest.json   scene, resolution, flags, seeds, the per-seed sigma of the image mean and the
                  sigma of the S-seed average, per channel (relative)

Each frame is the reference's own glibc rand() stream seeded with S (oracle/_ref/engine_seedO2_native,
-m 1: srand(S) through oracle/ref_shim.h), i.e. the reference's RNG semantics, not ours.  The tests
average the same number of seeds of the GPU (and oracle) renders under the counter RNG, so the
comparison is between two S-seed averages whose noise is ~sigma_avg * sqrt(2).
"""
import argparse
import json
import os
import shutil
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "c-raytracer_amd"))
sys.path.insert(0, HERE)
from rtxpy.tiffread import read_tiff  # noqa: E402
import standins  # noqa: E402

GOLDEN = os.path.join(REPO, "tests", "golden")
OUT = os.path.join(GOLDEN, "seeds")
REFBIN = os.path.join(REPO, "oracle", "_ref", "engine_seedO2_native")

# name, scene file (tests/golden/scenes), W, H, flags, number of seeds
CONFIGS = [
    ("s1_amb", "scene1.json", 64, 64, [], 16),
    ("s3_path16", "scene3.json", 64, 36, ["-g", "path", "-n", "16"], 16),
    ("s4_path4_blinn", "scene4.json", 64, 36, ["-g", "path", "-n", "4", "-s", "blinn"], 256),
    ("s5_path4", "scene5_standin.json", 48, 27, ["-g", "path", "-n", "4"], 16),
    ("s6_path8", "scene6_standin.json", 128, 72, ["-g", "path", "-n", "8"], 32),
]


def render(scene, w, h, flags, seed):
    wd = tempfile.mkdtemp(prefix="rtx_seed_")
    try:
        os.symlink(os.path.join(GOLDEN, "scenes"), os.path.join(wd, "scenes"))
        os.symlink(os.path.join(GOLDEN, "meshes"), os.path.join(wd, "meshes"))
        out = os.path.join(wd, "o.tif")
        cmd = [REFBIN, os.path.join("scenes", scene), out, str(w), str(h), "-f", "-m", "1"] + flags
        env = dict(os.environ, RTX_REF_SEED=str(seed), OMP_NUM_THREADS="1")
        p = subprocess.run(cmd, cwd=wd, env=env, capture_output=True, text=True)
        if p.returncode != 0:
            raise RuntimeError(f"{cmd} rc={p.returncode}: {p.stderr[-300:]}")
        img = read_tiff(out)
        return img["rgb"].astype(np.float64), img["z"].astype(np.float32)
    finally:
        shutil.rmtree(wd)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", nargs="*")
    ap.add_argument("-j", type=int, default=6)
    a = ap.parse_args()
    if not os.path.exists(REFBIN):
        sys.exit("build the reference first: make -C oracle ref")
    standins.ensure_scene("scene5")
    standins.ensure_scene("scene6")
    os.makedirs(OUT, exist_ok=True)
    mpath = os.path.join(OUT, "manifest.json")
    manifest = json.load(open(mpath)) if os.path.exists(mpath) else {}
    for name, scene, w, h, flags, ns in CONFIGS:
        if a.only and name not in a.only:
            continue
        seeds = list(range(1, ns + 1))
        with ThreadPoolExecutor(a.j) as ex:
            frames = list(ex.map(lambda s: render(scene, w, h, flags, s), seeds))
        rgbs = np.stack([f[0] for f in frames])
        z = frames[0][1]
        assert all(np.array_equal(f[1], z) for f in frames), "z-buffer must not depend on the seed"
        seed_means = rgbs.reshape(ns, -1, 3).mean(1)
        mu = seed_means.mean(0)
        sig = seed_means.std(0, ddof=1) / np.abs(mu)
        np.savez_compressed(os.path.join(OUT, name + ".npz"), mean_rgb=rgbs.mean(0).astype(np.float32), z=z,
                            seed_means=seed_means, seeds=np.array(seeds))
        manifest[name] = {"scene": scene, "width": w, "height": h, "flags": flags, "seeds": seeds,
                          "sigma_mean_rel": [round(float(x), 6) for x in sig],
                          "sigma_avg_rel": [round(float(x) / np.sqrt(ns), 6) for x in sig]}
        print(f"{name:16s} {w}x{h} {' '.join(flags):24s} seeds={ns} sigma(mean)={np.round(sig, 4)} "
              f"sigma(avg)={np.round(sig / np.sqrt(ns), 4)}", flush=True)
    with open(mpath, "w") as fh:
        json.dump(manifest, fh, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
