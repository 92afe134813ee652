#!/usr/bin/env python3
"""Generate golden fixtures from the compiled reference (oracle/_ref, built by
`make -C oracle ref` from /root/reference's own sources).  Runs HERE only (the
GPU box has no /root/reference); the outputs are committed under tests/golden/:

  tests/golden/kat.npz              per-function known answers (oracle/ref_kat.c)
  tests/golden/frames/<name>.npz    rgb (H,W,3 f32), z (H,W f32) of a reference render
  tests/golden/frames/manifest.json configs: scene, resolution, flags, RNG, ray counts

Frames use the reference's raw output (-f: float RGB + tag-65000 z-buffer).
const   : REF_CONST_RNG build (rand_flt()==0.5f), bit-reproducible, -m 8.  Two builds:
          <name>.npz    the reference as Makefile.rt builds it (-Ofast -march=native: FMA, rsqrt)
          <name>_o2.npz the same sources at -O2 (IEEE single precision, no contraction);
          manifest "floor" = the Ofast-vs-O2 difference, i.e. the reference's own
          numeric noise floor for that config
seed<S> : glibc rand() seeded with S, -m 1, -O2 build (statistical goldens; IEEE like the const _o2
          frames so checker-boundary flips do not masquerade as sampling differences)
Ray counts come from the instrumented build (oracle/ref_count_hook.c).
"""
import argparse
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "c-raytracer_amd"))
sys.path.insert(0, HERE)
from rtxpy.tiffread import read_tiff  # noqa: E402
import standins  # noqa: E402

GOLDEN = os.path.join(REPO, "tests", "golden")
FRAMES = os.path.join(GOLDEN, "frames")
REFBIN = os.path.join(REPO, "oracle", "_ref")

# name, scene file (tests/golden/scenes), W, H, flags, rng
CONFIGS = [
    ("s1_amb", "scene1.json", 128, 128, [], "const"),
    ("s1_path2", "scene1.json", 128, 128, ["-g", "path", "-n", "2"], "const"),
    ("s1_b0", "scene1.json", 64, 64, ["-b", "0"], "const"),
    ("s2_amb", "scene2.json", 128, 72, [], "const"),
    ("s2_blinn_lin", "scene2.json", 128, 72, ["-s", "blinn", "-l", "lin"], "const"),
    ("s2_path1_b2", "scene2.json", 96, 54, ["-g", "path", "-n", "1", "-b", "2", "-o", "2"], "const"),
    ("s3_amb", "scene3.json", 128, 72, [], "const"),
    ("s3_path2", "scene3.json", 128, 72, ["-g", "path", "-n", "2"], "const"),
    ("s3_none_b3", "scene3.json", 128, 72, ["-l", "none", "-b", "3", "-o", "0.5"], "const"),
    ("s3_rnorm", "scene3.json", 96, 54, ["-r", "norm", "-a", "0.1"], "const"),
    ("s4_amb", "scene4.json", 128, 72, [], "const"),
    ("s4_path2_blinn", "scene4.json", 96, 54, ["-g", "path", "-n", "2", "-s", "blinn"], "const"),
    ("st_amb", "scenetest.json", 128, 72, [], "const"),
    ("st2_r2", "scenetest2.json", 128, 72, ["-r", "2.0"], "const"),
    ("s5_amb", "scene5_standin.json", 96, 54, [], "const"),
    ("s5_path2", "scene5_standin.json", 64, 36, ["-g", "path", "-n", "2"], "const"),
    ("s6_amb", "scene6_standin.json", 96, 54, [], "const"),
    ("s6_path2", "scene6_standin.json", 64, 36, ["-g", "path", "-n", "2"], "const"),
    ("s1_seed_amb", "scene1.json", 64, 64, [], "seed1"),
    ("s3_seed_path16", "scene3.json", 64, 36, ["-g", "path", "-n", "16"], "seed1"),
    ("s3_seed_path16_s2", "scene3.json", 64, 36, ["-g", "path", "-n", "16"], "seed2"),
    ("s5_seed_path4", "scene5_standin.json", 48, 27, ["-g", "path", "-n", "4"], "seed1"),
]


def workdir():
    d = tempfile.mkdtemp(prefix="rtx_golden_")
    os.symlink(os.path.join(GOLDEN, "scenes"), os.path.join(d, "scenes"))
    os.symlink(os.path.join(GOLDEN, "meshes"), os.path.join(d, "meshes"))
    return d


def run_ref(binary, wd, scene, w, h, flags, threads, env_extra=None):
    out = os.path.join(wd, "out.tif")
    if os.path.exists(out):
        os.remove(out)
    cmd = [binary, os.path.join("scenes", scene), out, str(w), str(h), "-f", "-m", str(threads)] + flags
    env = dict(os.environ)
    env.update(env_extra or {})
    t0 = time.time()
    p = subprocess.run(cmd, cwd=wd, env=env, capture_output=True, text=True)
    dt = time.time() - t0
    if p.returncode != 0:
        raise RuntimeError(f"{cmd} failed: {p.stdout[-500:]} {p.stderr[-500:]}")
    counts = None
    for line in p.stderr.splitlines():
        if line.startswith("RTX_REF_COUNT"):
            kv = dict(x.split("=") for x in line.split()[1:])
            counts = (int(kv["closest"]), int(kv["shadow"]))
    img = read_tiff(out) if os.path.exists(out) else None
    return img, counts, dt


def floor_metrics(rgb, z, ref_rgb, ref_z):
    hit, ref_hit = z > 0, ref_z > 0
    both = hit & ref_hit
    zr = np.abs(z - ref_z) / np.maximum(ref_z, 1.0)
    tol = 1e-4 * float(np.abs(ref_rgb).max())
    return {"hit_mismatch": float((hit != ref_hit).mean()),
            "z_ok": float((zr[both] <= 1e-4).mean()) if both.any() else 1.0,
            "px_ok": float(((np.abs(rgb - ref_rgb) <= tol).all(axis=2)).mean()),
            "rel_l1": float(np.abs(rgb - ref_rgb).sum() / max(float(np.abs(ref_rgb).sum()), 1e-30))}


def make_kat():
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "kat.bin")
        subprocess.run([os.path.join(REFBIN, "ref_kat"), path, "4096"], check=True)
        data = open(path, "rb").read()
    off = 0
    arrays = {}
    from rtxpy.abi import KAT_NAMES
    while off < len(data):
        kind, n, wi, wo = np.frombuffer(data, "<i4", 4, off)
        off += 16
        xin = np.frombuffer(data, "<f4", n * wi, off).reshape(n, wi).copy()
        off += 4 * n * wi
        xout = np.frombuffer(data, "<f4", n * wo, off).reshape(n, wo).copy()
        off += 4 * n * wo
        arrays[f"{KAT_NAMES[kind]}_in"] = xin
        arrays[f"{KAT_NAMES[kind]}_out"] = xout
    np.savez_compressed(os.path.join(GOLDEN, "kat.npz"), **arrays)
    print("kat.npz:", sorted(arrays))


def make_frames(only=None):
    os.makedirs(FRAMES, exist_ok=True)
    standins.ensure_scene("scene5")
    standins.ensure_scene("scene6")
    manifest_path = os.path.join(FRAMES, "manifest.json")
    manifest = json.load(open(manifest_path)) if os.path.exists(manifest_path) else {}
    wd = workdir()
    try:
        for name, scene, w, h, flags, rng in CONFIGS:
            if only and name not in only:
                continue
            extra = {}
            if rng == "const":
                img, _, dt = run_ref(os.path.join(REFBIN, "engine_const_native"), wd, scene, w, h, flags, 8)
                _, counts, _ = run_ref(os.path.join(REFBIN, "engine_countconst_native"), wd, scene, w, h, flags, 8)
                o2, _, _ = run_ref(os.path.join(REFBIN, "engine_constO2_native"), wd, scene, w, h, flags, 8)
                _, counts_o2, _ = run_ref(os.path.join(REFBIN, "engine_countconstO2_native"), wd, scene, w, h,
                                          flags, 8)
                np.savez_compressed(os.path.join(FRAMES, name + "_o2.npz"), rgb=o2["rgb"].astype(np.float32),
                                    z=o2["z"].astype(np.float32))
                extra = {"closest_rays_o2": counts_o2[0], "shadow_rays_o2": counts_o2[1],
                         "floor": floor_metrics(o2["rgb"], o2["z"], img["rgb"], img["z"])}
                seed = None
            else:
                seed = int(rng[4:])
                env = {"RTX_REF_SEED": str(seed)}
                img, _, dt = run_ref(os.path.join(REFBIN, "engine_seedO2_native"), wd, scene, w, h, flags, 1, env)
                _, counts, _ = run_ref(os.path.join(REFBIN, "engine_count_native"), wd, scene, w, h, flags, 1, env)
            np.savez_compressed(os.path.join(FRAMES, name + ".npz"), rgb=img["rgb"].astype(np.float32),
                                z=img["z"].astype(np.float32))
            manifest[name] = {"scene": scene, "width": w, "height": h, "flags": flags, "rng": rng, "seed": seed,
                              "closest_rays": counts[0], "shadow_rays": counts[1], "ref_seconds": round(dt, 3)}
            manifest[name].update(extra)
            print(f"{name:20s} {w}x{h} {' '.join(flags):30s} {rng:6s} rays={counts} {dt:.2f}s", flush=True)
    finally:
        shutil.rmtree(wd)
    with open(manifest_path, "w") as fh:
        json.dump(manifest, fh, indent=1, sort_keys=True)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--kat", action="store_true")
    ap.add_argument("--frames", action="store_true")
    ap.add_argument("--only", nargs="*")
    a = ap.parse_args()
    if not os.path.exists(os.path.join(REFBIN, "ref_kat")):
        sys.exit("build the reference first: make -C oracle ref")
    if a.kat or not a.frames:
        make_kat()
    if a.frames or not a.kat:
        make_frames(a.only)
