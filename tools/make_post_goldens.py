#!/usr/bin/env python3
"""Golden fixtures for the postprocess path (src/postprocess/postproc.c).

Runs HERE only (needs oracle/_ref, built from /root/reference's own sources by
`make -C oracle ref`).  For each (input, flags) case it runs the reference's postprocess()
through oracle/_ref/post_dump (reference image_load + postprocess, float raster dumped
instead of save_image's 8-bit quantisation) and commits

  tests/golden/post/<input>.npz   rgb_in (H,W,3), z_in (H,W): the raw TIFF the reference read
  tests/golden/post/manifest.json case -> input, flags, output file
  tests/golden/post/<case>.npy    rgb_out (H,W,3) float32, the reference's result

Inputs:
  synth_*   synthetic frames written by OUR raw-TIFF writer (rtx_tiff_write): the reference
            postprocessor reading them is also the TIFF-compatibility check (§8(f) #4)
  s1_raw    a reference render (-f) of scenes/scene1.json (has background pixels, z = 0); the
            libtiff-written file itself is kept as s1_raw.tif for the C raw-TIFF reader test
Also records the reference postprocessor's own 8-bit TIFF for one case (save_image parity).
"""
import json
import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "c-raytracer_amd"))
sys.path.insert(0, HERE)
import rtxpy  # noqa: E402
from rtxpy.tiffread import read_tiff  # noqa: E402
from make_goldens import run_ref, workdir, REFBIN  # noqa: E402

OUT = os.path.join(REPO, "tests", "golden", "post")

CASES = [
    # name, input, flags
    ("b17", "synth_a", ["-b", "1.7"]),
    ("dof_small", "synth_a", ["--dof", "0.35", "0.2"]),
    ("dof_mid", "synth_a", ["--dof", "0.9", "-1.5"]),
    ("dof_big", "synth_b", ["--dof", "2.5", "0"]),
    ("dof_cam", "synth_b", ["--dof-camera", "1.5", "1.0", "4.0"]),
    ("mist_quad", "synth_a", ["--mist", "2", "5", "quad", "0.5", "0.6", "0.7"]),
    ("mist_lin", "synth_b", ["--mist", "1", "3", "lin", "1", "1", "1"]),
    ("mist_invq", "synth_a", ["--mist", "0.5", "4", "inv-quad", "0.2", "0.3", "0.4"]),
    ("combo", "synth_b", ["-b", "1.2", "--dof", "0.5", "-0.5", "--mist", "2", "6", "lin", "0.6", "0.6", "0.7"]),
    ("s1_dof", "s1_raw", ["--dof", "1.2", "-1"]),
    ("s1_mist", "s1_raw", ["-b", "0.8", "--mist", "3", "10", "quad", "0.7", "0.7", "0.8"]),
]


def synth(seed, w, h):
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
    z = (3.0 + 2.0 * np.sin(xx / 7.0) * np.cos(yy / 5.0) + (xx > w / 2) * 2.5).astype(np.float32)
    z += rng.uniform(0, 0.05, z.shape).astype(np.float32)
    rgb = rng.uniform(0, 1, (h, w, 3)).astype(np.float32)
    return rgb, z


def main():
    os.makedirs(OUT, exist_ok=True)
    tmp = tempfile.mkdtemp(prefix="rtx_post_")
    inputs = {}
    for name, seed, (w, h) in (("synth_a", 11, (64, 48)), ("synth_b", 12, (80, 40))):
        rgb, z = synth(seed, w, h)
        path = os.path.join(tmp, name + ".tif")
        rtxpy.write_tiff(path, rgb, z, raw=True)
        inputs[name] = path
    wd = workdir()
    run_ref(os.path.join(REFBIN, "engine_constO2_native"), wd, "scene1.json", 96, 54, [], 8)
    inputs["s1_raw"] = os.path.join(tmp, "s1_raw.tif")
    os.replace(os.path.join(wd, "out.tif"), inputs["s1_raw"])

    shutil.copy(inputs["s1_raw"], os.path.join(OUT, "s1_raw.tif"))  # libtiff-written raw TIFF (reader test)
    for name, path in inputs.items():
        img = read_tiff(path)
        np.savez_compressed(os.path.join(OUT, name + ".npz"), rgb_in=img["rgb"], z_in=img["z"])

    manifest = {}
    for case, inp, flags in CASES:
        dump = os.path.join(tmp, case + ".f32")
        subprocess.run([os.path.join(REFBIN, "post_dump"), inputs[inp], dump] + flags, check=True,
                       capture_output=True)
        raw = np.fromfile(dump, dtype=np.uint8)
        w, h = np.frombuffer(raw[:8].tobytes(), dtype=np.uint32)
        out = np.frombuffer(raw[8:].tobytes(), dtype=np.float32).reshape(h, w, 3)
        np.save(os.path.join(OUT, case + ".npy"), out)
        manifest[case] = {"input": inp, "flags": flags, "nan": int(np.isnan(out).sum())}
        print(case, inp, flags, "nan", manifest[case]["nan"], "max", float(np.nanmax(out)))
    # the reference's own save_image on one case: 8-bit quantisation parity of the CLI
    t8 = os.path.join(tmp, "combo8.tif")
    subprocess.run([os.path.join(REFBIN, "postprocess"), inputs["synth_b"], t8] + CASES[8][2], check=True,
                   capture_output=True)
    img8 = read_tiff(t8)
    np.save(os.path.join(OUT, "combo_u8.npy"), img8["rgb"])
    manifest["combo"]["u8"] = "combo_u8.npy"
    json.dump(manifest, open(os.path.join(OUT, "manifest.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
