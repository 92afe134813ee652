"""The drop-in renderer CLI (lib/engine, host/main.c) end to end on the GPU: the reference's
argument layout, JSON + STL loading from the working directory, rendering through the C-ABI,
and the raw (-f) TIFF it writes, against the same golden frames as the library tests."""
import os
import subprocess

import numpy as np
import pytest

import conftest as C
import rtxpy
import standins

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["s1_amb", "s2_blinn_lin", "s3_path2", "s5_path2"])
def test_gpu_engine_cli_matches_golden(name, tmp_path):
    m = C.manifest()[name]
    if "standin" in m["scene"]:
        standins.ensure_scene(m["scene"].split("_standin")[0])
    out = str(tmp_path / "o.tif")
    cmd = [rtxpy.ENGINE, os.path.join("scenes", m["scene"]), out, str(m["width"]), str(m["height"]), "-f",
           "--rng", "const"] + m["flags"]
    p = subprocess.run(cmd, cwd=C.GOLDEN, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    rgb, z = rtxpy.read_tiff_raw(out)
    ref_rgb, ref_z = C.golden_frame(name + "_o2")
    ok, info = C.compare_const(rgb, z, ref_rgb, ref_z)
    assert ok, info
    assert "Saving image" in p.stdout


def test_gpu_engine_8bit_output(tmp_path):
    """8-bit TIFF (no -f): save_tiff's clamp/truncate of the same raster."""
    m = C.manifest()["s3_path2"]
    base = [rtxpy.ENGINE, os.path.join("scenes", m["scene"])]
    args = [str(m["width"]), str(m["height"]), "--rng", "const"] + m["flags"]
    raw, u8 = str(tmp_path / "raw.tif"), str(tmp_path / "u8.tif")
    for o, extra in ((raw, ["-f"]), (u8, [])):
        p = subprocess.run(base + [o] + args + extra, cwd=C.GOLDEN, capture_output=True, text=True, timeout=300)
        assert p.returncode == 0, p.stdout[-1000:]
    rgb, _ = rtxpy.read_tiff_raw(raw)
    from rtxpy.tiffread import read_tiff
    img = read_tiff(u8)["rgb"]
    expect = np.clip(rgb * 255.0, 0, 255).astype(np.uint8)  # (uint8_t)fmaxf(fminf(v*255,255),0)
    assert np.array_equal(img, expect)
