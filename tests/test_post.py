"""Postprocess host side, no GPU: flag parsing with the reference's argv
semantics, the raw-TIFF reader against a file libtiff wrote (the reference engine's -f output)
and against our own writer, and the golden fixtures' provenance.

Fixtures: tests/golden/post (tools/make_post_goldens.py): the reference's own postprocess()
(oracle/_ref/post_dump, built from /root/reference/src/postprocess + src/core) on raw TIFFs.
"""
import json
import os
import subprocess

import numpy as np
import pytest

import conftest as C
import rtxpy
from rtxpy import abi

POST = os.path.join(C.GOLDEN, "post")
MANIFEST = json.load(open(os.path.join(POST, "manifest.json")))
DUMP = os.path.join(C.ROOT, "oracle", "_ref", "post_dump")


def test_post_flags_parse_like_reference():
    p = rtxpy.post_from_args(["-b", "1.7"])
    assert p.brighten == 1 and p.brighten_factor == np.float32(1.7) and p.dof == 0 and p.mist == 0
    p = rtxpy.post_from_args(["--dof", "0.9", "-1.5"])
    assert p.dof == abi.RTX_DOF_SCALE_BIAS and (p.dof_scale, p.dof_bias) == (np.float32(0.9), np.float32(-1.5))
    p = rtxpy.post_from_args(["--dof-camera", "1.5", "1.0", "4.0"])
    assert p.dof == abi.RTX_DOF_CAMERA and (p.aperture, p.focal_length, p.plane_in_focus) == (1.5, 1.0, 4.0)
    # --dof wins over --dof-camera (postproc.c:49-68: else-if)
    assert rtxpy.post_from_args(["--dof-camera", "1", "2", "3", "--dof", "1", "2"]).dof == abi.RTX_DOF_SCALE_BIAS
    for name, code in (("quad", abi.RTX_FALLOFF_QUAD), ("lin", abi.RTX_FALLOFF_LIN),
                       ("inv-quad", abi.RTX_FALLOFF_INV_QUAD)):
        p = rtxpy.post_from_args(["--mist", "2", "5", name, "0.5", "0.6", "0.7"])
        assert p.mist == 1 and p.mist_falloff == code and list(p.mist_color) == [np.float32(v) for v in (.5, .6, .7)]
    # too few arguments after a flag: ignored, as argv_check_with_args does
    assert rtxpy.post_from_args(["--mist", "2", "5", "quad"]).mist == 0
    assert rtxpy.post_from_args(["--dof", "1"]).dof == 0
    with pytest.raises(rtxpy.RtxError) as e:
        rtxpy.post_from_args(["--mist", "2", "5", "cubic", "0", "0", "0"])
    assert "Unrecognized falloff type [cubic]" in str(e.value)


def test_raw_tiff_reader_reads_libtiff_output():
    rgb, z = rtxpy.read_tiff_raw(os.path.join(POST, "s1_raw.tif"))
    ref = np.load(os.path.join(POST, "s1_raw.npz"))
    assert np.array_equal(rgb, ref["rgb_in"]) and np.array_equal(z, ref["z_in"])
    assert (z == 0).any() and (z > 0).any()  # background and geometry


def test_raw_tiff_round_trip_and_errors(tmp_path):
    rng = np.random.default_rng(3)
    for h, w in ((1, 1), (7, 5), (48, 64)):
        rgb = rng.standard_normal((h, w, 3)).astype(np.float32)
        z = rng.uniform(0, 9, (h, w)).astype(np.float32)
        p = str(tmp_path / f"r{h}x{w}.tif")
        rtxpy.write_tiff(p, rgb, z, raw=True)
        r2, z2 = rtxpy.read_tiff_raw(p)
        assert np.array_equal(r2, rgb) and np.array_equal(z2, z)
    p8 = str(tmp_path / "u8.tif")
    rtxpy.write_tiff(p8, rgb)
    with pytest.raises(rtxpy.RtxError):  # 8-bit TIFF: image.c:48 "Expected 32 bits per sample"
        rtxpy.read_tiff_raw(p8)
    with pytest.raises(rtxpy.RtxError):
        rtxpy.read_tiff_raw(str(tmp_path / "missing.tif"))


def test_post_fixture_inputs_cover_the_cases():
    for case, m in MANIFEST.items():
        assert os.path.exists(os.path.join(POST, case + ".npy")), case
        inp = np.load(os.path.join(POST, m["input"] + ".npz"))
        out = np.load(os.path.join(POST, case + ".npy"))
        assert out.shape == inp["rgb_in"].shape
        assert np.isfinite(out).all() and m["nan"] == 0


@pytest.mark.skipif(not os.path.exists(DUMP), reason="oracle/_ref not built (no /root/reference here)")
def test_post_fixtures_reproduce_from_reference(tmp_path):
    """The committed outputs are what the reference's own postprocess() produces today."""
    for case in ("dof_mid", "combo", "s1_mist"):
        m = MANIFEST[case]
        inp = np.load(os.path.join(POST, m["input"] + ".npz"))
        src = str(tmp_path / "in.tif")
        rtxpy.write_tiff(src, inp["rgb_in"], inp["z_in"], raw=True)
        dump = str(tmp_path / "out.f32")
        subprocess.run([DUMP, src, dump] + m["flags"], check=True, capture_output=True)
        raw = np.fromfile(dump, dtype=np.uint8)
        w, h = np.frombuffer(raw[:8].tobytes(), dtype=np.uint32)
        out = np.frombuffer(raw[8:].tobytes(), dtype=np.float32).reshape(h, w, 3)
        assert np.array_equal(out, np.load(os.path.join(POST, case + ".npy"))), case
