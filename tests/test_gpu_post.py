"""GPU postprocess (csrc/rtx_post.hip through rtx_postprocess*) against the reference's own
postprocess() (tests/golden/post, made by tools/make_post_goldens.py from oracle/_ref/post_dump).

The bar is bit-exact: brighten, mist and the DoF normalisation are the same float operations
in the same order, and the DoF gather sums every destination pixel's contributions in the
reference scatter's source order.
"""
import json
import os
import subprocess

import numpy as np
import pytest

import conftest as C
import rtxpy

pytestmark = pytest.mark.gpu

POST = os.path.join(C.GOLDEN, "post")
MANIFEST = json.load(open(os.path.join(POST, "manifest.json")))


@pytest.fixture(scope="module")
def renderer():
    r = rtxpy.Renderer(0)
    yield r
    r.close()


@pytest.mark.parametrize("case", sorted(MANIFEST))
def test_gpu_postprocess_bit_exact(renderer, case):
    m = MANIFEST[case]
    inp = np.load(os.path.join(POST, m["input"] + ".npz"))
    ref = np.load(os.path.join(POST, case + ".npy"))
    out = renderer.postprocess(rtxpy.post_from_args(m["flags"]), inp["rgb_in"], inp["z_in"])
    bad = ~((out == ref) | (np.isnan(out) & np.isnan(ref)))
    assert not bad.any(), (case, int(bad.sum()), float(np.nanmax(np.abs(out - ref))))


def test_gpu_postprocess_device_buffers(renderer):
    import torch
    m = MANIFEST["combo"]
    inp = np.load(os.path.join(POST, m["input"] + ".npz"))
    h, w = inp["z_in"].shape
    d_rgb = torch.from_numpy(inp["rgb_in"].copy()).cuda()
    d_z = torch.from_numpy(inp["z_in"].copy()).cuda()
    s = torch.cuda.current_stream()
    renderer.postprocess_device(rtxpy.post_from_args(m["flags"]), w, h, d_rgb.data_ptr(), d_z.data_ptr(), s.cuda_stream)
    assert np.array_equal(d_rgb.cpu().numpy(), np.load(os.path.join(POST, "combo.npy")))


def test_gpu_postprocess_noop_and_errors(renderer):
    inp = np.load(os.path.join(POST, "synth_a.npz"))
    out = renderer.postprocess(rtxpy.post_from_args([]), inp["rgb_in"], inp["z_in"])
    assert np.array_equal(out, inp["rgb_in"])
    bad = rtxpy.post_from_args(["--mist", "1", "2", "lin", "0", "0", "0"])
    bad.mist_falloff = 7
    with pytest.raises(rtxpy.RtxError):
        renderer.postprocess(bad, inp["rgb_in"], inp["z_in"])


def test_gpu_postprocess_cli_matches_reference_u8(tmp_path):
    """lib/postprocess (host/post_main.c): raw TIFF in, 8-bit TIFF out, same bytes as the
    reference postprocessor's save_image on the same input and flags."""
    m = MANIFEST["combo"]
    inp = np.load(os.path.join(POST, m["input"] + ".npz"))
    src, dst = str(tmp_path / "in.tif"), str(tmp_path / "out.tif")
    rtxpy.write_tiff(src, inp["rgb_in"], inp["z_in"], raw=True)
    exe = os.path.join(rtxpy.LIB_DIR, "postprocess")
    p = subprocess.run([exe, src, dst] + m["flags"], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
    from rtxpy.tiffread import read_tiff
    assert np.array_equal(read_tiff(dst)["rgb"], np.load(os.path.join(POST, "combo_u8.npy")))
