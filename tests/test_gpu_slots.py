"""k_shadow's lane slots (rtx.h RTX_OPT_SHADOW_SLOT): a shade point's light samples fill slots of
B lanes; each slot reduces in a fixed butterfly and lane 0 folds the slot sums into the point's
total in slot order (rtx_shadow.hip, the several-points-per-packet path).  For every B the ray
counts are exact and the frame does not depend on how points pack into packets (a chunked render
packs them differently); across B only the float association of the per-point sums changes."""
import numpy as np
import pytest

import conftest as C
import rtxpy
from rtxpy import abi

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["s6_amb", "s3_path2"])
def test_gpu_slot_sizes(name):
    scene, _, params, _ = C.load_config(name)
    frame = scene.frame(192, 108)
    r = rtxpy.Renderer(0)
    out = {}
    try:
        r.upload(scene)
        for b in (1, 2, 4, 8, 16, 32, 64):
            r.set_option(abi.RTX_OPT_SHADOW_SLOT, b)
            r.set_option(abi.RTX_OPT_CHUNK_TILES, 0)
            img, z = r.render(frame, params)
            s = r.stats()
            r.set_option(abi.RTX_OPT_CHUNK_TILES, 5)  # other packings of the same points
            img2, z2 = r.render(frame, params)
            s2 = r.stats()
            assert s2.chunks > 1
            assert np.array_equal(img2, img) and np.array_equal(z2, z), (name, b)
            out[b] = (img, z, (s.closest_rays, s.shadow_rays, s.shade_points))
    finally:
        r.close()
    ref_img, ref_z, ref_counts = out[64]
    for b, (img, z, counts) in out.items():
        assert counts == ref_counts, (name, b)
        assert np.array_equal(z, ref_z), (name, b)
        scale = np.maximum(np.abs(ref_img), 1e-3)
        assert (np.abs(img - ref_img) / scale).max() <= 2e-5, (name, b)
