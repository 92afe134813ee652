"""A render in several chunks (rtx_api.cpp rtx_render_common) is the one-chunk render, bit for bit.

A frame's 8x8 tiles are traced, lit and accumulated chunk by chunk: the shade-point buffers are
sized for a chunk from an estimate of shade points per tile, and a chunk whose shade points
overflow that estimate is halved and traced again, then the chunk size grows back by a quarter
per chunk that fits.  Pixels are independent, so neither the chunk boundaries nor the retries may
change a pixel or a ray count.  RTX_OPT_CHUNK_TILES caps the chunk size; RTX_OPT_SP_PER_TILE
forces a low estimate and with it the overflow-and-retry path.
"""
import numpy as np
import pytest

import conftest as C
import rtxpy
from rtxpy import abi

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["s5_path2", "s6_amb", "s3_path2", "s2_blinn_lin"])
def test_gpu_chunked_render_is_the_one_chunk_render(name):
    scene, _, params, _ = C.load_config(name)
    frame = scene.frame(256, 144)  # 576 tiles: more shade points than one overflowing chunk's retry margin
    tiles = ((frame.width + 7) // 8) * ((frame.height + 7) // 8)
    r = rtxpy.Renderer(0)
    try:
        r.upload(scene)
        a, za = r.render(frame, params)
        sa = r.stats()
        assert sa.chunks == 1
        r.set_option(abi.RTX_OPT_CHUNK_TILES, 3)
        b, zb = r.render(frame, params)
        sb = r.stats()
        assert sb.chunks == -(-tiles // 3)
        r.set_option(abi.RTX_OPT_CHUNK_TILES, 0)
        r.set_option(abi.RTX_OPT_SP_PER_TILE, 1)  # every chunk sized for 1 shade point per tile
        c, zc = r.render(frame, params)
        sc = r.stats()
        assert sc.chunks > 1
    finally:
        r.close()
    for img, z, s in ((b, zb, sb), (c, zc, sc)):
        assert np.array_equal(img, a) and np.array_equal(z, za), (name, s.chunks)
        assert (s.closest_rays, s.shadow_rays, s.shade_points) == (sa.closest_rays, sa.shadow_rays, sa.shade_points)


def test_gpu_chunk_options_reject_bad_values():
    r = rtxpy.Renderer(0)
    try:
        for opt, bad in ((abi.RTX_OPT_CHUNK_TILES, -1), (abi.RTX_OPT_SP_PER_TILE, -1), (abi.RTX_OPT_SP_PER_TILE, 1 << 21)):
            with pytest.raises(rtxpy.RtxError) as e:
                r.set_option(opt, bad)
            assert e.value.code == abi.RTX_ERR_ARG
    finally:
        r.close()

