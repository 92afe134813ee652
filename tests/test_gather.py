"""Tile records of the multi-device gather (include/rtx.h rtx_tile_*, csrc/rtx_tiles.h), on the
host: the index math rtx_group_render's pack / unpack kernels share (rtx_gather.hip).

Every pixel of a frame belongs to exactly one shard, a shard's records follow its tiles in
increasing tile order with 64 row-major pixels each, pixels outside the frame pack as zeros,
and unpacking every shard rebuilds the frame bit for bit -- for ragged frame sizes and any
shard count.  The same layout is what the torch.distributed bench path packs (rtxpy/dist.py).
"""
import numpy as np
import pytest

import rtxpy
from rtxpy.dist import rank_tiles, tile_pixel_index

SIZES = [(8, 8), (13, 5), (64, 24), (37, 29), (1, 1), (120, 7)]


@pytest.mark.parametrize("w,h", SIZES)
@pytest.mark.parametrize("n", [1, 2, 3, 8])
def test_pack_unpack_round_trip(w, h, n):
    rng = np.random.default_rng(w * 131 + h * 7 + n)
    rgb = rng.random((h, w, 3), dtype=np.float32)
    z = rng.random((h, w), dtype=np.float32) * 10
    out_rgb = np.full_like(rgb, -1.0)
    out_z = np.full_like(z, -1.0)
    lib = rtxpy.rtx_lib()
    total = 0
    for r in range(n):
        rec = rtxpy.tile_pack(rgb, z, r, n)
        tiles = rank_tiles(w, h, r, n)
        assert rec.shape == (len(tiles) * 64, 4) == (lib.rtx_tile_pack_count(w, h, r, n), 4)
        idx = tile_pixel_index(w, h, tiles).reshape(-1)  # the bench path's layout: same order
        inside = idx >= 0
        assert np.array_equal(rec[inside, :3], rgb.reshape(-1, 3)[idx[inside]])
        assert np.array_equal(rec[inside, 3], z.reshape(-1)[idx[inside]])
        assert not rec[~inside].any()
        rtxpy.tile_unpack(rec, out_rgb, out_z, r, n)
        total += int(inside.sum())
    assert total == w * h
    assert np.array_equal(out_rgb, rgb) and np.array_equal(out_z, z)


def test_pack_count_edges():
    lib = rtxpy.rtx_lib()
    assert lib.rtx_tile_pack_count(16, 16, 0, 1) == 4 * 64
    assert lib.rtx_tile_pack_count(16, 16, 3, 4) == 64
    assert lib.rtx_tile_pack_count(16, 16, 4, 8) == 0      # more shards than tiles
    assert lib.rtx_tile_pack_count(16, 16, 2, 2) == 0      # offset outside the stride
    with pytest.raises(rtxpy.RtxError):
        rtxpy.tile_pack(np.zeros((8, 8, 3), np.float32), np.zeros((8, 8), np.float32), 1, 1)


def test_group_open_fails_cleanly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by tests/test_gpu_group.py")
    with pytest.raises(rtxpy.RtxError) as e:
        rtxpy.Group([0])
    assert e.value.code == rtxpy.abi.RTX_ERR_NODEV
    with pytest.raises(rtxpy.RtxError) as e:
        rtxpy.Group([0, 0])
    assert e.value.code == rtxpy.abi.RTX_ERR_ARG
