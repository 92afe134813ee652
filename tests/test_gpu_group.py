"""Multi-device C-ABI (include/rtx.h rtx_group_*, csrc/rtx_group.cpp) on the one-GPU box.

A group of one device is the same render as rtx_render, bit for bit, with the same upload (the
BVHs built on device 0: device SAH and the 8-wide collapse, the same tree as a single context).
The gather's device kernels (rtx_tile_pack_device / rtx_tile_unpack_device, csrc/rtx_gather.hip)
are checked on one device: packing the shards of a rendered frame equals the host reference
records, and unpacking every shard rebuilds the frame.

NOT exercised here: a group of n > 1 devices, i.e. the peer copies of the built trees
(hipMemcpyPeer in rtx_group_upload_scene) and the grouped RCCL ncclSend / ncclRecv of the
shards.  This box has one GPU, and the driver's multi-GPU runs have so far been skipped (no 8-GPU
node), so that path has never run.  What stands in for it: the shard deal and record layout on
the host (tests/test_gather.py), the same records gathered over torch.distributed with gloo
(tests/test_distributed.py), and the group line's schema (tests/test_bench_cli.py).
"""
import numpy as np
import pytest

import conftest as C
import rtxpy
from rtxpy import abi

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["s5_path2", "st_amb", "s6_amb"])
def test_gpu_group_of_one_matches_render(name):
    scene, frame, params, _ = C.load_config(name)
    r = rtxpy.Renderer(0)
    r.upload(scene)
    a, za = r.render(frame, params)
    sa = r.stats()
    r.close()
    g = rtxpy.Group([0])
    g.upload(scene)
    b, zb = g.render(frame, params)
    sb = g.stats()
    g.close()
    assert np.array_equal(a, b) and np.array_equal(za, zb)
    assert (sa.closest_rays, sa.shadow_rays) == (sb.closest_rays, sb.shadow_rays)
    assert sb.devices == 1 and sb.gather_ms == 0.0
    assert sb.wide_nodes == sa.wide_nodes and sb.bvh_nodes == sa.bvh_nodes
    # the group's upload is the single context's: device SAH + device 8-wide collapse
    assert sb.builder == sa.builder == abi.RTX_BUILD_SAH_GPU
    assert (sb.shadow_walk, sb.wide_entries, sb.wide_depth, sb.tree_rotated) == \
        (sa.shadow_walk, sa.wide_entries, sa.wide_depth, sa.tree_rotated)


def test_gpu_group_rejects_shard_params_and_bad_devices():
    scene, frame, params, _ = C.load_config("s1_amb")
    g = rtxpy.Group([0])
    with pytest.raises(rtxpy.RtxError) as e:
        g.render(frame, params)  # before upload
    assert e.value.code == abi.RTX_ERR_STATE
    g.upload(scene)
    params.tile_offset, params.tile_stride = 1, 2
    with pytest.raises(rtxpy.RtxError) as e:
        g.render(frame, params)
    assert e.value.code == abi.RTX_ERR_ARG
    g.close()
    with pytest.raises(rtxpy.RtxError) as e:
        rtxpy.Group([0, 0])
    assert e.value.code == abi.RTX_ERR_ARG
    with pytest.raises(rtxpy.RtxError):
        rtxpy.Group([0, 4096])


def test_gpu_tile_pack_unpack_device():
    import torch
    scene, frame, params, _ = C.load_config("s3_path2")
    r = rtxpy.Renderer(0)
    r.upload(scene)
    rgb, z = r.render(frame, params)
    h, w = z.shape
    d_rgb = torch.from_numpy(rgb.copy()).cuda()
    d_z = torch.from_numpy(z.copy()).cuda()
    o_rgb = torch.zeros_like(d_rgb)
    o_z = torch.zeros_like(d_z)
    lib = rtxpy.rtx_lib()
    n = 3
    torch.cuda.synchronize()
    for k in range(n):
        cnt = lib.rtx_tile_pack_count(w, h, k, n)
        d_rec = torch.empty((cnt, 4), dtype=torch.float32, device="cuda")
        rtxpy._check(lib.rtx_tile_pack_device(r._ctx, d_rgb.data_ptr(), d_z.data_ptr(), w, h, k, n, d_rec.data_ptr(),
                                              None))
        host = rtxpy.tile_pack(rgb, z, k, n)
        assert np.array_equal(d_rec.cpu().numpy(), host)
        rtxpy._check(lib.rtx_tile_unpack_device(r._ctx, d_rec.data_ptr(), w, h, k, n, o_rgb.data_ptr(), o_z.data_ptr(),
                                                None))
    torch.cuda.synchronize()
    assert np.array_equal(o_rgb.cpu().numpy(), rgb) and np.array_equal(o_z.cpu().numpy(), z)
    r.close()
