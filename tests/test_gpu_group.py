"""Multi-device C-ABI (include/rtx.h rtx_group_*, csrc/rtx_group.cpp) on the one-GPU box.

A group of one device is the same render as rtx_render, bit for bit (the BVH built once on the
host, uploaded through the group path).  The gather's device kernels (rtx_tile_pack_device /
rtx_tile_unpack_device, csrc/rtx_gather.hip) are checked on one device: packing the shards of
a rendered frame equals the host reference records, and unpacking every shard rebuilds the
frame; the RCCL send/recv between them is exercised by the driver's multi-GPU runs (the
torch.distributed bench path gathers the same records, tests/test_distributed.py).
"""
import numpy as np
import pytest

import conftest as C
import rtxpy
from rtxpy import abi

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["s5_path2", "st_amb"])
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
