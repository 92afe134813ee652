"""Multi-device C-ABI (include/rtx.h rtx_group_*, csrc/rtx_group.cpp) on the one-GPU box.

A group of one device is the same render as rtx_render, bit for bit, with the same upload (the
BVHs built on device 0: device SAH and the 8-wide collapse, the same tree as a single context).
The gather's device kernels (rtx_tile_pack_device / rtx_tile_unpack_device, csrc/rtx_gather.hip)
are checked on one device: packing the shards of a rendered frame equals the host reference
records, and unpacking every shard rebuilds the frame.

A group of n > 1 shards runs here through the loopback transport (rtx_group_open_loopback: n
contexts on device 0).  That is the group's own orchestration at n = 2, 3 and 8: the scene built
once and copied to every context from one host thread each, one host thread per shard rendering
tiles t % n == r, the shard pack on each context, the unpack on the first and the statistics
summed over the shards; only the transport differs (a device-to-device copy instead of grouped
RCCL ncclSend / ncclRecv).  The frame must equal rtx_render's bit for bit, with equal summed ray
counts (render.c:349-352 is the parallel point the shards replace).

The RCCL calls themselves run through rtx_group_open_rccl_self: one device with a one-rank
communicator, whose whole frame is packed, sent to itself by the group's grouped ncclSend /
ncclRecv into a NaN-filled buffer and unpacked.

NOT exercised here: RCCL between distinct devices and peer copies (this box has one GPU, and the
driver's 8-GPU runs have been skipped for want of a node).  What stands in for them: the two
transports above, the record layout on the host (tests/test_gather.py), the same records
gathered over torch.distributed with gloo (tests/test_distributed.py), and the group line's
schema (tests/test_bench_cli.py).
"""
import os

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


@pytest.mark.parametrize("n", [2, 3, 8])
@pytest.mark.parametrize("name", ["s5_path2", "s6_amb", "s3_path2"])
def test_gpu_loopback_group_matches_render(name, n):
    """rtx_group_render at n shards (loopback transport) is rtx_render, bit for bit, with the ray
    counts of the shards summing to the single render's"""
    scene, frame, params, _ = C.load_config(name)
    r = rtxpy.Renderer(0)
    r.upload(scene)
    a, za = r.render(frame, params)
    sa = r.stats()
    r.close()
    g = rtxpy.Group([0], loopback=n)
    assert g.size() == n
    g.upload(scene)
    b, zb = g.render(frame, params)
    sb = g.stats()
    per = [g.device_stats(k) for k in range(n)]
    # a second frame through the same group (buffers reused, chunk sizes from the first)
    b2, zb2 = g.render(frame, params)
    g.close()
    assert np.array_equal(a, b) and np.array_equal(za, zb)
    assert np.array_equal(b, b2) and np.array_equal(zb, zb2)
    assert (sb.closest_rays, sb.shadow_rays, sb.shade_points) == (sa.closest_rays, sa.shadow_rays, sa.shade_points)
    assert sum(p.closest_rays for p in per) == sa.closest_rays
    assert sum(p.shadow_rays for p in per) == sa.shadow_rays
    assert sb.devices == n and sb.gather_ms > 0.0 and sb.transport == abi.RTX_TRANSPORT_LOOPBACK
    for k, p in enumerate(per):  # every context holds the tree built on the first one
        assert (p.wide_nodes, p.wide_entries, p.wide_depth, p.bvh_nodes, p.tree_rotated, p.shadow_walk) == \
            (sa.wide_nodes, sa.wide_entries, sa.wide_depth, sa.bvh_nodes, sa.tree_rotated, sa.shadow_walk)
        assert (p.upload_copy_ms > 0.0) == (k > 0)
        assert p.closest_rays > 0


@pytest.mark.parametrize("name", ["s5_path2", "s3_path2"])
def test_gpu_rccl_self_group_matches_render(name):
    """The group's RCCL code on one GPU (rtx_group_open_rccl_self): a one-rank communicator, the
    whole frame packed, sent to itself by the grouped ncclSend / ncclRecv into a NaN-filled buffer
    and unpacked over the frame.  The image is rtx_render's bit for bit only if RCCL delivered
    every record; the member reads its communicator back (count 1, rank 0, its own device)."""
    scene, frame, params, _ = C.load_config(name)
    r = rtxpy.Renderer(0)
    r.upload(scene)
    a, za = r.render(frame, params)
    sa = r.stats()
    r.close()
    g = rtxpy.Group([0], rccl_self=True)
    assert g.size() == 1
    m = g.member(0)
    assert (m["comm_count"], m["comm_rank"], m["comm_device"], m["device"]) == (1, 0, 0, 0)
    assert m["transport"] == abi.RTX_TRANSPORT_RCCL_SELF
    g.upload(scene)
    b, zb = g.render(frame, params)
    sb = g.stats()
    b2, zb2 = g.render(frame, params)
    g.close()
    assert np.array_equal(a, b) and np.array_equal(za, zb)
    assert np.array_equal(b, b2) and np.array_equal(zb, zb2)
    assert (sb.closest_rays, sb.shadow_rays) == (sa.closest_rays, sa.shadow_rays)
    assert sb.gather_ms > 0.0 and sb.transport == abi.RTX_TRANSPORT_RCCL_SELF


def test_gpu_loopback_group_sharding_of_a_tall_ragged_frame():
    """a frame whose tile count is not a multiple of n (and smaller than n in one dimension)"""
    scene, _, params, _ = C.load_config("s1_amb")
    frame = scene.frame(20, 61)
    r = rtxpy.Renderer(0)
    r.upload(scene)
    a, za = r.render(frame, params)
    r.close()
    for n in (5, 16):  # 3 x 8 = 24 tiles over 5 shards; 16 shards, some with 1 tile
        g = rtxpy.Group([0], loopback=n)
        g.upload(scene)
        b, zb = g.render(frame, params)
        g.close()
        assert np.array_equal(a, b) and np.array_equal(za, zb), n


def test_gpu_bench_group_line_on_the_loopback_group(tmp_path):
    """bench.py's device-group mode (main_group: --gpus N without torchrun) run end to end on the
    one-GPU box through the loopback group: the line's per-device rays add up to the frame's, every
    shard has kernel times, and it reports one GPU with N shards (a rehearsal, not a scaling line)"""
    import json
    import subprocess
    import sys
    cmd = [sys.executable, os.path.join(C.ROOT, "bench.py"), "--gpus", "3", "--loopback", "--scene", "scene3",
           "--width", "192", "--height", "108", "--spp", "2", "--steps", "2", "--warmup", "1", "--no-cpu-baseline"]
    p = subprocess.run(cmd, cwd=C.ROOT, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    out = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
    assert out["n_gpus"] == 1 and out["shards"] == 3 and out["value"] > 0
    g = out["group"]
    assert g["rtx_group_size"] == 3 and g["rccl_devices"] == 0 and g["transport"].startswith("loopback")
    assert [d["device"] for d in g["devices"]] == [0, 1, 2]
    assert sum(d["rays"] for d in g["devices"]) == out["config"]["rays_per_frame"]
    assert all(d["kernel_ms"] > 0 for d in g["devices"]) and g["gather_ms"] > 0
    assert g["upload"]["peer_copy_ms"][0] == 0.0 and min(g["upload"]["peer_copy_ms"][1:]) > 0
    assert out["roofline"]["kernel"] == "k_shadow" and out["roofline"]["device"] == 0
    # the line validates itself: members read back, the one-context frame equal to
    # the gathered one in rays and bits
    v = out["validation"]
    assert v["ok"], v["checks"]
    assert [m["device"] for m in v["members"]] == [0, 0, 0] and all(m["comm_count"] == 0 for m in v["members"])
    assert all(m["transport"] == 2 and m["pci_bus_id"] for m in v["members"])
    assert v["rays_per_frame"] == v["one_gpu_frame_rays"] and sum(v["rays_per_frame"]) == out["config"]["rays_per_frame"]
    assert v["gathered_frame_sha256_16"] == v["one_gpu_frame_sha256_16"]
