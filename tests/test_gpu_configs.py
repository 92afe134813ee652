"""Parity at the BASELINE.json workloads themselves (the frames bench.py and the scaling runs time).

Each config renders on the GPU through the C-ABI at its full size, flags and spp, with the
default RNG (counter-based i.i.d. light samples, seed 1, as bench.py).  The oracle
(oracle/restate.c, bit-exact with the reference built at -O2, tests/test_oracle.py) renders an evenly spaced sample of the same frame's 8x8
tiles with the same RNG stream, and the GPU pixels of those tiles must agree within SURVEY
§8(c)'s tolerances (conftest.compare_const):
    hit mask <= 0.01 % of pixels (+1 px); |dz| <= 1e-4*max(z,1) on >= 99.9 % of hit pixels;
    per-channel |d rgb| <= 1e-4*max(ref) on >= 99.5 % of pixels; relL1 <= 1e-2.
A second GPU render of only the sampled tiles (the multi-GPU sharding path) must reproduce the
full-frame pixels bit for bit and count exactly the oracle's cast_ray / is_light_blocked calls
for those tiles.

  configs[1]  scene3 1920x1080 -g path -n 16
  configs[2]  scene5 (dragon stand-in) 1920x1080 -g path -n 64    (bench.py's workload)
  configs[3]  scene5 1920x1080 -n 256, one rank's tile shard of an 8-GPU split
  configs[4]  scene6 (Menger stand-in) 3840x2160 -g path -n 128 on one GPU
(configs[0], scene1 512x512 ambient, is the reference's CPU case: test_cpu_config0 below and
 the 512x512 frame in test_gpu_config0.)
"""
import os

import numpy as np
import pytest

import conftest as C
import rtxpy
from rtxpy import abi, oracle
from rtxpy.dist import rank_tiles, tile_pixel_index

CONFIGS = {
    # name: (scene, width, height, spp, oracle tile stride, GPU shard (offset, stride) or None)
    # strides: 1 tile in 53 / 47 / 1048 (of the shard's, 1 in 131) / 199
    "k2_scene3_1080p_n16": ("scene3", 1920, 1080, 16, 53, None),
    "k3_scene5_1080p_n64": ("scene5", 1920, 1080, 64, 47, None),
    "k4_scene5_1080p_n256_shard0of8": ("scene5", 1920, 1080, 256, 8 * 131, (0, 8)),
    "k5_scene6_2160p_n128": ("scene6", 3840, 2160, 128, 199, None),
}


def load(name):
    import standins
    if name in ("scene5", "scene6"):
        standins.ensure_scene(name)
        return rtxpy.Scene.load(os.path.join(C.SCENES, f"{name}_standin.json"), base_dir=C.GOLDEN)
    return rtxpy.Scene.load(os.path.join(C.SCENES, f"{name}.json"), base_dir=C.GOLDEN)


def params_for(spp, offset=0, stride=1):
    p = rtxpy.params_from_args(["-g", "path", "-n", str(spp)], seed=1)
    p.rng = abi.RTX_RNG_COUNTER  # bench.py's mode (the library default: i.i.d. like rand_flt)
    p.tile_offset, p.tile_stride = offset, stride
    return p


def sample_index(w, h, offset, stride):
    idx = tile_pixel_index(w, h, rank_tiles(w, h, offset, stride)).reshape(-1)
    return idx[idx >= 0]


@pytest.fixture(scope="module")
def renderer():
    r = rtxpy.Renderer(0)
    yield r
    r.close()


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", list(CONFIGS))
def test_gpu_baseline_config_vs_oracle(renderer, cfg):
    scene_name, w, h, spp, ostride, shard = CONFIGS[cfg]
    scene = load(scene_name)
    frame = scene.frame(w, h)
    off, stride = shard or (0, 1)
    renderer.upload(scene)
    rgb = np.zeros((h, w, 3), np.float32)
    z = np.zeros((h, w), np.float32)
    rgb, z = renderer.render(frame, params_for(spp, off, stride), rgb, z)
    full = renderer.stats()
    assert np.isfinite(rgb).all() and (rgb >= 0).all()
    if shard is None:
        assert (z > 0).any()
    # the oracle's sample: tiles t = off (mod ostride), a subset of the GPU's shard
    assert ostride % stride == 0
    o_rgb, o_z, (nc, ns) = oracle.render(scene, frame, params_for(spp, off, ostride))
    idx = sample_index(w, h, off, ostride)
    g_rgb, g_z = rgb.reshape(-1, 3)[idx], z.reshape(-1)[idx]
    r_rgb, r_z = o_rgb.reshape(-1, 3)[idx], o_z.reshape(-1)[idx]
    ok, info = C.compare_const(g_rgb[:, None, :], g_z[:, None], r_rgb[:, None, :], r_z[:, None])
    info["sample_px"] = int(idx.size)
    print(cfg, info, "gpu rays", full.closest_rays, full.shadow_rays, "ms", round(full.kernel_ms, 1))
    assert ok, info
    # the whole frame's (or shard's) depth and hit mask against the oracle's primary hits: z does not
    # depend on the light samples (render.c:342, 364), so every pixel is checked at full size
    pz, _ = oracle.primary(scene, frame)
    sidx = sample_index(w, h, off, stride)
    gz, oz = z.reshape(-1)[sidx], pz.reshape(-1)[sidx]
    hit_mismatch = float(((gz > 0) != (oz > 0)).mean())
    both = (gz > 0) & (oz > 0)
    z_ok = float((np.abs(gz[both] - oz[both]) / np.maximum(oz[both], 1.0) <= 1e-4).mean())
    print(cfg, "frame-wide", {"px": int(sidx.size), "hit_mismatch": hit_mismatch, "z_ok": z_ok,
                              "z_equal": float((gz == oz).mean())})
    assert hit_mismatch <= 1e-4 + 1.0 / sidx.size and z_ok >= 0.999, (hit_mismatch, z_ok)
    # the sharded render of exactly the oracle's tiles: bit-identical pixels, exact ray counts
    s_rgb, s_z = renderer.render(frame, params_for(spp, off, ostride))
    st = renderer.stats()
    assert np.array_equal(s_rgb.reshape(-1, 3)[idx], g_rgb) and np.array_equal(s_z.reshape(-1)[idx], g_z)
    # cast_ray calls are exact; is_light_blocked calls may differ by a few shade points' lights:
    # a path-GI direction (acosf / sinf / cosf, render.c:281-283) rounded 1 ulp apart by OCML and
    # glibc can flip a grazing hit or the is_outside sign of one child in ~1e6 (measured: one
    # point of 300 lights in 80.5 M shadow rays on k3).  Bound: 2e-5 of the count.
    assert st.closest_rays == nc
    assert abs(st.shadow_rays - ns) <= 2e-5 * ns, (st.shadow_rays, ns)


@pytest.mark.gpu
def test_gpu_config0_scene1_512(renderer):
    """configs[0]: scene1 512x512 ambient, const RNG: the whole frame against the oracle."""
    scene = load("scene1")
    frame = scene.frame(512, 512)
    p = rtxpy.params_from_args([])
    p.rng = abi.RTX_RNG_CONST
    renderer.upload(scene)
    rgb, z = renderer.render(frame, p)
    st = renderer.stats()
    o_rgb, o_z, (nc, ns) = oracle.render(scene, frame, p)
    ok, info = C.compare_const(rgb, z, o_rgb, o_z)
    assert ok, info
    assert (st.closest_rays, st.shadow_rays) == (nc, ns)


def test_cpu_config_sample_indices():
    """The oracle samples are subsets of the GPU shards they are compared with."""
    for cfg, (_, w, h, _, ostride, shard) in CONFIGS.items():
        off, stride = shard or (0, 1)
        a = set(sample_index(w, h, off, ostride).tolist())
        b = set(sample_index(w, h, off, stride).tolist())
        assert a and a <= b, cfg


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,shards", [("k4_scene5_1080p_n256_shard0of8", 8), ("k5_scene6_2160p_n128", 8)])
def test_gpu_eight_gpu_configs_through_the_group_path(renderer, cfg, shards):
    """configs[3] (scene5 1080p -n 256) and configs[4] (scene6 2160p -n 128) are quoted for 8 GPUs:
    their whole frame through the device group's path at 8 shards (the loopback transport:
    scene copies, one host thread per shard, tile pack / unpack, statistics; RCCL aside) is the
    one-device frame bit for bit, with the shards' ray counts summing to its counts"""
    scene_name, w, h, spp, _, _ = CONFIGS[cfg]
    scene = load(scene_name)
    frame = scene.frame(w, h)
    p = params_for(spp)
    renderer.upload(scene)
    a, za = renderer.render(frame, p)
    sa = renderer.stats()
    g = rtxpy.Group([0], loopback=shards)
    try:
        g.upload(scene)
        b, zb = g.render(frame, p)
        sb = g.stats()
        per = [g.device_stats(k) for k in range(shards)]
    finally:
        g.close()
    assert np.array_equal(a, b) and np.array_equal(za, zb), cfg
    assert (sb.closest_rays, sb.shadow_rays) == (sa.closest_rays, sa.shadow_rays)
    assert sum(s.shadow_rays for s in per) == sa.shadow_rays
    # the interleaved tile deal balances the shards: every shard's rays within 10 % of the mean
    rays = np.array([s.closest_rays + s.shadow_rays for s in per], np.float64)
    assert rays.max() <= 1.1 * rays.mean() and rays.min() >= 0.9 * rays.mean(), rays / rays.mean()
