"""k_shadow's cone cull (rtx.h RTX_OPT_SHADOW_CULL, rtx_shadow.hip cone_clear, rtx_api.cpp
build_cull): a packet of one shade point's samples of one emitter skips the 8-wide walk when the
cone from the point around the emitter's bounding sphere meets none of the bounding spheres of the
tree's second level.  Every shadow ray of the packet lies in that cone, so a skipped walk is one
that could reach no primitive: the image, the depth buffer and the ray counts are the same bit for
bit with the cull on and off (is_light_blocked, render.c:126-134, finds nothing in the tree either
way).  The counting render reports how many rays skipped their walk (rtx_stats.shadow_cone_clear).
"""
import os

import numpy as np
import pytest

import conftest as C
import rtxpy
from rtxpy import abi
from test_gpu_configs import load

pytestmark = pytest.mark.gpu


def render_both(scene, frame, params, slot=0, frame_opt=abi.RTX_FRAME_AUTO, on=1):
    out = {}
    r = rtxpy.Renderer(0)
    try:
        r.set_option(abi.RTX_OPT_TREE_FRAME, frame_opt)
        r.upload(scene)
        r.set_option(abi.RTX_OPT_SHADOW_SLOT, slot)
        for cull in (on, 0):
            r.set_option(abi.RTX_OPT_SHADOW_CULL, cull)
            for count in (0, 1):
                p = rtxpy.default_params(**{f: getattr(params, f) for f, _ in abi.Params._fields_})
                p.count_traversal = count
                rgb, z = r.render(frame, p)
                out[(min(cull, 1), count)] = (rgb, z, r.stats())
    finally:
        r.close()
    return out


def check(out, want_clear):
    rgb0, z0, s0 = out[(0, 0)]
    for key, (rgb, z, s) in out.items():
        assert np.array_equal(rgb, rgb0) and np.array_equal(z, z0), key
        assert (s.closest_rays, s.shadow_rays, s.shade_points) == (s0.closest_rays, s0.shadow_rays, s0.shade_points), key
    on, off = out[(1, 1)][2], out[(0, 1)][2]
    assert off.shadow_cone_clear == 0
    if want_clear:
        assert on.shadow_cone_clear > 0
        # the cleared rays' walks are gone: fewer box tests, no other change in what was tested
        assert on.shadow_node_visits < off.shadow_node_visits
    return on.shadow_cone_clear / max(1, on.shadow_rays)


@pytest.mark.parametrize("name", ["s5_path2", "s3_path2", "s2_blinn_lin", "s6_amb"])
def test_gpu_cone_cull_is_invisible(name):
    scene, frame, params, _ = C.load_config(name)
    out = render_both(scene, frame, params, slot=64)  # 64-lane packets: one point per packet
    frac = check(out, want_clear=False)
    print(name, "cleared", round(frac, 4))


@pytest.mark.parametrize("slot", [0, 16, 4])
def test_gpu_cone_cull_on_the_bench_scene(slot):
    """scene5 with the dragon stand-in (bench.py's scene, a smaller frame): most floor and wall
    points see the light past the dragon, so most packets skip the walk; the frame is the same.
    slot 0: the automatic layout (64-lane packets of one point, cone_mask); 16 / 4: lane slots of
    several points per packet (RTX_OPT_SHADOW_CULL 2, cone_mask_lane: a packet skips when all its
    lanes' points are clear)"""
    scene = load("scene5")
    frame = scene.frame(320, 180)
    params = rtxpy.params_from_args(["-g", "path", "-n", "4"], seed=1)
    params.rng = abi.RTX_RNG_COUNTER
    out = render_both(scene, frame, params, slot=slot, on=2 if slot else 1)
    frac = check(out, want_clear=True)
    print("scene5 slot", slot, "cleared", round(frac, 4))
    assert frac > 0.3
    if slot:  # option 1 leaves the lane slots walking
        r = rtxpy.Renderer(0)
        try:
            r.upload(scene)
            r.set_option(abi.RTX_OPT_SHADOW_SLOT, slot)
            p = rtxpy.default_params(**{f: getattr(params, f) for f, _ in abi.Params._fields_})
            p.count_traversal = 1
            r.render(frame, p)
            assert r.stats().shadow_cone_clear == 0
        finally:
            r.close()


@pytest.mark.parametrize("frame_opt", [abi.RTX_FRAME_AUTO, abi.RTX_FRAME_WORLD])
def test_gpu_cone_cull_in_the_rotated_frame(frame_opt):
    """scene6's Menger stand-in builds its trees in a rotated frame: the spheres are formed in it
    and moved to world space (x = R^T x' + c); with 64-lane packets the cull runs, and the frame is
    the same as without it in both tree frames"""
    scene = load("scene6")
    frame = scene.frame(160, 90)
    params = rtxpy.params_from_args(["-g", "path", "-n", "2"], seed=1)
    params.rng = abi.RTX_RNG_COUNTER
    out = render_both(scene, frame, params, slot=64, frame_opt=frame_opt)
    frac = check(out, want_clear=False)
    print("scene6 frame", frame_opt, "cleared", round(frac, 4))


def three_emitter_scene(tmp_path):
    """the bench scene with two more emitters: a second sphere light and a triangle light (its
    bounding sphere is its padded world box's), 428 samples per point, so packets of one emitter
    and packets straddling two (which take the per-lane emitter path and are never culled)"""
    import json
    import shutil
    load("scene5")  # writes the dragon stand-in
    with open(os.path.join(C.SCENES, "scene5_standin.json")) as fh:
        d = json.load(fh)
    os.makedirs(tmp_path / "meshes", exist_ok=True)
    shutil.copy(os.path.join(C.GOLDEN, "meshes", "dragon_standin.stl"), tmp_path / "meshes" / "dragon_standin.stl")
    d["Objects"].append({"type": "Sphere", "parameters": {"material": 2, "epsilon": 0.0003, "position": [5.5, -3.5, 1.5],
                                                          "radius": 0.3, "lights": 64}})
    d["Objects"].append({"type": "Triangle", "parameters": {"material": 2, "epsilon": 0.0001, "lights": 64,
                                                            "vertex_1": [-0.4, -4.6, 2.6], "vertex_2": [0.4, -4.6, 2.6],
                                                            "vertex_3": [0.0, -4.6, 3.3]}})
    path = tmp_path / "three.json"
    path.write_text(json.dumps(d))
    return rtxpy.Scene.load(str(path), base_dir=str(tmp_path))


def test_gpu_cone_cull_with_three_emitters(tmp_path):
    """a point's cone_mask holds one bit per emitter: with three emitters (two spheres, one
    triangle) the frame is the same with the cull on and off, and some rays are culled"""
    scene = three_emitter_scene(tmp_path)
    frame = scene.frame(160, 90)
    params = rtxpy.params_from_args(["-g", "path", "-n", "2"], seed=3)
    params.rng = abi.RTX_RNG_COUNTER
    out = render_both(scene, frame, params)
    frac = check(out, want_clear=True)
    print("three emitters cleared", round(frac, 4))
