"""The 4-wide shadow-walk BVH (rtx_device.h RTX_W_STACK, rtx_shadow.hip shadow_walk4) against the
threaded BVH2 walk it replaced (RTX_WIDE=0 keeps the BVH2 walk, the fallback for trees too deep
for the wide walk's LDS stacks).

Both walks answer is_light_blocked (render.c:126-134, accel.c:360-387) exactly: the same boxes,
quantised the same way, cull the same primitives, and any-hit needs no visit order.  Only the
order in which transparent blockers multiply a ray's transmittance may differ (leaves are met
in another order), so z-buffers and ray counts are identical and colours agree to float
rounding; both stay inside the reference goldens' tolerance.
"""
import numpy as np
import pytest

import conftest as C
import rtxpy
from rtxpy import abi

pytestmark = pytest.mark.gpu

CONFIGS = ["s1_amb", "s3_path2", "s4_path2_blinn", "s5_path2", "s6_amb", "st_amb", "st2_r2"]


@pytest.fixture(scope="module")
def renderer():
    r = rtxpy.Renderer(0)
    yield r
    r.close()


def render(r, scene, frame, params):
    r.upload(scene)
    rgb, z = r.render(frame, params)
    return rgb, z, r.stats()


@pytest.mark.parametrize("name", CONFIGS)
def test_gpu_wide_walk_matches_bvh2_walk(renderer, name, monkeypatch):
    scene, frame, params, _ = C.load_config(name)
    renderer.set_builder(abi.RTX_BUILD_SAH_HOST)
    a, za, sa = render(renderer, scene, frame, params)
    assert sa.wide_nodes > 0 and 1 <= sa.wide_depth <= 13
    monkeypatch.setenv("RTX_WIDE", "0")
    b, zb, sb = render(renderer, scene, frame, params)
    assert sb.wide_nodes == 0 and sb.wide_depth == 0
    assert np.array_equal(za, zb), name
    assert (sa.closest_rays, sa.shadow_rays) == (sb.closest_rays, sb.shadow_rays)
    assert np.abs(a - b).max() <= 1e-5 * max(1.0, float(np.abs(b).max())), name
    ref_rgb, ref_z = C.golden_frame(name + "_o2")
    for rgb, z in ((a, za), (b, zb)):
        ok, info = C.compare_const(rgb, z, ref_rgb, ref_z)
        assert ok, (name, info)


@pytest.mark.parametrize("leaf", ["2", "5"])
def test_gpu_wide_walk_multi_primitive_leaves(renderer, leaf, monkeypatch):
    """Leaves of several primitives (RTX_BVH_LEAF > 1): the wide tree's leaf slots hold the
    BVH2 leaves whole and the walk tests their primitives in order."""
    monkeypatch.setenv("RTX_BVH_LEAF", leaf)
    for name in ("s5_path2", "st_amb"):
        scene, frame, params, _ = C.load_config(name)
        renderer.set_builder(abi.RTX_BUILD_SAH_HOST)
        a, za, sa = render(renderer, scene, frame, params)
        assert sa.wide_nodes > 0
        ref_rgb, ref_z = C.golden_frame(name + "_o2")
        ok, info = C.compare_const(a, za, ref_rgb, ref_z)
        assert ok, (name, leaf, info)


def test_gpu_wide_walk_counts(renderer):
    """count_traversal on the wide walk: four box tests per node fetch at most, every fetch is a
    global (no LDS top), and the wave's leaf rounds never exceed its node steps' leaf slots."""
    scene, frame, params, _ = C.load_config("s5_path2")
    renderer.set_builder(abi.RTX_BUILD_SAH_HOST)
    renderer.upload(scene)
    p = rtxpy.default_params(**{f: getattr(params, f) for f, _ in abi.Params._fields_})
    p.count_traversal = 1
    renderer.render(frame, p)
    st = renderer.stats()
    assert st.shadow_rays > 0 and st.shadow_box_tests > 0
    assert st.shadow_global_box_tests == st.shadow_box_tests
    assert st.shadow_wave_steps * 64 * 4 >= st.shadow_box_tests
    assert 0 < st.shadow_leaf_rounds <= 4 * st.shadow_wave_steps
