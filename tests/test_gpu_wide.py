"""The shadow walks over their BVH layouts (include/rtx.h RTX_WALK_*, rtx_shadow.hip):

  RTX_WALK_W8    8-wide compressed BVH (rtx_device.h DW8, shadow_walk8), the default
  RTX_WALK_BVH2  threaded BVH2 (shadow_walk): small scenes (its top levels fit LDS) and trees the
                 8-wide layout cannot hold
  RTX_WALK_LINEAR no tree: every bounded object tested one by one (tiny scenes, <= 8 objects)

All answer is_light_blocked (render.c:126-134, accel.c:360-387) exactly: each culls only with
conservative boxes and any-hit needs no visit order.  Only the order in which transparent
blockers multiply a ray's transmittance may differ (leaves are met in another order), so
z-buffers and ray counts are identical and colours agree to float rounding; every walk stays
inside the reference goldens' tolerance.
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


@pytest.fixture(autouse=True)
def _defaults(renderer):
    yield
    renderer.set_builder(abi.RTX_BUILD_SAH_GPU)
    renderer.set_option(abi.RTX_OPT_SHADOW_WALK, abi.RTX_WALK_AUTO)
    renderer.set_option(abi.RTX_OPT_BVH_LEAF, 1)
    renderer.set_option(abi.RTX_OPT_SHADOW_LDS_STACK, 8)
    renderer.set_option(abi.RTX_OPT_TREE_FRAME, abi.RTX_FRAME_AUTO)


def render(r, scene, frame, params, walk=abi.RTX_WALK_AUTO):
    r.set_option(abi.RTX_OPT_SHADOW_WALK, walk)
    r.upload(scene)
    rgb, z = r.render(frame, params)
    return rgb, z, r.stats()


SMALL = {"s1_amb", "s3_path2", "st_amb", "st2_r2"}  # threaded BVH2 within the LDS top (<= 1024 primitives)


def auto_walk(scene, name):
    nb = sum(1 for o in scene.objects() if o.type != abi.RTX_PLANE)
    if nb <= abi.RTX_SHADOW_LINEAR_MAX:
        return abi.RTX_WALK_LINEAR
    return abi.RTX_WALK_BVH2 if name in SMALL else abi.RTX_WALK_W8


@pytest.mark.parametrize("name", CONFIGS)
def test_gpu_walks_agree(renderer, name):
    scene, frame, params, _ = C.load_config(name)
    a, za, sa = render(renderer, scene, frame, params, abi.RTX_WALK_W8)
    assert sa.shadow_walk == abi.RTX_WALK_W8 and sa.wide_nodes > 0 and sa.wide_depth >= 1
    assert sa.wide_entries >= 8 * sa.wide_nodes
    ref_rgb, ref_z = C.golden_frame(name + "_o2")
    # RTX_WALK_AUTO: no tree for tiny scenes, the LDS-resident threaded BVH2 for small ones, the
    # 8-wide tree otherwise
    _, _, sd = render(renderer, scene, frame, params)
    assert sd.shadow_walk == auto_walk(scene, name), name
    for walk in (abi.RTX_WALK_BVH2, abi.RTX_WALK_LINEAR):
        if walk == abi.RTX_WALK_LINEAR and len(scene.objects()) > 64:
            continue  # one by one over a mesh: correct, but not a walk anyone would run
        b, zb, sb = render(renderer, scene, frame, params, walk)
        assert sb.shadow_walk == walk
        assert np.array_equal(za, zb), (name, walk)
        assert (sa.closest_rays, sa.shadow_rays) == (sb.closest_rays, sb.shadow_rays)
        assert np.abs(a - b).max() <= 1e-5 * max(1.0, float(np.abs(b).max())), (name, walk)
        ok, info = C.compare_const(b, zb, ref_rgb, ref_z)
        assert ok, (name, walk, info)
    ok, info = C.compare_const(a, za, ref_rgb, ref_z)
    assert ok, (name, info)


@pytest.mark.parametrize("name", ["s5_path2", "s6_amb", "s4_path2_blinn"])
def test_gpu_w8_lane_stack_spill(renderer, name):
    """Trees deeper than the LDS lane stack walk on with the deeper entries in HBM: with one LDS
    entry every wide node below the second level spills (the path the depth-cliff fallback of
    the round-2 4-wide walk never had); the frame is bit-identical to the all-LDS walk and matches the
    reference."""
    scene, frame, params, _ = C.load_config(name)
    params.rng = abi.RTX_RNG_COUNTER
    a, za, sa = render(renderer, scene, frame, params)
    renderer.set_option(abi.RTX_OPT_SHADOW_LDS_STACK, 1)
    b, zb, sb = render(renderer, scene, frame, params)
    assert sb.shadow_walk == abi.RTX_WALK_W8 and sb.wide_depth > 2
    assert np.array_equal(a, b) and np.array_equal(za, zb)
    assert (sa.closest_rays, sa.shadow_rays) == (sb.closest_rays, sb.shadow_rays)
    from rtxpy import oracle
    o_rgb, o_z, _ = oracle.render(scene, frame, params)
    ok, info = C.compare_const(b, zb, o_rgb, o_z)
    assert ok, info


@pytest.mark.parametrize("leaf", [2, 5])
def test_gpu_wide_walk_multi_primitive_leaves(renderer, leaf):
    """BVH2 leaves of several primitives (RTX_OPT_BVH_LEAF > 1): the 8-wide collapse opens them
    into one slot per primitive (boxes from the records), the threaded BVH2 keeps them whole."""
    renderer.set_option(abi.RTX_OPT_BVH_LEAF, leaf)
    for name in ("s5_path2", "st_amb"):
        scene, frame, params, _ = C.load_config(name)
        ref_rgb, ref_z = C.golden_frame(name + "_o2")
        for walk in (abi.RTX_WALK_W8, abi.RTX_WALK_BVH2):
            a, za, sa = render(renderer, scene, frame, params, walk)
            assert sa.shadow_walk == walk and (sa.wide_nodes > 0) == (walk == abi.RTX_WALK_W8)
            ok, info = C.compare_const(a, za, ref_rgb, ref_z)
            assert ok, (name, leaf, walk, info)


def test_gpu_w8_walk_counts(renderer):
    """count_traversal on the 8-wide walk: at most eight box tests per node fetch, and leaf
    rounds no more than the node steps' leaf slots."""
    scene, frame, params, _ = C.load_config("s5_path2")
    renderer.upload(scene)
    p = rtxpy.default_params(**{f: getattr(params, f) for f, _ in abi.Params._fields_})
    p.count_traversal = 1
    renderer.render(frame, p)
    st = renderer.stats()
    assert st.shadow_walk == abi.RTX_WALK_W8
    assert st.shadow_rays > 0 and st.shadow_box_tests > 0
    assert st.shadow_global_box_tests == st.shadow_box_tests
    assert st.shadow_wave_steps * 64 * 8 >= st.shadow_box_tests
    assert 0 < st.shadow_leaf_rounds <= 8 * st.shadow_wave_steps


def test_gpu_options_reject_bad_values(renderer):
    for opt, bad in ((abi.RTX_OPT_SHADOW_WALK, 4), (abi.RTX_OPT_SHADOW_WALK, 1), (abi.RTX_OPT_TREE_FRAME, 2),
                     (abi.RTX_OPT_BVH_LEAF, 0), (abi.RTX_OPT_SPSORT, 2),
                     (abi.RTX_OPT_SHADOW_SLOT, 3), (abi.RTX_OPT_SHADOW_GRAB, 0), (abi.RTX_OPT_SHADOW_LDS_STACK, 9),
                     (99, 1)):
        with pytest.raises(rtxpy.RtxError) as e:
            renderer.set_option(opt, bad)
        assert e.value.code == abi.RTX_ERR_ARG
