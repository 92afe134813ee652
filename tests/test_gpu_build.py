"""GPU BVH builder (csrc/rtx_build.hip via rtx_set_builder(RTX_BUILD_LBVH_GPU)).

Closest-hit answers do not depend on the tree (up to exact ties), so frames rendered over the
GPU-built LBVH must match the reference goldens exactly as well as frames over the host SAH
tree do, and the z-buffer must equal the SAH render's; shadow transmittance products may be
formed in another order (1-ulp-level colour differences, inside the frame tolerance).
"""
import numpy as np
import pytest

import conftest as C
import rtxpy
from rtxpy import abi

pytestmark = pytest.mark.gpu

CONFIGS = ["s1_amb", "s3_path2", "s5_path2", "s6_amb", "st_amb"]


@pytest.fixture(scope="module")
def renderer():
    r = rtxpy.Renderer(0)
    yield r
    r.close()


def render(r, builder, scene, frame, params):
    r.set_builder(builder)
    r.upload(scene)
    rgb, z = r.render(frame, params)
    return rgb, z, r.stats()


@pytest.mark.parametrize("name", CONFIGS)
def test_gpu_lbvh_frames_match(renderer, name):
    scene, frame, params, m = C.load_config(name)
    a, za, sa = render(renderer, abi.RTX_BUILD_SAH_HOST, scene, frame, params)
    b, zb, sb = render(renderer, abi.RTX_BUILD_LBVH_GPU, scene, frame, params)
    assert sb.builder == abi.RTX_BUILD_LBVH_GPU and sa.builder == abi.RTX_BUILD_SAH_HOST
    assert sb.bvh_depth <= 63 and sb.build_ms > 0
    assert np.array_equal(za, zb), name  # closest hits do not depend on the tree
    assert (sa.closest_rays, sa.shadow_rays) == (sb.closest_rays, sb.shadow_rays)
    ref_rgb, ref_z = C.golden_frame(name + "_o2")
    ok, info = C.compare_const(b, zb, ref_rgb, ref_z)
    assert ok, info
    assert np.abs(a - b).max() <= 1e-5 * max(1.0, float(np.abs(a).max())), name


def test_gpu_lbvh_deterministic_and_tiny_scenes(renderer):
    scene, frame, params, _ = C.load_config("s5_path2")
    a, za, st = render(renderer, abi.RTX_BUILD_LBVH_GPU, scene, frame, params)
    b, zb, _ = render(renderer, abi.RTX_BUILD_LBVH_GPU, scene, frame, params)
    assert np.array_equal(a, b) and np.array_equal(za, zb)
    assert st.bvh_nodes == st.bvh_prims - 1  # single-primitive leaves (the default): a full binary tree
    # scene1: 3 spheres + a light -> with leaves of up to 4 primitives, a single-leaf root
    renderer.set_option(abi.RTX_OPT_BVH_LEAF, 4)
    scene, frame, params, _ = C.load_config("s1_amb")
    try:
        a, za, st = render(renderer, abi.RTX_BUILD_LBVH_GPU, scene, frame, params)
    finally:
        renderer.set_option(abi.RTX_OPT_BVH_LEAF, 1)
    assert st.bvh_nodes == 0
    o_rgb, o_z = C.golden_frame("s1_amb_o2")
    ok, info = C.compare_const(a, za, o_rgb, o_z)
    assert ok, info
    with pytest.raises(rtxpy.RtxError):
        renderer.set_builder(7)
    renderer.set_builder(abi.RTX_BUILD_SAH_HOST)
