"""Debug: sphere tests of the closest-hit BVH2 walk from a far camera, per tree frame"""
import os
import sys
import pathlib
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "c-raytracer_amd"), os.path.join(ROOT, "tools")]
import numpy as np  # noqa: E402
import rtxpy  # noqa: E402
from rtxpy import abi  # noqa: E402
import test_gpu_frame as T  # noqa: E402

tmp = pathlib.Path(tempfile.mkdtemp())
r = rtxpy.Renderer(0)
for dist in (3.0, 60.0, 2000.0):
    scene = T.far_camera_scene(tmp, dist)
    frame = scene.frame(96, 96)
    params = rtxpy.params_from_args(["-b", "0"], seed=1)
    params.count_traversal = 1
    for tw in (abi.RTX_WALK_BVH2, abi.RTX_WALK_W8):
        for fr in (abi.RTX_FRAME_AUTO, abi.RTX_FRAME_WORLD):
            for leaf in (1,):
                r.set_option(abi.RTX_OPT_BVH_LEAF, leaf)
                opts = {abi.RTX_OPT_SHADOW_WALK: abi.RTX_WALK_W8, abi.RTX_OPT_TRACE_WALK: tw}
                rgb, z, st = T._render(r, scene, frame, params, fr, opts)
                print(dist, abi.WALK_NAMES[tw], "rot" if st.tree_rotated else "world", "leaf", leaf,
                      "closest sph tests", st.sphere_tests - st.shadow_sphere_tests,
                      "tri", st.tri_tests - st.shadow_tri_tests, "nodes", st.node_visits - st.shadow_node_visits,
                      "bvh nodes", st.bvh_nodes, "depth", st.bvh_depth, "z<1999.5", int(((z > 0) & (z < dist - 0.5)).sum()))
r.close()
