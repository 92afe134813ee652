"""Debug: the far-camera frames (tests/test_gpu_frame.py far_camera_scene) under each trace walk
and tree frame, with a brute-force float32 closest hit (the reference's moller_trumbore order) for
the pixels where they differ."""
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

dist = float(sys.argv[1]) if len(sys.argv) > 1 else 2000.0
tmp = pathlib.Path(tempfile.mkdtemp())
scene = T.far_camera_scene(tmp, dist)
frame = scene.frame(96, 96)
params = rtxpy.params_from_args([], seed=1)
r = rtxpy.Renderer(0)
out = {}
for tw in (abi.RTX_WALK_BVH2, abi.RTX_WALK_W8):
    for fr in (abi.RTX_FRAME_AUTO, abi.RTX_FRAME_WORLD):
        opts = {abi.RTX_OPT_SHADOW_WALK: abi.RTX_WALK_W8, abi.RTX_OPT_TRACE_WALK: tw}
        params.count_traversal = 1
        rgb, z, st = T._render(r, scene, frame, params, fr, opts)
        out[(tw, fr)] = z
        print("walk", abi.WALK_NAMES[tw], "frame", fr, "rotated", st.tree_rotated, "far_closest", st.far_closest_rays,
              "far_shadow", st.far_shadow_rays, "closest", st.closest_rays)
r.close()
from rtxpy import oracle
params.count_traversal = 0
orgb, oz, _ = oracle.render(scene, frame, params)
A, B = out[(abi.RTX_WALK_BVH2, abi.RTX_FRAME_AUTO)], out[(abi.RTX_WALK_BVH2, abi.RTX_FRAME_WORLD)]
W = out[(abi.RTX_WALK_W8, abi.RTX_FRAME_AUTO)]
for key, z in out.items():
    print(key, "differs from the oracle on", int((z != oz).sum()))
diff = np.argwhere(A != B)
print("bvh2 auto vs world", len(diff))
for (py, px) in diff[:40]:
    print("   px", px, py, "auto", A[py, px], "world", B[py, px], "w8", W[py, px], "oracle", oz[py, px])
