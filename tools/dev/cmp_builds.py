"""Development check: traversal counts of the s6_amb golden config over the host and device SAH
builds, twice each (tree-frame auto / world)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "c-raytracer_amd"), os.path.join(ROOT, "tools")]
import numpy as np
import conftest as C
import rtxpy
from rtxpy import abi
scene, frame, params, _ = C.load_config(sys.argv[1] if len(sys.argv) > 1 else "s6_amb")
params.count_traversal = 1
r = rtxpy.Renderer(0)
F = ("closest_rays", "shadow_rays", "node_visits", "tri_tests", "shadow_tri_tests", "shadow_box_tests", "shadow_wave_steps",
     "wide_nodes", "wide_entries")
imgs = {}
for fr in (abi.RTX_FRAME_AUTO, abi.RTX_FRAME_WORLD):
    r.set_option(abi.RTX_OPT_TREE_FRAME, fr)
    for b in (abi.RTX_BUILD_SAH_HOST, abi.RTX_BUILD_SAH_GPU):
        r.set_builder(b)
        r.set_option(abi.RTX_OPT_SHADOW_WALK, abi.RTX_WALK_W8)
        r.upload(scene)
        for k in range(2):
            rgb, z = r.render(frame, params)
            s = r.stats()
            imgs[(fr, b, k)] = (rgb, z)
            print(fr, b, k, " ".join(f"{f}={getattr(s, f)}" for f in F), flush=True)
base = imgs[(abi.RTX_FRAME_WORLD, abi.RTX_BUILD_SAH_HOST, 0)]
for key, (rgb, z) in imgs.items():
    print(key, "rgb==", np.array_equal(rgb, base[0]), "z==", np.array_equal(z, base[1]), "maxdiff", float(np.abs(rgb - base[0]).max()))
