"""Measure: ray-count differences of the GPU path against the -O2 reference goldens and the oracle on
every frame case tests/test_gpu_parity.py checks (to set its tolerances to what the code achieves)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "c-raytracer_amd"), os.path.join(ROOT, "tools")]
import conftest as C  # noqa: E402
import rtxpy  # noqa: E402
from rtxpy import abi, oracle  # noqa: E402
import test_gpu_parity as T  # noqa: E402

r = rtxpy.Renderer(0)
for name in T.CONST:
    scene, frame, params, m = C.load_config(name)
    rgb, z, st = T.render(r, scene, frame, params)
    print("ieee", name, params.gi, st.closest_rays - m["closest_rays_o2"], st.shadow_rays - m["shadow_rays_o2"],
          m["closest_rays_o2"], m["shadow_rays_o2"], flush=True)
for rng in (abi.RTX_RNG_COUNTER, abi.RTX_RNG_STRAT):
    for name in ["s1_path2", "s3_path2", "s4_path2_blinn", "s5_path2", "s6_path2", "s2_amb"]:
        scene, frame, params, m = C.load_config(name)
        params.rng = rng
        params.seed = 12345
        if params.gi == abi.RTX_GI_PATH:
            params.samples = 8
        rgb, z, st = T.render(r, scene, frame, params)
        _, _, (nc, ns) = oracle.render(scene, frame, params)
        print("counter", rng, name, st.closest_rays - nc, st.shadow_rays - ns, nc, ns, flush=True)
for args in ([], ["-g", "path", "-n", "3"], ["-b", "0"], ["-s", "blinn", "-l", "none"]):
    scene = rtxpy.Scene.parse(T.EDGE_SCENE)
    frame = scene.frame(40, 24)
    params = rtxpy.params_from_args(args, rng=abi.RTX_RNG_COUNTER, seed=3)
    rgb, z, st = T.render(r, scene, frame, params)
    _, _, (nc, ns) = oracle.render(scene, frame, params)
    print("edge", args, st.closest_rays - nc, st.shadow_rays - ns, nc, ns, flush=True)
r.close()
