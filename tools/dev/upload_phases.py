"""Development check: upload phases of a scene, three uploads in one process (measurement build
via RTX_LIBRTX=lib/var/meas/librtx.so prints per-phase times)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "c-raytracer_amd"), os.path.join(ROOT, "tools")]
import rtxpy
import standins
which = sys.argv[1] if len(sys.argv) > 1 else "scene5"
scene = rtxpy.Scene.load(standins.ensure_scene(which), base_dir=os.path.join(ROOT, "tests", "golden"))
t0 = time.perf_counter()
r = rtxpy.Renderer(0)
print(f"open: {1e3 * (time.perf_counter() - t0):.1f} ms", file=sys.stderr, flush=True)
for i in range(3):
    t0 = time.perf_counter()
    r.upload(scene)
    dt = time.perf_counter() - t0
    s = r.stats()
    print(f"upload {i}: wall {dt * 1e3:.1f} ms, build_ms {s.build_ms:.1f}, frame_ms {s.frame_ms:.1f}", file=sys.stderr, flush=True)
