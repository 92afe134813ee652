"""Debug: the drop-ins (INTEGRATION's -Ofast recipe and the -O2 build) with the constant light-sample
stream against the reference's own -Ofast and -O2 goldens"""
import os
import sys
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "c-raytracer_amd"), os.path.join(ROOT, "tools")]
import numpy as np  # noqa: E402
import conftest as C  # noqa: E402
import rtxpy  # noqa: E402
import standins  # noqa: E402

tmp = tempfile.mkdtemp()
for name in sys.argv[1:] or ["s1_amb", "s2_blinn_lin", "s3_path2", "s5_path2", "s6_amb"]:
    m = C.manifest()[name]
    if "standin" in m["scene"]:
        standins.ensure_scene(m["scene"].split("_standin")[0])
    fr = {}
    for exe in ("engine_dropin_rt", "engine_dropin"):
        out = os.path.join(tmp, exe + ".tif")
        cmd = [os.path.join(ROOT, "oracle", "_ref", exe), os.path.join("scenes", m["scene"]), out, str(m["width"]),
               str(m["height"]), "-f", "--rng", "const"] + m["flags"]
        p = subprocess.run(cmd, cwd=C.GOLDEN, capture_output=True, text=True, timeout=300)
        assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
        fr[exe] = rtxpy.read_tiff_raw(out)
    g_fast, g_o2 = C.golden_frame(name), C.golden_frame(name + "_o2")
    tol = C.floor_tolerance(m)
    for exe, (a, za) in fr.items():
        for gname, (b, zb) in (("ofast", g_fast), ("o2", g_o2)):
            ok, info = C.compare_const(a, za, b, zb, **tol)
            print(name, exe, "vs", gname, ok, info, flush=True)
    (a, za), (b, zb) = fr["engine_dropin_rt"], fr["engine_dropin"]
    ok, info = C.compare_const(a, za, b, zb, **tol)
    print(name, "rt vs O2 drop-in", ok, info, "floor", m["floor"], flush=True)
    d = np.abs(a - b).max(axis=2)
    tolv = 1e-4 * float(np.abs(b).max())
    bad = np.argwhere(d > tolv)
    print("   z equal", bool(np.array_equal(za, zb)), "bad px", len(bad), "max diff", float(d.max()),
          "rel of bad", np.quantile(d[d > tolv] / np.maximum(np.abs(b).max(axis=2)[d > tolv], 1e-9), [0, .5, 1]) if len(bad) else None)
    for (y, x) in bad[:12]:
        print("     px", x, y, "z", za[y, x], zb[y, x], "rgb", a[y, x], b[y, x])
