#!/usr/bin/env python3
"""Deterministic stand-ins for the two meshes missing from the reference snapshot
(.MISSING_LARGE_BLOBS: meshes/dragon.stl, meshes/menger_sponge.stl), per SURVEY.md §8(d):

* dragon stand-in: level-7 subdivided icosphere (20*4^7 = 327,680 triangles),
  radius displaced by r = 1 + 0.15*sin(7x)*sin(9y)*sin(5z), outward CCW winding.
  Scene: scenes/scene5.json with the Mesh at position [0,-1,3], scale 0.8.
  (level 8 = 1,310,720 triangles brackets the full-resolution Stanford dragon.)
* Menger stand-in: level-4 sponge, interior faces culled (672,768 triangles),
  side 2.56 centred at the origin; scene6.json transform unchanged.

No RNG; float64 construction rounded once to float32.
"""
import argparse
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
GOLDEN = os.path.join(REPO, "tests", "golden")


def icosphere(level):
    t = (1.0 + 5 ** 0.5) / 2.0
    v = np.array([[-1, t, 0], [1, t, 0], [-1, -t, 0], [1, -t, 0], [0, -1, t], [0, 1, t], [0, -1, -t], [0, 1, -t],
                  [t, 0, -1], [t, 0, 1], [-t, 0, -1], [-t, 0, 1]], np.float64)
    v /= np.linalg.norm(v, axis=1, keepdims=True)
    f = np.array([[0, 11, 5], [0, 5, 1], [0, 1, 7], [0, 7, 10], [0, 10, 11], [1, 5, 9], [5, 11, 4], [11, 10, 2],
                  [10, 7, 6], [7, 1, 8], [3, 9, 4], [3, 4, 2], [3, 2, 6], [3, 6, 8], [3, 8, 9], [4, 9, 5],
                  [2, 4, 11], [6, 2, 10], [8, 6, 7], [9, 8, 1]], np.int64)
    for _ in range(level):
        nv = v.shape[0]
        edges = np.concatenate([f[:, [0, 1]], f[:, [1, 2]], f[:, [2, 0]]])
        key = np.minimum(edges[:, 0], edges[:, 1]) * (nv + 1) + np.maximum(edges[:, 0], edges[:, 1])
        uniq, inv = np.unique(key, return_inverse=True)
        a = uniq // (nv + 1)
        b = uniq % (nv + 1)
        mid = v[a] + v[b]
        mid /= np.linalg.norm(mid, axis=1, keepdims=True)
        v = np.concatenate([v, mid])
        m = inv.reshape(3, -1) + nv  # m01, m12, m20 per face
        m01, m12, m20 = m[0], m[1], m[2]
        f = np.concatenate([np.stack([f[:, 0], m01, m20], 1), np.stack([f[:, 1], m12, m01], 1),
                            np.stack([f[:, 2], m20, m12], 1), np.stack([m01, m12, m20], 1)])
    return v, f


def dragon_standin(level=7):
    v, f = icosphere(level)
    x, y, z = v[:, 0], v[:, 1], v[:, 2]
    r = 1.0 + 0.15 * np.sin(7 * x) * np.sin(9 * y) * np.sin(5 * z)
    v = v * r[:, None]
    tris = v[f]  # (n,3,3)
    # outward CCW: flip any face whose normal points inward
    n = np.cross(tris[:, 1] - tris[:, 0], tris[:, 2] - tris[:, 0])
    c = tris.mean(axis=1)
    flip = (n * c).sum(1) < 0
    tris[flip] = tris[flip][:, [0, 2, 1]]
    return tris.astype(np.float32)


def menger_cells(level):
    n = 3 ** level
    idx = np.arange(n)
    keep = np.ones((n, n, n), bool)
    for lv in range(level):
        d = (idx // 3 ** lv) % 3 == 1
        dx, dy, dz = np.meshgrid(d, d, d, indexing="ij")
        keep &= (dx.astype(int) + dy.astype(int) + dz.astype(int)) < 2
    return keep


def menger_standin(level=4, side=2.56):
    keep = menger_cells(level)
    n = keep.shape[0]
    h = side / n
    pad = np.zeros((n + 2, n + 2, n + 2), bool)
    pad[1:-1, 1:-1, 1:-1] = keep
    cells = np.argwhere(keep)
    quads = []
    # faces: axis, direction; quad corners (CCW seen from outside)
    for axis in range(3):
        for sgn in (-1, 1):
            off = np.zeros(3, int)
            off[axis] = sgn
            nb = pad[cells[:, 0] + 1 + off[0], cells[:, 1] + 1 + off[1], cells[:, 2] + 1 + off[2]]
            c = cells[~nb].astype(np.float64)
            u, w = [a for a in range(3) if a != axis]
            base = c.copy()
            if sgn > 0:
                base[:, axis] += 1
            p0 = base.copy()
            p1 = base.copy()
            p1[:, u] += 1
            p2 = base.copy()
            p2[:, u] += 1
            p2[:, w] += 1
            p3 = base.copy()
            p3[:, w] += 1
            q = np.stack([p0, p1, p2, p3], 1)
            # orientation: normal of (p1-p0)x(p3-p0) is +axis when (u,w) is a right-handed pair
            nrm = np.cross(q[:, 1] - q[:, 0], q[:, 3] - q[:, 0])[:, axis]
            wrong = np.sign(nrm) != sgn
            q[wrong] = q[wrong][:, [0, 3, 2, 1]]
            quads.append(q)
    q = np.concatenate(quads)
    tris = np.concatenate([q[:, [0, 1, 2]], q[:, [0, 2, 3]]])
    tris = tris * h - side / 2.0
    return tris.astype(np.float32)


def write_stl(path, tris):
    tris = np.ascontiguousarray(tris, np.float32).reshape(-1, 3, 3)
    rec = np.zeros(tris.shape[0], dtype=[("n", "<f4", 3), ("v", "<f4", (3, 3)), ("a", "<u2")])
    rec["v"] = tris
    with open(path, "wb") as fh:
        hdr = b"binary STL stand-in (rtx tools/standins.py)".ljust(80, b"\0")
        fh.write(hdr)
        fh.write(np.uint32(tris.shape[0]).tobytes())
        fh.write(rec.tobytes())


STANDINS = {
    "dragon_standin.stl": lambda: dragon_standin(7),
    "dragon_standin_l8.stl": lambda: dragon_standin(8),
    "menger_standin.stl": lambda: menger_standin(4),
}


def ensure_mesh(name, mesh_dir=None):
    mesh_dir = mesh_dir or os.path.join(GOLDEN, "meshes")
    os.makedirs(mesh_dir, exist_ok=True)
    path = os.path.join(mesh_dir, name)
    if not os.path.exists(path):
        tmp = path + ".tmp%d" % os.getpid()
        write_stl(tmp, STANDINS[name]())
        os.replace(tmp, path)
    return path


def standin_scene_json(which):
    """scene5/scene6 JSON with the Mesh entry pointed at the stand-in."""
    src = {"scene5": "scene5.json", "scene5_l8": "scene5.json", "scene6": "scene6.json"}[which]
    with open(os.path.join(GOLDEN, "scenes", src)) as fh:
        d = json.load(fh)
    for o in d["Objects"]:
        if o["type"] == "Mesh":
            p = o["parameters"]
            if which.startswith("scene5"):
                p["filename"] = "meshes/dragon_standin_l8.stl" if which == "scene5_l8" else "meshes/dragon_standin.stl"
                p["position"] = [0, -1, 3]
                p["scale"] = 0.8
            else:
                p["filename"] = "meshes/menger_standin.stl"
    return json.dumps(d, indent=1)


def ensure_scene(which):
    """Write tests/golden/scenes/<which>_standin.json and its mesh; return the scene path."""
    mesh = {"scene5": "dragon_standin.stl", "scene5_l8": "dragon_standin_l8.stl", "scene6": "menger_standin.stl"}[which]
    ensure_mesh(mesh)
    path = os.path.join(GOLDEN, "scenes", f"{which}_standin.json")
    text = standin_scene_json(which)
    if not os.path.exists(path) or open(path).read() != text:
        with open(path, "w") as fh:
            fh.write(text)
    return path


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("which", nargs="*", default=["scene5", "scene6"])
    a = ap.parse_args()
    for w in a.which:
        print(ensure_scene(w))
    sys.exit(0)
