"""Host glue (librtxscene): scene JSON loader, STL ingest, image plane, CLI flags, TIFF writer.

Mirrors the reference's scene.c / object.c / image.c / render.c:61-116 behaviour
and error conditions (the reference calls error() -> exit(1); here the call
returns RTX_ERR_SCENE / RTX_ERR_IO with the same message).
"""
import json
import os
import struct

import numpy as np
import pytest

import conftest as C
import rtxpy
from rtxpy import abi
from rtxpy.tiffread import read_tiff

SCENE1 = os.path.join(C.SCENES, "scene1.json")


def load_json(name):
    with open(os.path.join(C.SCENES, name)) as fh:
        return json.load(fh)


def test_hash_djb_matches_reference_constants():
    # constants from the reference's switch statements (render.c:76-110, scene.c:201-340, system.c:45-61)
    expect = {"phong": 187940251, "blinn": 175795714, "ambient": 354625309, "path": 2088095368, "none": 2087865487,
              "lin": 193412846, "sqr": 193433013, "norm": 2087865883, "uniform": 3226203393,
              "checkerboard": 2234799246, "brick": 176032948, "noisy periodic": 202158024, "Sphere": 3324768284,
              "Triangle": 103185867, "Plane": 232719795, "Mesh": 2088783990, "max": 193414065, "real": 2088303039,
              "cpu": 193416643, "sin": 193433777, "saw": 193433504, "triangle": 837065195, "square": 2144888260}
    for k, v in expect.items():
        assert rtxpy.hash_djb(k) == v, k


def test_scene1_contents():
    s = rtxpy.Scene.load(SCENE1)
    objs = s.objects()
    assert [o.type for o in objs] == [abi.RTX_SPHERE] * 3 + [abi.RTX_PLANE, abi.RTX_SPHERE]
    assert s.emitters() == [4]
    assert objs[4].num_lights == 200 and objs[0].num_lights == 0
    # default epsilons: sphere r*0.0003 (object.c:235-236), plane 1e-6 unless given
    d = load_json("scene1.json")
    for o, j in zip(objs, d["Objects"]):
        p = j["parameters"]
        if "epsilon" in p:
            assert o.epsilon == np.float32(p["epsilon"])
        elif o.type == abi.RTX_SPHERE:
            assert o.epsilon == np.float32(np.float32(p["radius"]) * np.float32(0.0003))
    m = s.materials()
    assert all(mm.emittant == (np.linalg.norm(mm.ke) > 1e-6) for mm in m)
    cam = s.desc.camera
    v = np.array(cam.vectors)
    assert np.allclose(np.linalg.norm(v[:2], axis=1), 1, atol=1e-6)
    assert np.allclose(v[2], np.cross(v[0], v[1]), atol=1e-6)


def test_mesh_triangles_inserted_in_place_with_template_header():
    s = rtxpy.Scene.load(os.path.join(C.SCENES, "scenetest.json"), base_dir=C.GOLDEN)
    d = load_json("scenetest.json")
    types = [o.type for o in s.objects()]
    n_mesh = len(types) - (len(d["Objects"]) - 1)
    mesh_idx = [i for i, j in enumerate(d["Objects"]) if j["type"] == "Mesh"][0]
    assert types[mesh_idx:mesh_idx + n_mesh] == [abi.RTX_TRIANGLE] * n_mesh
    with open(os.path.join(C.GOLDEN, d["Objects"][mesh_idx]["parameters"]["filename"]), "rb") as fh:
        fh.seek(80)
        assert struct.unpack("<I", fh.read(4))[0] == n_mesh


def test_triangle_postinit_edges_normal_epsilon():
    s = rtxpy.Scene.parse(json.dumps(minimal_scene([{"type": "Triangle", "parameters": {
        "material": 0, "vertex_1": [0, 0, 0], "vertex_2": [2, 0, 0], "vertex_3": [0, 1, 0]}}])))
    t = [o for o in s.objects() if o.type == abi.RTX_TRIANGLE][0]
    assert list(t.e1) == [2, 0, 0] and list(t.e2) == [0, 1, 0]
    assert np.allclose(t.n, [0, 0, 1])
    expect = np.float32(0.003) * np.float32(np.power(np.float32(0.5 * 2 * 1 * 1), 0.75))
    assert abs(t.epsilon - expect) < 1e-9


def minimal_scene(extra_objects, emitter=True, **over):
    d = {
        "Camera": {"position": [0, 0, -1], "vector_x": [1, 0, 0], "vector_y": [0, 1, 0], "fov": 90,
                   "focal_length": 1},
        "Materials": [
            {"id": 0, "ks": [0, 0, 0], "ka": [0, 0, 0], "kr": [0, 0, 0], "kt": [0, 0, 0], "ke": [0, 0, 0],
             "shininess": 1, "refractive_index": 1, "texture": {"type": "uniform", "color": [1, 1, 1]}},
            {"id": 1, "ks": [0, 0, 0], "ka": [0, 0, 0], "kr": [0, 0, 0], "kt": [0, 0, 0], "ke": [1, 1, 1],
             "shininess": 1, "refractive_index": 1, "texture": {"type": "uniform", "color": [1, 1, 1]}}],
        "Objects": list(extra_objects) + ([{"type": "Sphere", "parameters": {
            "material": 1, "position": [0, 3, 3], "radius": 0.5, "lights": 4}}] if emitter else []),
    }
    d.update(over)
    return d


@pytest.mark.parametrize("mutate,msg", [
    (lambda d: d.pop("Camera"), "Expected token [Camera] of type [Object]"),
    (lambda d: d["Camera"].pop("fov"), "Expected token [Camera] to contain 5 elements."),
    (lambda d: d["Camera"].update(fov=180), "Expected camera fov"),
    (lambda d: d.update(Materials=[]), "Expected token [Materials] to contain nonzero element count"),
    (lambda d: d["Materials"][0].update(ks=[0, 0]), "Expected token [ks] of length [3]"),
    (lambda d: d["Materials"][0]["texture"].update(type="wood"), "Unrecognized token [wood] in texture"),
    (lambda d: d["Objects"][0]["parameters"].update(material=9), "Failed to get material id [9]."),
    (lambda d: d["Objects"].append({"type": "Plane", "parameters": {"material": 1, "position": [0, 0, 0],
                                                                    "normal": [0, 1, 0]}}),
     "Plane cannot be emittant"),
])
def test_scene_errors_like_reference(mutate, msg):
    d = minimal_scene([])
    mutate(d)
    with pytest.raises(rtxpy.RtxError) as e:
        rtxpy.Scene.parse(json.dumps(d), name="t.json")
    assert e.value.code == abi.RTX_ERR_SCENE
    assert msg in str(e.value)


def test_scene_requires_an_emitter():
    with pytest.raises(rtxpy.RtxError) as e:
        rtxpy.Scene.parse(json.dumps(minimal_scene([{"type": "Sphere", "parameters": {
            "material": 0, "position": [0, 0, 1], "radius": 1}}], emitter=False)))
    assert "Expected non-zero number of emittant objects" in str(e.value)


def test_stl_ascii_and_missing_rejected(tmp_path):
    ascii_stl = tmp_path / "a.stl"
    ascii_stl.write_bytes(b"solid x\n" + b"\0" * 100)
    obj = {"type": "Mesh", "parameters": {"material": 0, "filename": "a.stl", "position": [0, 0, 0],
                                          "rotation": [0, 0, 0], "scale": 1}}
    with pytest.raises(rtxpy.RtxError) as e:
        rtxpy.Scene.parse(json.dumps(minimal_scene([obj])), base_dir=str(tmp_path))
    assert "does not use binary encoding" in str(e.value)
    obj["parameters"]["filename"] = "missing.stl"
    with pytest.raises(rtxpy.RtxError) as e:
        rtxpy.Scene.parse(json.dumps(minimal_scene([obj])), base_dir=str(tmp_path))
    assert e.value.code == abi.RTX_ERR_IO


def test_stl_transform_zyx(tmp_path):
    tri = np.array([[1, 0, 0, 0, 1, 0, 0, 0, 1]], np.float32)
    rtxpy.write_stl(str(tmp_path / "t.stl"), tri)
    rot = [0.3, -0.7, 1.1]
    obj = {"type": "Mesh", "parameters": {"material": 0, "filename": "t.stl", "position": [1, 2, 3],
                                          "rotation": rot, "scale": 2}}
    s = rtxpy.Scene.parse(json.dumps(minimal_scene([obj])), base_dir=str(tmp_path))
    t = s.objects()[0]
    x, y, z = rot
    Rz = np.array([[np.cos(z), -np.sin(z), 0], [np.sin(z), np.cos(z), 0], [0, 0, 1]])
    Ry = np.array([[np.cos(y), 0, np.sin(y)], [0, 1, 0], [-np.sin(y), 0, np.cos(y)]])
    Rx = np.array([[1, 0, 0], [0, np.cos(x), -np.sin(x)], [0, np.sin(x), np.cos(x)]])
    R = Rz @ Ry @ Rx  # object.c:550-562 is the ZYX product
    v = tri.reshape(3, 3) @ R.T * 2 + [1, 2, 3]
    assert np.allclose([list(t.p0), list(t.p1), list(t.p2)], v, atol=1e-5)


def test_scale_norm_and_factor():
    s = rtxpy.Scene.load(os.path.join(C.SCENES, "scene3.json"))
    s2 = rtxpy.Scene.load(os.path.join(C.SCENES, "scene3.json"), scale="2.0")
    a, b = s.objects(), s2.objects()
    for o, p in zip(a, b):
        if o.type == abi.RTX_SPHERE:
            assert np.allclose(np.array(p.p0), 2 * np.array(o.p0)) and p.radius == 2 * o.radius
            assert p.epsilon == np.float32(2 * o.epsilon)
        if o.type == abi.RTX_PLANE:
            assert np.isclose(p.d, 2 * o.d, atol=1e-5)
    assert s2.desc.camera.focal_length == 2 * s.desc.camera.focal_length
    sn = rtxpy.Scene.load(os.path.join(C.SCENES, "scene3.json"), scale="norm")
    assert sn.desc.camera.focal_length != s.desc.camera.focal_length


def test_frame_setup_matches_image_init():
    s = rtxpy.Scene.load(SCENE1)
    cam = s.desc.camera
    fr = s.frame(160, 90)
    f32 = np.float32
    size_x = f32(2) * f32(cam.focal_length) * f32(np.tan(f32(f32(cam.fov) * f32(3.1415927) / f32(360))))
    v = np.array(cam.vectors, np.float32)
    assert np.allclose(fr.step_x, v[0] * (size_x / f32(160)), rtol=1e-6)
    center = v[2] * f32(cam.focal_length) + np.array(cam.position, np.float32)
    size_y = size_x * f32(90) / f32(160)
    corner = center + np.array(fr.step_x) * f32(0.5 - 80) + v[1] * (size_y / f32(90)) * f32(0.5 - 45)
    assert np.allclose(fr.corner, corner, rtol=1e-5, atol=1e-6)


def test_params_from_argv_like_render_init():
    p = rtxpy.params_from_args(["-b", "-3", "-a", "0.1", "-s", "blinn", "-g", "path", "-n", "16", "-l", "lin",
                                "-o", "2.5"])
    assert p.max_bounces == 3 and abs(p.min_intensity_sqr - 0.01) < 1e-7
    assert p.reflection == abi.RTX_BLINN and p.gi == abi.RTX_GI_PATH and p.samples == 16
    assert p.attenuation == abi.RTX_ATT_LIN and p.attenuation_offset == 2.5
    q = rtxpy.params_from_args(["-s", "gouraud", "-l"])  # unknown value keeps default; flag without value ignored
    assert q.reflection == abi.RTX_PHONG and q.attenuation == abi.RTX_ATT_SQR


def test_tiff_roundtrip_raw_and_8bit(tmp_path):
    rng = np.random.default_rng(0)
    rgb = rng.uniform(-0.2, 1.5, (9, 13, 3)).astype(np.float32)
    z = rng.uniform(0, 10, (9, 13)).astype(np.float32)
    rtxpy.write_tiff(str(tmp_path / "raw.tif"), rgb, z, raw=True)
    t = read_tiff(str(tmp_path / "raw.tif"))
    assert t["bits"] == 32 and np.array_equal(t["rgb"], rgb) and np.array_equal(t["z"], z)
    assert 339 not in t["tags"]  # no SampleFormat tag, like image.c:64-85
    rtxpy.write_tiff(str(tmp_path / "b.tif"), rgb)
    t = read_tiff(str(tmp_path / "b.tif"))
    expect = np.maximum(np.minimum(rgb * np.float32(255), 255), 0).astype(np.uint8)
    assert t["bits"] == 8 and np.array_equal(t["rgb"], expect)
    assert t["tags"][278][0] == 1 and t["tags"][262][0] == 2 and t["tags"][274][0] == 1


def test_tiff_matches_reference_reader_layout():
    """A raw TIFF written by the reference (via libtiff) and by us decode to the same data."""
    name = "s1_b0"
    rgb, z = C.golden_frame(name)
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "x.tif")
        rtxpy.write_tiff(p, rgb, z, raw=True)
        t = read_tiff(p)
    assert np.array_equal(t["rgb"], rgb) and np.array_equal(t["z"], z)
