"""rtxpy — Python (ctypes) driver for the rtx C-ABI (include/rtx.h, include/rtx_scene.h).

Host plumbing for tests and bench.py.  The product is the C-ABI library
``c-raytracer_amd/lib/librtx.so`` (HIP kernels for gfx950) and the C host glue
``librtxscene.so``; this module only loads them.  There is no CPU fallback:
``Renderer`` raises if librtx.so is missing or no gfx950 device is usable.

The CPU oracle (``oracle/librtx_oracle.so``) is test infrastructure and is
reached only through ``rtxpy.oracle`` by tests/, ``__graft_entry__.smoke()``
and bench.py's cpu_baseline leg.
"""
import ctypes as C
import os

import numpy as np

from . import abi
from .abi import (Frame, Params, SceneDesc, Stats, RTX_OK)  # noqa: F401

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REPO_ROOT = os.path.dirname(PKG_DIR)
LIB_DIR = os.path.join(PKG_DIR, "lib")
LIBRTX = os.environ.get("RTX_LIBRTX") or os.path.join(LIB_DIR, "librtx.so")  # override: build variants
LIBSCENE = os.path.join(LIB_DIR, "librtxscene.so")
ENGINE = os.path.join(LIB_DIR, "engine")

_scene_lib = None
_rtx_lib = None


class RtxError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"rtx error {code}: {msg}")
        self.code = code


def scene_lib():
    global _scene_lib
    if _scene_lib is None:
        if not os.path.exists(LIBSCENE):
            raise RtxError(abi.RTX_ERR_STATE, f"{LIBSCENE} not built (run __graft_entry__.build())")
        lib = C.CDLL(LIBSCENE)
        abi.declare_scene(lib)
        _scene_lib = lib
    return _scene_lib


def rtx_lib():
    """Load librtx.so (the HIP path).  Raises when it is missing: no fallback."""
    global _rtx_lib
    if _rtx_lib is None:
        if not os.path.exists(LIBRTX):
            raise RtxError(abi.RTX_ERR_STATE, f"{LIBRTX} not built (run __graft_entry__.build())")
        lib = C.CDLL(LIBRTX)
        abi.declare_rtx(lib)
        _rtx_lib = lib
    return _rtx_lib


def _check_scene(rc):
    if rc != RTX_OK:
        raise RtxError(rc, scene_lib().rtx_scene_last_error().decode(errors="replace"))


def _check(rc):
    if rc != RTX_OK:
        raise RtxError(rc, rtx_lib().rtx_last_error().decode(errors="replace"))


class Scene:
    """A loaded scene (owner of the C rtx_scene)."""

    def __init__(self, handle):
        self._h = handle
        self.desc = scene_lib().rtx_scene_desc_of(handle).contents

    @classmethod
    def load(cls, path, scale=None, base_dir=None):
        h = C.c_void_p()
        _check_scene(scene_lib().rtx_scene_load(os.fsencode(path), scale.encode() if scale else None,
                                                os.fsencode(base_dir) if base_dir else None, C.byref(h)))
        return cls(h)

    @classmethod
    def parse(cls, text, name="<memory>", scale=None, base_dir=None):
        data = text.encode() if isinstance(text, str) else text
        h = C.c_void_p()
        _check_scene(scene_lib().rtx_scene_parse(data, len(data), name.encode(), scale.encode() if scale else None,
                                                 os.fsencode(base_dir) if base_dir else None, C.byref(h)))
        return cls(h)

    def frame(self, width, height):
        fr = Frame()
        _check_scene(scene_lib().rtx_frame_setup(C.byref(self.desc.camera), width, height, C.byref(fr)))
        return fr

    @property
    def num_objects(self):
        return self.desc.num_objects

    def objects(self):
        return [self.desc.objects[i] for i in range(self.desc.num_objects)]

    def materials(self):
        return [self.desc.materials[i] for i in range(self.desc.num_materials)]

    def emitters(self):
        return [self.desc.emitters[i] for i in range(self.desc.num_emitters)]

    def close(self):
        if self._h:
            scene_lib().rtx_scene_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def default_params(**kw):
    """rtx_params_default (render.c:53-60 defaults) plus overrides."""
    p = Params()
    p.max_bounces = 10
    p.min_intensity_sqr = 0.01 * 0.01
    p.reflection = abi.RTX_PHONG
    p.gi = abi.RTX_GI_AMBIENT
    p.samples = 1
    p.attenuation = abi.RTX_ATT_SQR
    p.attenuation_offset = 1.0
    p.rng = abi.RTX_RNG_COUNTER
    p.seed = 1
    p.u32conv = abi.RTX_U32_SAT
    p.tile_offset = 0
    p.tile_stride = 1
    p.count_traversal = 0
    # float32 rounding of .01f*.01f like the C default
    p.min_intensity_sqr = float(np.float32(np.float32(0.01) * np.float32(0.01)))
    for k, v in kw.items():
        if not hasattr(p, k):
            raise AttributeError(k)
        setattr(p, k, v)
    return p


def params_from_args(args, **kw):
    """render_init (render.c:61-116) over a reference-style argument list."""
    p = default_params(**kw)
    argv = [b"engine"] + [a.encode() for a in args]
    arr = (C.c_char_p * len(argv))(*argv)
    scene_lib().rtx_params_from_argv(len(argv), arr, C.byref(p))
    return p


def hash_djb(s):
    return scene_lib().rtx_hash_djb(s.encode())


def write_tiff(path, rgb, z=None, raw=False):
    rgb = np.ascontiguousarray(rgb, dtype=np.float32)
    h, w = rgb.shape[:2]
    zz = None
    if raw:
        zz = np.ascontiguousarray(z, dtype=np.float32)
    rc = scene_lib().rtx_tiff_write(os.fsencode(path), w, h, rgb.ctypes.data,
                                    zz.ctypes.data if zz is not None else None, 1 if raw else 0)
    if rc != RTX_OK:
        raise RtxError(rc, f"tiff write failed: {path}")


def read_tiff_raw(path):
    """rtx_tiff_read_raw (librtxscene): (rgb (H,W,3), z (H,W)) float32 of a raw TIFF."""
    w, h = C.c_uint32(), C.c_uint32()
    prgb, pz = C.c_void_p(), C.c_void_p()
    rc = scene_lib().rtx_tiff_read_raw(os.fsencode(path), C.byref(w), C.byref(h), C.byref(prgb), C.byref(pz))
    if rc != RTX_OK:
        raise RtxError(rc, f"raw tiff read failed: {path}")
    try:
        n = w.value * h.value
        rgb = np.ctypeslib.as_array((C.c_float * (3 * n)).from_address(prgb.value)).reshape(h.value, w.value, 3).copy()
        z = np.ctypeslib.as_array((C.c_float * n).from_address(pz.value)).reshape(h.value, w.value).copy()
    finally:
        scene_lib().rtx_buffer_free(prgb)
        scene_lib().rtx_buffer_free(pz)
    return rgb, z


def post_from_args(args):
    """rtx_post_from_argv over ["postprocess", "<in>", "<out>"] + args (the reference's argv layout)."""
    from .abi import Post
    argv = [b"postprocess", b"in.tif", b"out.tif"] + [a.encode() for a in args]
    arr = (C.c_char_p * len(argv))(*argv)
    p = Post()
    rc = scene_lib().rtx_post_from_argv(len(argv), arr, C.byref(p))
    if rc != RTX_OK:
        raise RtxError(rc, scene_lib().rtx_scene_last_error().decode())
    return p


def write_stl(path, tris):
    tris = np.ascontiguousarray(tris, dtype=np.float32).reshape(-1, 9)
    _check_scene(scene_lib().rtx_stl_write(os.fsencode(path), tris.shape[0], tris.ctypes.data))


class Renderer:
    """One rtx context on one HIP device (rtx_open .. rtx_close)."""

    def __init__(self, device=0):
        self.lib = rtx_lib()
        self._ctx = C.c_void_p()
        _check(self.lib.rtx_open(device, C.byref(self._ctx)))
        self.device = device

    def set_builder(self, builder):
        """rtx_set_builder: abi.RTX_BUILD_SAH_GPU (default), abi.RTX_BUILD_SAH_HOST, abi.RTX_BUILD_LBVH_GPU or
        abi.RTX_BUILD_PLOC_GPU."""
        _check(self.lib.rtx_set_builder(self._ctx, builder))

    def set_option(self, option, value):
        """rtx_set_option: abi.RTX_OPT_* (shadow walk, BVH leaf size, shade-point sort, k_shadow
        slot and grab sizes); build options take effect at the next upload."""
        _check(self.lib.rtx_set_option(self._ctx, option, int(value)))

    def upload(self, scene):
        _check(self.lib.rtx_upload_scene(self._ctx, C.byref(scene.desc)))

    def render(self, frame, params, rgb=None, z=None):
        w, h = frame.width, frame.height
        if rgb is None:
            rgb = np.zeros((h, w, 3), np.float32)
        if z is None:
            z = np.zeros((h, w), np.float32)
        assert rgb.dtype == np.float32 and rgb.flags.c_contiguous and rgb.size == w * h * 3
        assert z.dtype == np.float32 and z.flags.c_contiguous and z.size == w * h
        _check(self.lib.rtx_render(self._ctx, C.byref(frame), C.byref(params), rgb.ctypes.data, z.ctypes.data))
        return rgb, z

    def render_device(self, frame, params, d_rgb, d_z, stream=None):
        """d_rgb / d_z: device pointers (ints), stream: hipStream_t as int or None."""
        _check(self.lib.rtx_render_device(self._ctx, C.byref(frame), C.byref(params), C.c_void_p(d_rgb),
                                          C.c_void_p(d_z), C.c_void_p(stream) if stream else None))

    def postprocess(self, post, rgb, z):
        """rtx_postprocess on host arrays: returns the postprocessed (H,W,3) float32 copy."""
        out = np.ascontiguousarray(rgb, dtype=np.float32).copy()
        zz = np.ascontiguousarray(z, dtype=np.float32)
        h, w = out.shape[:2]
        _check(self.lib.rtx_postprocess(self._ctx, w, h, C.byref(post), out.ctypes.data, zz.ctypes.data))
        return out

    def postprocess_device(self, post, width, height, d_rgb, d_z, stream=None):
        _check(self.lib.rtx_postprocess_device(self._ctx, width, height, C.byref(post), C.c_void_p(d_rgb),
                                               C.c_void_p(d_z), C.c_void_p(stream) if stream else None))

    def wide_tree(self):
        """the uploaded 8-wide tree (rtx_read_wide_tree): (entries uint32 (n, 16), frame float32 (6,))"""
        n = C.c_uint32(0)
        frame = np.zeros(6, np.float32)
        _check(self.lib.rtx_read_wide_tree(self._ctx, None, 0, C.byref(n), frame.ctypes.data))
        ent = np.zeros((n.value, 16), np.uint32)
        if n.value:
            _check(self.lib.rtx_read_wide_tree(self._ctx, ent.ctypes.data, n.value, C.byref(n), frame.ctypes.data))
        return ent, frame

    def stats(self):
        s = Stats()
        _check(self.lib.rtx_get_stats(self._ctx, C.byref(s)))
        return s

    def close(self):
        if self._ctx:
            self.lib.rtx_close(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def tree_frame(scene):
    """rtx_tree_frame (no device needed): (rotated, R (3, 3), centre (3,), cost ratio) of the frame
    rtx_upload_scene builds the scene's BVHs in under RTX_FRAME_AUTO"""
    rot = np.zeros(9, np.float32)
    cen = np.zeros(3, np.float32)
    flag = C.c_int()
    ratio = C.c_double()
    _check(rtx_lib().rtx_tree_frame(C.byref(scene.desc), C.byref(flag), rot.ctypes.data, cen.ctypes.data, C.byref(ratio)))
    return bool(flag.value), rot.reshape(3, 3), cen, ratio.value


def gpu_kat(kind, records, params=None):
    records = np.ascontiguousarray(records, dtype=np.float32).reshape(-1, abi.KAT_IN[kind])
    out = np.zeros((records.shape[0], abi.KAT_OUT[kind]), np.float32)
    p = params or default_params()
    _check(rtx_lib().rtx_kat(kind, records.shape[0], records.ctypes.data, out.ctypes.data, C.byref(p)))
    return out


class Group:
    """Several HIP devices rendering one frame (rtx_group_open .. rtx_group_close): tiles dealt
    round-robin over the devices, gathered to the first one over RCCL.  loopback=n: n shards as
    n contexts on device devices[0] (rtx_group_open_loopback, the test transport).  rccl_self:
    one device whose shard still travels through RCCL, to itself (rtx_group_open_rccl_self)."""

    def __init__(self, devices, loopback=None, rccl_self=False):
        self.lib = rtx_lib()
        self._g = C.c_void_p()
        if rccl_self:
            _check(self.lib.rtx_group_open_rccl_self(int(devices[0]), C.byref(self._g)))
            self.devices = [devices[0]]
        elif loopback:
            _check(self.lib.rtx_group_open_loopback(int(loopback), int(devices[0]), C.byref(self._g)))
            self.devices = [devices[0]] * int(loopback)
        else:
            devs = (C.c_int * len(devices))(*devices)
            _check(self.lib.rtx_group_open(len(devices), devs, C.byref(self._g)))
            self.devices = list(devices)

    def set_builder(self, builder):
        _check(self.lib.rtx_group_set_builder(self._g, builder))

    def set_option(self, option, value):
        _check(self.lib.rtx_group_set_option(self._g, option, int(value)))

    def upload(self, scene):
        _check(self.lib.rtx_group_upload_scene(self._g, C.byref(scene.desc)))

    def render(self, frame, params, rgb=None, z=None):
        """the whole frame on the group's first device's host side; rgb / z: optional preallocated
        float32 (H, W, 3) / (H, W) host arrays (pinned ones make the copy faster)"""
        w, h = frame.width, frame.height
        if rgb is None:
            rgb = np.zeros((h, w, 3), np.float32)
        if z is None:
            z = np.zeros((h, w), np.float32)
        assert rgb.dtype == np.float32 and rgb.flags.c_contiguous and rgb.size == w * h * 3
        assert z.dtype == np.float32 and z.flags.c_contiguous and z.size == w * h
        _check(self.lib.rtx_group_render(self._g, C.byref(frame), C.byref(params), rgb.ctypes.data, z.ctypes.data))
        return rgb, z

    def size(self):
        return self.lib.rtx_group_size(self._g)

    def stats(self):
        s = Stats()
        _check(self.lib.rtx_group_get_stats(self._g, C.byref(s)))
        return s

    def device_stats(self, r):
        s = Stats()
        _check(self.lib.rtx_group_device_stats(self._g, r, C.byref(s)))
        return s

    def member(self, r):
        """what the runtime reports about member r (rtx_group_member_info): its device, its RCCL
        communicator's count / rank / device, peer access to and from member 0, PCI bus id"""
        m = abi.GroupMember()
        _check(self.lib.rtx_group_member_info(self._g, r, C.byref(m)))
        return {"device": m.device, "comm_count": m.comm_count, "comm_rank": m.comm_rank, "comm_device": m.comm_device,
                "can_access_peer0": m.can_access_peer0, "peer0_can_access": m.peer0_can_access,
                "peer_enabled": m.peer_enabled, "transport": m.transport, "pci_bus_id": m.pci_bus_id.decode()}

    def close(self):
        if self._g:
            self.lib.rtx_group_close(self._g)
            self._g = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def tile_pack(rgb, z, offset, stride):
    """rtx_tile_pack_host: the shard's (N, 4) float32 tile records {r, g, b, z}."""
    rgb = np.ascontiguousarray(rgb, dtype=np.float32)
    z = np.ascontiguousarray(z, dtype=np.float32)
    h, w = z.shape
    lib = rtx_lib()
    n = lib.rtx_tile_pack_count(w, h, offset, stride)
    out = np.zeros((n, 4), np.float32)
    _check(lib.rtx_tile_pack_host(rgb.ctypes.data, z.ctypes.data, w, h, offset, stride, out.ctypes.data))
    return out


def tile_unpack(records, rgb, z, offset, stride):
    """rtx_tile_unpack_host: writes the shard's pixels of records into rgb / z in place."""
    records = np.ascontiguousarray(records, dtype=np.float32)
    assert rgb.dtype == np.float32 and rgb.flags.c_contiguous and z.dtype == np.float32 and z.flags.c_contiguous
    h, w = z.shape
    _check(rtx_lib().rtx_tile_unpack_host(records.ctypes.data, w, h, offset, stride, rgb.ctypes.data, z.ctypes.data))
