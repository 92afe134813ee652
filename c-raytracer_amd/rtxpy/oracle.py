"""ORACLE TEST INFRASTRUCTURE — ctypes access to oracle/librtx_oracle.so.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module; the product path (librtx.so, rtxpy.Renderer, engine) never does.
"""
import ctypes as C
import os

import numpy as np

from . import REPO_ROOT, RtxError, abi, default_params

ORACLE_DIR = os.path.join(REPO_ROOT, "oracle")
LIBORACLE = os.path.join(ORACLE_DIR, "librtx_oracle.so")
REF_DIR = os.path.join(ORACLE_DIR, "_ref")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIBORACLE):
            raise RtxError(abi.RTX_ERR_STATE, f"{LIBORACLE} not built (make -C oracle restate)")
        _lib = C.CDLL(LIBORACLE)
        abi.declare_oracle(_lib)
    return _lib


def render(scene, frame, params=None, threads=0):
    """CPU restatement of render() (render.c:345-368).  Returns rgb, z, (closest, shadow)."""
    p = params or default_params()
    w, h = frame.width, frame.height
    rgb = np.zeros((h, w, 3), np.float32)
    z = np.zeros((h, w), np.float32)
    counts = (C.c_uint64 * 2)()
    rc = lib().rtx_oracle_render(C.byref(scene.desc), C.byref(frame), C.byref(p), rgb.ctypes.data, z.ctypes.data,
                                 counts, threads)
    if rc != 0:
        raise RtxError(rc, "oracle render failed")
    return rgb, z, (int(counts[0]), int(counts[1]))


def primary(scene, frame, threads=0):
    """the primary hits alone (rtx_oracle_primary): z as render() writes it for -b >= 1, and the hit
    object's index (-1 on a miss); independent of the light samples"""
    w, h = frame.width, frame.height
    z = np.zeros((h, w), np.float32)
    obj = np.zeros((h, w), np.int32)
    rc = lib().rtx_oracle_primary(C.byref(scene.desc), C.byref(frame), z.ctypes.data, obj.ctypes.data, threads)
    if rc != 0:
        raise RtxError(rc, "oracle primary failed")
    return z, obj


def kat(kind, records, params=None):
    records = np.ascontiguousarray(records, dtype=np.float32).reshape(-1, abi.KAT_IN[kind])
    out = np.zeros((records.shape[0], abi.KAT_OUT[kind]), np.float32)
    p = params or default_params()
    rc = lib().rtx_oracle_kat(kind, records.shape[0], records.ctypes.data, out.ctypes.data, C.byref(p))
    if rc != 0:
        raise RtxError(rc, "oracle kat failed")
    return out
