"""Minimal TIFF reader for the reference's outputs (image.c:64-139) and ours.

Reads strips of 8-bit or 32-bit RGB (32-bit samples are raw IEEE floats: the
reference writes them without a SampleFormat tag, so PIL misreads them) and the
private tag 65000 (FLOAT[W*H]) z-buffer.  Little-endian ("II") files only.
"""
import struct

import numpy as np

_TYPE_SIZE = {1: 1, 2: 1, 3: 2, 4: 4, 5: 8, 6: 1, 7: 1, 8: 2, 9: 4, 10: 8, 11: 4, 12: 8, 16: 8}
_TYPE_FMT = {1: "B", 3: "H", 4: "I", 11: "f", 12: "d", 16: "Q"}


def read_tiff(path):
    """Returns dict(width, height, bits, rgb (H,W,3 float32 or uint8), z (H,W) or None, tags)."""
    with open(path, "rb") as f:
        data = f.read()
    if data[:4] != b"II*\x00":
        raise ValueError(f"{path}: not a little-endian classic TIFF")
    (ifd,) = struct.unpack_from("<I", data, 4)
    (n,) = struct.unpack_from("<H", data, ifd)
    tags = {}
    for i in range(n):
        tag, typ, cnt, val = struct.unpack_from("<HHI4s", data, ifd + 2 + 12 * i)
        size = _TYPE_SIZE.get(typ, 1) * cnt
        raw = val if size <= 4 else data[struct.unpack("<I", val)[0]:struct.unpack("<I", val)[0] + size]
        fmt = _TYPE_FMT.get(typ)
        if fmt:
            vals = struct.unpack_from("<%d%s" % (cnt, fmt), raw[:size] if size <= 4 else raw)
        else:
            vals = raw
        tags[tag] = vals
    w, h = tags[256][0], tags[257][0]
    bits = tags[258][0]
    spp = tags.get(277, (1,))[0]
    offs, counts = tags[273], tags[279]
    buf = b"".join(data[o:o + c] for o, c in zip(offs, counts))
    if bits == 8:
        rgb = np.frombuffer(buf, np.uint8).reshape(h, w, spp).copy()
    elif bits == 32:
        rgb = np.frombuffer(buf, "<f4").reshape(h, w, spp).copy()
    else:
        raise ValueError(f"{path}: unsupported BitsPerSample {bits}")
    z = None
    if 65000 in tags:
        z = np.asarray(tags[65000], np.float32).reshape(h, w)
    return {"width": w, "height": h, "bits": bits, "rgb": rgb, "z": z, "tags": tags}
