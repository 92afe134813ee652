"""The C-ABI libraries load on a CPU-only host and export every symbol the headers declare."""
import ctypes
import os
import re

import pytest

import rtxpy
from rtxpy import abi

INCLUDE = os.path.join(rtxpy.REPO_ROOT, "include")
ROOT = rtxpy.REPO_ROOT


def declared(header):
    text = open(os.path.join(INCLUDE, header)).read()
    return sorted(set(re.findall(r"^\s*(?:int|void|const char \*|uint32_t|size_t|const rtx_scene_desc \*)\s*\*?(rtx_\w+)\(",
                                 text, re.M)))


def test_librtx_exports_header_symbols():
    lib = ctypes.CDLL(rtxpy.LIBRTX)  # loads without a GPU (HIP runtime is lazy)
    names = declared("rtx.h")
    assert set(names) == set(abi.RTX_SYMBOLS), names
    for n in names:
        assert hasattr(lib, n), n


def test_librtxscene_exports_header_symbols():
    lib = ctypes.CDLL(rtxpy.LIBSCENE)
    names = declared("rtx_scene.h")
    assert set(names) == set(abi.RTX_SCENE_SYMBOLS), names
    for n in names:
        assert hasattr(lib, n), n


def test_params_default_matches_python_mirror():
    lib = rtxpy.rtx_lib()
    p = abi.Params()
    lib.rtx_params_default(ctypes.byref(p))
    q = rtxpy.default_params()
    for f, _ in abi.Params._fields_:
        assert getattr(p, f) == getattr(q, f), f


def test_device_count_and_open_fail_cleanly_without_gpu():
    lib = rtxpy.rtx_lib()
    n = ctypes.c_int(-1)
    assert lib.rtx_device_count(ctypes.byref(n)) == 0
    if n.value == 0:
        ctx = ctypes.c_void_p()
        rc = lib.rtx_open(0, ctypes.byref(ctx))
        assert rc == abi.RTX_ERR_NODEV and not ctx.value
        assert b"device" in lib.rtx_last_error()
        assert lib.rtx_kat(0, 1, None, None, None) == abi.RTX_ERR_ARG


def test_struct_sizes_match_c():
    # ctypes layouts must match the C structs byte for byte
    assert ctypes.sizeof(abi.Material) == 4 * (1 + 15 + 2 + 2 + 6 + 5 + 3)
    assert ctypes.sizeof(abi.Object) == 4 * (4 + 18 + 2)
    assert ctypes.sizeof(abi.Frame) == 4 * (2 + 12)
    assert ctypes.sizeof(abi.Params) == 56
    assert ctypes.sizeof(abi.Stats) == 11 * 8 + 6 * 8 + 6 * 4 + 4 * 8 + 2 * 4 + 8 + 8 + 2 * 4 + 8 + 2 * 4 + 2 * 4 + 2 * 4 + 2 * 8 + 8 + 2 * 4 + 4 * 8


def test_struct_layouts_match_compiled_header(tmp_path):
    """every field offset and struct size of the ctypes mirror against include/rtx.h as gcc lays it out"""
    import shutil
    import subprocess
    if not shutil.which("gcc"):
        pytest.skip("gcc not available")
    structs = {"rtx_material": abi.Material, "rtx_object": abi.Object, "rtx_frame": abi.Frame,
               "rtx_params": abi.Params, "rtx_stats": abi.Stats, "rtx_post": abi.Post,
               "rtx_group_member": abi.GroupMember}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "rtx.h"', "int main(void) {"]
    for cname, py in structs.items():
        lines.append(f'printf("{cname} %zu\\n", sizeof({cname}));')
        for f, _ in py._fields_:
            lines.append(f'printf("{cname}.{f} %zu\\n", offsetof({cname}, {f}));')
    lines.append("return 0; }")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = dict(l.split() for l in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.splitlines())
    for cname, py in structs.items():
        assert int(got[cname]) == ctypes.sizeof(py), cname
        for f, _ in py._fields_:
            assert int(got[f"{cname}.{f}"]) == getattr(py, f).offset, (cname, f)
