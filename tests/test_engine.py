"""The drop-in CLIs (lib/engine: src/raytracer/main.c flow; lib/postprocess: src/postprocess/main.c),
host-side behaviour without a GPU: help, argument errors, and that a machine without a gfx950
device gets a loud error, never a CPU fallback."""
import os
import subprocess

import pytest

import conftest as C
import rtxpy

ENGINE = rtxpy.ENGINE
POSTPROC = os.path.join(rtxpy.LIB_DIR, "postprocess")


def run(args, **kw):
    return subprocess.run(args, capture_output=True, text=True, timeout=120, **kw)


def test_engine_help_and_usage():
    p = run([ENGINE, "--help"])
    assert p.returncode == 0 and "Usage: ./engine <input> <output> <resolution>" in p.stdout
    p = run([ENGINE, "x.json"])
    assert p.returncode == 1 and "Too few arguments" in p.stdout


def test_postprocess_help_and_usage():
    p = run([POSTPROC, "-h"])
    assert p.returncode == 0 and "Usage: ./postprocess <input> <output>" in p.stdout
    p = run([POSTPROC, "in.tif"])
    assert p.returncode == 1 and "Too few arguments" in p.stdout
    p = run([POSTPROC, "in.tif", "out.tif", "--mist", "1", "2", "cubic", "0", "0", "0"])
    assert p.returncode == 1 and "Unrecognized falloff type [cubic]" in p.stderr


def test_engine_scene_errors(tmp_path):
    bad = tmp_path / "bad.json"
    bad.write_text('{"Camera": {}}')
    p = run([ENGINE, str(bad), str(tmp_path / "o.tif"), "16", "16"])
    assert p.returncode == 1 and "Materials" in p.stdout + p.stderr  # scene.c's error text


def _has_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.mark.skipif(_has_gpu(), reason="a GPU is present")
def test_engine_without_gpu_fails_loudly(tmp_path):
    p = run([ENGINE, os.path.join(C.SCENES, "scene1.json"), str(tmp_path / "o.tif"), "16", "16"])
    assert p.returncode != 0
    assert "gfx950" in (p.stdout + p.stderr) or "device" in (p.stdout + p.stderr).lower()
    assert not (tmp_path / "o.tif").exists()
