"""Pin the CPU oracle (oracle/restate.c) to the compiled reference.

Fixtures (tests/golden, made by tools/make_goldens.py from oracle/_ref, i.e. the
reference built from /root/reference's own sources):
  kat.npz         per-function known answers of the reference's own functions
  frames/*.npz    reference renders (raw float rgb + z) with ray counts
The oracle must reproduce them within SURVEY.md §8(c)'s tolerances; only then
is it trusted as the checker of the GPU path (tests/test_gpu_parity.py).
"""
import os

import numpy as np
import pytest

import conftest as C
import rtxpy
from rtxpy import abi, oracle

KAT = np.load(os.path.join(C.GOLDEN, "kat.npz"))


def _kat(name, params=None):
    kind = abi.KAT_NAMES.index(name)
    x = KAT[name + "_in"]
    return x, KAT[name + "_out"], oracle.kat(kind, x, params)


def test_kat_moller_trumbore():
    x, ref, out = _kat("moller")
    assert (out[:, 0] == ref[:, 0]).mean() >= 0.999  # hit/miss (boundary flips from FMA only)
    both = (out[:, 0] == 1) & (ref[:, 0] == 1)
    rel = np.abs(out[both, 1] - ref[both, 1]) / np.maximum(np.abs(ref[both, 1]), 1e-3)
    assert rel.max() <= 1e-4


def test_kat_sphere():
    x, ref, out = _kat("sphere")
    assert (out[:, 0] == ref[:, 0]).mean() >= 0.999
    both = (out[:, 0] == 1) & (ref[:, 0] == 1)
    t_rel = np.abs(out[both, 1] - ref[both, 1]) / np.maximum(np.abs(ref[both, 1]), 1.0)
    assert t_rel.max() <= 1e-4
    # normal = (o + t d - c)/r inherits the t difference and the rounding of P, divided by r
    dn = np.abs(out[both, 2:] - ref[both, 2:]).max(axis=1)
    dt = np.abs(out[both, 1] - ref[both, 1])
    scale = np.abs(x[both, :3]).max(1) + np.abs(out[both, 1]) + np.abs(x[both, 6:9]).max(1)
    assert (dn <= (dt + 4e-7 * scale) / x[both, 9] + 1e-7).all()


def test_kat_plane():
    x, ref, out = _kat("plane")
    assert (out[:, 0] == ref[:, 0]).all()
    both = out[:, 0] == 1
    assert np.allclose(out[both, 1], ref[both, 1], rtol=1e-5, atol=1e-6)
    assert (out[both, 2:] == ref[both, 2:]).all()


def test_kat_slab():
    x, ref, out = _kat("slab")
    assert (out == ref).all()


def test_kat_simplex_noise():
    x, ref, out = _kat("noise")
    assert np.abs(out - ref).max() <= 5e-5


def test_kat_textures_and_u32_mode():
    # the reference was built -march=native on an AVX-512 host: float->uint32 saturates
    x, ref, out = _kat("texture", rtxpy.default_params(u32conv=abi.RTX_U32_SAT))
    close = np.isclose(out, ref, rtol=1e-4, atol=1e-5).all(axis=1)
    assert close.mean() >= 0.995  # noisy-periodic near discontinuities of saw/square
    assert close[x[:, 0] != 3].all()  # uniform / checkerboard / brick exact
    xw, refw, outw = _kat("texture", rtxpy.default_params(u32conv=abi.RTX_U32_WRAP))
    assert np.isclose(outw, refw, rtol=1e-4, atol=1e-5).all(axis=1).mean() < 0.95


def test_kat_u32_conversion():
    x, ref, out = _kat("u32")
    assert (out[:, 0].view(np.uint32) == ref[:, 0].view(np.uint32)).all()


def test_kat_light_samplers():
    for name in ("sph_light", "tri_light"):
        x, ref, out = _kat(name)
        assert np.allclose(out, ref, rtol=1e-4, atol=2e-6), name


def test_kat_morton():
    x, ref, out = _kat("morton")
    assert (out.view(np.uint32) == ref.view(np.uint32)).all()


CONST = [k for k, v in C.manifest().items() if v["rng"] == "const"]


@pytest.mark.parametrize("name", CONST)
def test_frame_bit_exact_vs_reference_ieee(name):
    """The restatement reproduces the reference built at -O2 (IEEE single precision) BIT-EXACTLY:
    every rgb and z value, and the cast_ray / is_light_blocked call counts."""
    scene, frame, params, m = C.load_config(name)
    rgb, z, (nc, ns) = oracle.render(scene, frame, params, threads=0)
    ref_rgb, ref_z = C.golden_frame(name + "_o2")
    assert np.array_equal(z, ref_z)
    assert np.array_equal(rgb, ref_rgb), float(np.abs(rgb - ref_rgb).max())
    assert (nc, ns) == (m["closest_rays_o2"], m["shadow_rays_o2"])


@pytest.mark.parametrize("name", CONST)
def test_frame_vs_reference_ofast(name):
    """Against the reference exactly as Makefile.rt builds it (-Ofast: FMA, rsqrt) the difference
    stays within SURVEY §8(c) tolerances or the reference's own Ofast-vs-O2 noise floor."""
    scene, frame, params, m = C.load_config(name)
    rgb, z, (nc, ns) = oracle.render(scene, frame, params, threads=0)
    ref_rgb, ref_z = C.golden_frame(name)
    ok, info = C.compare_const(rgb, z, ref_rgb, ref_z, **C.floor_tolerance(m))
    assert ok, (info, m["floor"])
    assert abs(nc - m["closest_rays"]) <= 0.005 * m["closest_rays"] + 16
    assert abs(ns - m["shadow_rays"]) <= 0.005 * m["shadow_rays"] + 600


@pytest.mark.parametrize("name", [k for k in CONST if "_b0" not in k])
def test_primary_mode_is_the_reference_z(name):
    """rtx_oracle_primary (the primary hits alone, used for the frame-wide depth checks of the
    BASELINE configs) writes exactly the z-buffer of the reference built at -O2"""
    scene, frame, params, m = C.load_config(name)
    z, obj = oracle.primary(scene, frame)
    ref_rgb, ref_z = C.golden_frame(name + "_o2")
    assert np.array_equal(z, ref_z)
    assert np.array_equal(obj >= 0, ref_z > 0)


def test_frame_b0_has_zero_z():
    # -b 0: the primary call itself has no bounces left, so every z is 0
    scene, frame, params, m = C.load_config("s1_b0")
    rgb, z, _ = oracle.render(scene, frame, params)
    assert (z == 0).all() and rgb.max() > 0


SEEDSETS = sorted(C.seed_manifest())
ORACLE_MAX_SEEDS = {"s6_path8": 16}  # the CPU suite averages at most this many seeds (default 64)


@pytest.mark.parametrize("name", SEEDSETS)
def test_frame_statistical(name):
    """Counter RNG vs the reference's seeded glibc stream: the oracle's image
    averaged over seeds against the reference's average over its seeds, per-channel means within
    1 % and 8x8 box-filtered relL1 <= 3 %; z is RNG-independent.  The fixtures' seed-averaged
    mean has a relative sigma <= 0.2 % (manifest sigma_avg_rel)."""
    scene, frame, params, m, g = C.load_seedset(name)
    assert max(m["sigma_avg_rel"]) <= 0.002
    params.rng = abi.RTX_RNG_COUNTER
    seeds = m["seeds"][:ORACLE_MAX_SEEDS.get(name, 64)]
    avg, z = C.seed_average(lambda p: oracle.render(scene, frame, p, threads=0)[:2], params, seeds)
    assert np.array_equal(z, g["z"])
    ok, info = C.compare_stat(avg, z, g)
    assert ok, info


def test_reference_self_noise_floor():
    """Two seeds of the reference itself: the statistical tolerance must exceed its own MC noise."""
    a, _ = C.golden_frame("s3_seed_path16")
    b, _ = C.golden_frame("s3_seed_path16_s2")
    rel = np.abs(C.box_filter(a) - C.box_filter(b)).sum() / np.abs(C.box_filter(a)).sum()
    assert rel <= 0.08


def test_oracle_tile_sharding_is_exact():
    scene, frame, params, _ = C.load_config("s3_amb")
    full, zf, cf = oracle.render(scene, frame, params)
    parts = np.zeros_like(full)
    zp = np.zeros_like(zf)
    tot = [0, 0]
    for r in range(3):
        p = rtxpy.default_params(**{f: getattr(params, f) for f, _ in abi.Params._fields_})
        p.tile_offset, p.tile_stride = r, 3
        rgb, z, c = oracle.render(scene, frame, p)
        from rtxpy.dist import rank_tiles, tile_pixel_index
        idx = tile_pixel_index(frame.width, frame.height, rank_tiles(frame.width, frame.height, r, 3)).reshape(-1)
        idx = idx[idx >= 0]
        parts.reshape(-1, 3)[idx] = rgb.reshape(-1, 3)[idx]
        zp.reshape(-1)[idx] = z.reshape(-1)[idx]
        tot[0] += c[0]
        tot[1] += c[1]
    assert (parts == full).all() and (zp == zf).all()
    assert tuple(tot) == cf


def test_kat_fast_forms_oracle_side():
    """The oracle's exact answers for the fast-form KATs (rtx_kat.h 12-14), pinned to the
    reference's own known answers: any-hit = moller_trumbore hit with t < tlim; the sphere light
    = light_point; the box answer is the double-precision slab test."""
    import kat_fast
    kat = np.load(os.path.join(C.GOLDEN, "kat.npz"))
    recs, want = kat_fast.any_tri_records(kat)
    got = oracle.kat(abi.KAT_ANY_TRI, recs)[:, 0] > 0
    assert (got == want).mean() >= 0.999
    x, ref = kat["sph_light_in"], kat["sph_light_out"]
    assert np.allclose(oracle.kat(abi.KAT_SPH_LIGHT_SH, x), ref, rtol=1e-4, atol=2e-6)
    b = kat_fast.box_q_records(2000)
    out = oracle.kat(abi.KAT_BOX_Q, b)
    assert out.shape == (2000, 2) and 0.05 < out[:, 0].mean() < 0.95


def test_kat_spec_pow_oracle_is_libm():
    """The oracle's specular power is the reference's expression (render.c:224) on glibc powf."""
    import kat_fast
    recs = kat_fast.spec_pow_records(4000)
    out = oracle.kat(abi.KAT_SPEC_POW, recs)[:, 0]
    assert np.array_equal(out, kat_fast.libm_spec_pow(recs))


def test_oracle_stratified_light_samples_keep_the_expectation():
    """RTX_RNG_STRAT (include/rtx.h) only moves each light sample inside its stratum: the image
    differs sample for sample from the plain counter RNG but keeps its mean, with less noise."""
    scene, frame, params, _ = C.load_config("s3_path2")
    params.seed = 7
    params.rng = abi.RTX_RNG_COUNTER
    a, za, (ca, sa) = oracle.render(scene, frame, params)
    params.rng = abi.RTX_RNG_STRAT
    b, zb, (cb, sb) = oracle.render(scene, frame, params)
    assert np.array_equal(za, zb) and (ca, sa) == (cb, sb)  # same rays, same primary hits
    assert not np.array_equal(a, b)
    ma, mb = a.reshape(-1, 3).mean(0), b.reshape(-1, 3).mean(0)
    assert np.all(np.abs(ma - mb) <= 0.02 * np.abs(ma) + 1e-7), (ma, mb)
