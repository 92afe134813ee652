"""Records and exact answers for the KATs of the fast device functions k_shadow runs
(include/rtx_kat.h kinds ANY_TRI, SPH_LIGHT_SH, BOX_Q).  Built from the reference's own
known answers (tests/golden/kat.npz, oracle/ref_kat.c) plus seeded synthetic boxes; used by
tests/test_oracle.py (CPU) and tests/test_gpu_parity.py (GPU)."""
import numpy as np

FLT_MAX = np.float32(3.4028235e38)


def any_tri_records(kat):
    """moller_in records x 4 segment ends: the reference's t scaled by 0.999 / 1.001, 2 t, FLT_MAX.
    Expected (reference, object.c:422-441 + the any-hit window t < tlim): hit and t < tlim."""
    x, ref = kat["moller_in"].astype(np.float32), kat["moller_out"]
    hit, t = ref[:, 0] > 0, ref[:, 1].astype(np.float32)
    base = np.where(hit, t, np.float32(1.0))
    recs, want = [], []
    for f in (np.float32(0.999), np.float32(1.001), np.float32(2.0), None):
        tl = np.full_like(base, FLT_MAX) if f is None else (base * f).astype(np.float32)
        recs.append(np.concatenate([x, tl[:, None]], 1))
        want.append(hit & (t < tl))
    return np.concatenate(recs).astype(np.float32), np.concatenate(want)


def mt_margin(recs):
    """float64 Moller-Trumbore of each record: the relative distance of the decision to its
    nearest boundary (|a| vs eps, u, v, u+v vs 1, t vs eps, t vs tlim).  Records whose IEEE and
    fast decisions may legitimately differ have a small margin."""
    r = recs.astype(np.float64)
    o, d, v0, e1, e2, eps, tl = r[:, 0:3], r[:, 3:6], r[:, 6:9], r[:, 9:12], r[:, 12:15], r[:, 15], r[:, 16]
    h = np.cross(d, e2)
    a = (e1 * h).sum(1)
    with np.errstate(divide="ignore", invalid="ignore"):
        f = 1.0 / a
        s = o - v0
        u = f * (s * h).sum(1)
        q = np.cross(s, e1)
        v = f * (d * q).sum(1)
        t = f * (e2 * q).sum(1)
        m = np.stack([np.abs(np.abs(a) - eps) / np.maximum(np.abs(a), 1e-30), np.abs(u), np.abs(v),
                      np.abs(1 - u - v), np.abs(t - eps) / np.maximum(np.abs(t), 1e-30),
                      np.abs(tl - t) / np.maximum(np.abs(t), 1e-30)], 1)
    m = np.where(np.isfinite(m), m, 0.0)
    return m.min(1)


def box_q_records(n=20000, seed=11):
    """Seeded rays and boxes in a quantisation frame of extent ~4 (the walk's frame: the bounded
    objects' box, 65533 steps per axis): boxes from 1e-4 to the whole frame, ray origins up to
    50 frame extents away, directions with exactly-zero components, segment ends around the box.
    Record: o3 d3 lo3 hi3 qo3 qs3 tlim."""
    rng = np.random.default_rng(seed)
    flo, fhi = np.array([-2.0, -1.5, -2.5]), np.array([2.0, 2.5, 1.5])
    ext = fhi - flo
    qs = 65533.0 / ext
    c = flo + rng.random((n, 3)) * ext
    half = ext * 10.0 ** rng.uniform(-4, -0.3, (n, 3)) / 2
    lo, hi = np.maximum(c - half, flo), np.minimum(c + half, fhi)
    scale = 10.0 ** rng.uniform(-1, np.log10(50.0), (n, 1))
    o = c + rng.normal(size=(n, 3)) * ext * scale
    d = rng.normal(size=(n, 3))
    zero = rng.random((n, 3)) < 0.05
    d[zero] = 0.0
    d[(d == 0).all(1), 0] = 1.0
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    # aim half of the rays at the box centre
    aim = rng.random(n) < 0.5
    dc = c - o
    dc /= np.linalg.norm(dc, axis=1, keepdims=True)
    d[aim] = dc[aim]
    dist = np.linalg.norm(c - o, axis=1)
    tl = dist * rng.uniform(0.2, 2.0, n)
    tl[rng.random(n) < 0.1] = FLT_MAX
    recs = np.concatenate([o, d, lo, hi, np.tile(flo, (n, 1)), np.tile(qs, (n, 1)), tl[:, None]], 1)
    return recs.astype(np.float32)


def spec_pow_records(n=40000, seed=5):
    """(specular_mul, shininess) pairs for the specular power (render.c:224): specular_mul over
    [-1, 1] with 0, +-1, denormals and values a few ulp from +-1; shininess from the scenes'
    values (0, 0.1, 1, 5, 10, 15, 20, 35), odd and even integers up to 1000 and uniform reals."""
    rng = np.random.default_rng(seed)
    x = rng.uniform(-1.0, 1.0, n)
    k = rng.random(n)
    x[k < 0.05] = 0.0
    x[(k >= 0.05) & (k < 0.08)] = 1.0
    x[(k >= 0.08) & (k < 0.10)] = -1.0
    near = (k >= 0.10) & (k < 0.20)
    x[near] = np.sign(rng.normal(size=near.sum())) * (1.0 - rng.integers(1, 64, near.sum()) * 2.0 ** -24)
    tiny = (k >= 0.20) & (k < 0.23)
    x[tiny] = rng.uniform(-1, 1, tiny.sum()) * 1e-38
    y = rng.choice(np.array([0.0, 0.1, 1.0, 5.0, 10.0, 15.0, 20.0, 35.0]), n)
    j = rng.random(n)
    y[j < 0.3] = rng.integers(0, 1000, (j < 0.3).sum())
    y[(j >= 0.3) & (j < 0.5)] = rng.uniform(0, 200, ((j >= 0.3) & (j < 0.5)).sum())
    return np.stack([x, y], 1).astype(np.float32)


def libm_spec_pow(recs):
    """fmaxf(0, powf(x, y)) with the C library's powf (the reference's libm)."""
    import ctypes
    libm = ctypes.CDLL("libm.so.6")
    libm.powf.argtypes = [ctypes.c_float, ctypes.c_float]
    libm.powf.restype = ctypes.c_float
    out = np.empty(len(recs), np.float32)
    for i, (x, y) in enumerate(recs):
        p = libm.powf(float(x), float(y))
        out[i] = p if p > 0.0 else 0.0  # fmaxf(0, NaN) = 0
    return out


def quantise16(lo, hi, qo, qs):
    """rtx_quant.h rtx_quantise in float64 on the float32 inputs: (lo16, hi16) grid planes"""
    lo, hi = lo.astype(np.float32).astype(np.float64), hi.astype(np.float32).astype(np.float64)
    qo, qs = qo.astype(np.float32).astype(np.float64), qs.astype(np.float32).astype(np.float64)
    a = np.floor((lo - qo) * qs) - 1.0
    b = np.ceil((hi - qo) * qs) + 1.0
    return np.clip(a, 0, 65535).astype(np.int64), np.clip(b, 0, 65535).astype(np.int64)


def box_q8_records(n=20000, seed=13):
    """box_q_records plus an 8-wide node frame per axis (rtx_device.h DW8): an origin at or below
    the box's 16-bit lo (down to the frame's 0) and a step exponent at or above the smallest one
    whose 255 steps reach the box's 16-bit hi (up to 3 more), as the 8-wide builder may choose
    for a box among siblings.  Record: o3 d3 lo3 hi3 qo3 qs3 tlim org3 e3."""
    rng = np.random.default_rng(seed)
    base = box_q_records(n, seed)
    ql, qh = quantise16(base[:, 6:9], base[:, 9:12], base[:, 12:15], base[:, 15:18])
    org = (ql * rng.random((n, 3)) ** 4).astype(np.int64)  # mostly close to lo, sometimes far below
    ext = qh - org
    e = np.zeros((n, 3), np.int64)
    while True:
        big = ((ext + (1 << e) - 1) >> e) > 255
        if not big.any():
            break
        e[big] += 1
    e += rng.integers(0, 4, (n, 3)) * (rng.random((n, 3)) < 0.3)
    e = np.minimum(e, 15)
    return np.concatenate([base, org.astype(np.float32), e.astype(np.float32)], 1).astype(np.float32)
