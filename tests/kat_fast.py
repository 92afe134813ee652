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
