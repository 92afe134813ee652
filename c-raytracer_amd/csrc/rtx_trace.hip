/*
 * MI355X (gfx950) closest-hit kernels for C-Raytracer's trace/shade path.
 *
 * The reference's cast_ray() recursion (render.c:136-343) runs per chunk of 8x8
 * pixel tiles as k_trace -> [shade-point sort] -> k_shadow (rtx_shadow.hip) -> k_accum:
 *
 *  k_trace  (persistent, one wave per workgroup; tiles from a device queue) every
 *           closest-hit query of the tile's ray trees: primaries, then
 *           reflection/refraction children from a per-wave LIFO task stack in HBM
 *           (__ballot/mbcnt compaction on push), and the path-GI samples of each
 *           batch flattened over (hit, sample) 64 at a time.  Per-lane BVH2
 *           traversal with the stack in LDS ([entry][lane], conflict-free).  Local
 *           terms (ke, ambient) go straight to the tile's pixels; every hit that
 *           sees lights becomes a 96-byte shade point (rtx_wave.h), appended in a
 *           fixed order to a per-wave staging region and moved to the chunk's
 *           contiguous array at tile end.
 *  k_accum  (one wave per tile) adds the shade points' light terms, computed by
 *           k_shadow, to their pixels in emission order.
 *  k_kat    per-function known answers of the device intersectors/samplers.
 *
 * No float atomics anywhere: a pixel's value is bit-identical whichever wave,
 * GPU or tile order renders it.
 */
#include <hip/hip_runtime.h>
#include <float.h>
#include <stdlib.h>

#include "rtx_kat.h"
#include "rtx_wave.h"
#include "rtx_w8.h"

/* ------------------------------------------------------------------------ */
/* closest hit: inside-object shortcut, planes, then BVH (render.c:118-147)  */
/* per-lane traversal, stack in LDS laid out [entry][lane]                  */
/* ------------------------------------------------------------------------ */
struct TraceCount {
	uint32_t nodes, tris, sph, pln, far;
};

template <bool COUNT>
__device__ void trace_closest_bvh2(const DScene &S, uint32_t *stk, bool act, f3 o, f3 d, uint32_t inside, float &t_out,
				   uint32_t &hid_out, TraceCount &tc)
{
	float tbest = FLT_MAX;
	uint32_t hid = RTX_NONE;
	if (act && isnan3(d)) /* TIR / degenerate directions hit nothing */
		act = false;
	if (act && inside != RTX_NONE) {
		float t;
		bool h;
		if (inside & RTX_PLANE_BIT) {
			const DPlane &pl = S.planes[inside & ~RTX_PLANE_BIT];
			h = hit_plane(ld3(pl.n), pl.d, o, d, pl.eps, t);
		} else {
			const DPrim &pr = S.prims[inside];
			if ((__float_as_uint(pr.c[3]) >> 24) == RTX_SPHERE)
				h = hit_sphere(mk3(pr.a[0], pr.a[1], pr.a[2]), pr.b[0], o, d, pr.a[3], t);
			else
				h = hit_triangle(mk3(pr.a[0], pr.a[1], pr.a[2]), mk3(pr.b[0], pr.b[1], pr.b[2]),
						 mk3(pr.c[0], pr.c[1], pr.c[2]), o, d, pr.a[3], t);
		}
		if (h) {
			tbest = t;
			hid = inside;
			act = false;
		}
	}
	if (act) {
		for (uint32_t i = 0; i < S.num_planes; i++) {
			const DPlane &pl = S.planes[i];
			float t;
			if (COUNT)
				tc.pln++;
			if (hit_plane(ld3(pl.n), pl.d, o, d, pl.eps, t) && t < tbest) {
				tbest = t;
				hid = RTX_PLANE_BIT | i;
			}
		}
	}
	if (act && S.root_ref != RTX_EMPTY_REF) {
		/* boxes in the trees' frame (rtx_device.h DTreeFrame), primitives in world space; a far
		 * origin's frame origin moves to t0 along the ray (tf_shift: boxes tested against tbest - t0) */
		const f3 db = S.tf.rotated ? tf_dir(S.tf.r, d) : d;
		const f3 inv = safe_inv(db);
		float t0 = 0.f;
		f3 ob = S.tf.rotated ? tf_point(S.tf.r, S.tf.c, o) : o;
		const bool far = tf_far(ob, S.tf.cf, S.tf.rad);
		if (far) {
			ob = tf_shift(S.tf.r, S.tf.c, S.tf.cf, S.tf.rad, o, d, t0);
			if (COUNT)
				tc.far++;
		}
		const f3 oi = mul3v(ob, inv);
		uint32_t ref = S.root_ref;
		uint32_t sp = 0;
		/* entries from RTX_TRACE_LSTK on live in HBM, [entry][grid lane]; lane addresses formed at
		 * each use (lane_id), none kept live across the walk */
		lds_u32 *ls = (lds_u32 *)stk;
		uint32_t *ostk = S.ostk + (size_t)blockIdx.x * WAVE;
		const size_t ostride = (size_t)gridDim.x * WAVE;
		auto push = [&](uint32_t v) {
			if (sp < RTX_TRACE_LSTK)
				ls[sp * WAVE + lane_id()] = v;
			else
				ostk[(sp - RTX_TRACE_LSTK) * ostride + lane_id()] = v;
			sp++;
		};
		auto pop = [&]() -> uint32_t {
			sp--;
			return sp < RTX_TRACE_LSTK ? ls[sp * WAVE + lane_id()] : ostk[(sp - RTX_TRACE_LSTK) * ostride + lane_id()];
		};
		for (;;) {
			if (ref & RTX_REF_LEAF) {
				const uint32_t first = (ref & RTX_REF_OFF) / (uint32_t)sizeof(DNode) - S.num_nodes,
					       cnt = (ref & RTX_REF_CNT) + 1;
				for (uint32_t k = 0; k < cnt; k++) {
					const float4 *pr = (const float4 *)(S.prims + first + k);
					const float4 a = pr[0], b = pr[1], c = pr[2];
					float t;
					bool h;
					if ((__float_as_uint(c.w) >> 24) == RTX_SPHERE) {
						if (COUNT)
							tc.sph++;
						h = (!far || far_sphere_box(mk3(a.x, a.y, a.z), b.x, o, d, t0, tbest - t0)) &&
						    hit_sphere(mk3(a.x, a.y, a.z), b.x, o, d, a.w, t);
					} else {
						if (COUNT)
							tc.tris++;
						h = hit_triangle(mk3(a.x, a.y, a.z), mk3(b.x, b.y, b.z), mk3(c.x, c.y, c.z), o, d,
								 a.w, t);
					}
					if (h && t < tbest) {
						tbest = t;
						hid = first + k;
					}
				}
				if (sp == 0)
					break;
				ref = pop();
			} else {
				const float4 *nd = (const float4 *)((const char *)S.nodes + (ref & RTX_REF_OFF));
				const float4 n0 = nd[0], n1 = nd[1], n2 = nd[2];
				const uint4 n3 = *(const uint4 *)(nd + 3);
				if (COUNT)
					tc.nodes++;
				float tn0, tn1;
				const float tlim = tbest - t0; /* tbest itself when t0 = 0 */
				const bool h0 = slab(n0.x, n0.y, n0.z, n0.w, n1.x, n1.y, oi, inv, tlim, tn0) && tn0 < tlim;
				const bool h1 = slab(n1.z, n1.w, n2.x, n2.y, n2.z, n2.w, oi, inv, tlim, tn1) && tn1 < tlim;
				if (h0 && h1) {
					/* nearer child first; tie -> right first (accel.c:341-345) */
					const bool l_first = tn0 < tn1;
					push(l_first ? n3.y : n3.x);
					ref = l_first ? n3.x : n3.y;
				} else if (h0) {
					ref = n3.x;
				} else if (h1) {
					ref = n3.y;
				} else {
					if (sp == 0)
						break;
					ref = pop();
				}
			}
		}
	}
	t_out = tbest;
	hid_out = hid;
}

/* Closest hit over the 8-wide compressed BVH (rtx_device.h DW8): the reference's
 * bvh_get_closest_intersection (accel.c:322-353) with eight children per node.  Hit leaf
 * slots are tested at once with the exact IEEE intersectors (the same t as the reference);
 * hit inner children are taken in the octant's visit order (front to back, roughly), the
 * first visited next, the rest kept as one group (base << 8 | mask) in a register and older
 * groups on the lane's stack (LDS, deeper entries in HBM), and every node's boxes are tested
 * against the current closest t.  The emitters the tree leaves out (DScene.w8noemit) are
 * tested before the walk.  Strict < everywhere: the first hit found at the least t wins. */
#ifndef RTX_TRACE_SCALAR
#define RTX_TRACE_SCALAR 1 /* a step where every lane is at one node reads its scalar-path copy (rtx_device.h DW8S) */
#endif
#ifndef RTX_TRACE_NEAR
#define RTX_TRACE_NEAR 1 /* closest hits: visit the nearest hit inner child first (scene6 k_trace 605 -> 417 ms) */
#endif
#ifndef RTX_TRACE_CULL
#define RTX_TRACE_CULL 0 /* closest hits: drop kept sibling groups that start beyond the closest hit */
#endif
#ifndef RTX_TRACE_EMPTYCOUNT
#define RTX_TRACE_EMPTYCOUNT 0 /* measurement builds: count only the visits that hit no child */
#endif
/* FAR: some lane of the wave has a far origin (t0 and the per-lane far flag live across the walk);
 * the other instances take t0 = 0 and no far lane as constants, so the waves of near rays (all of
 * them in the reference scenes' views) keep those registers for the walk */
template <bool COUNT, int OCT, bool FAR>
__device__ __forceinline__ void closest_walk8(const DScene &S, lds_u32 *stk, uint32_t *ostk, size_t ostride, f3 o, f3 d,
					      f3 ob, f3 inv, float t0_, bool far_, float &tbest, uint32_t &hid,
					      TraceCount &tc)
{
	const float t0 = FAR ? t0_ : 0.f;
	const bool far = FAR && far_;
	/* the lane stack: stk / ostk are the wave's bases (LDS, then HBM [entry][grid lane]); a lane's
	 * address is formed at each use (lane_id), none kept live across the walk */
	uint32_t sp = 0;
	auto push = [&](uint32_t v) {
		if (sp < RTX_TRACE_LSTK)
			stk[sp * WAVE + lane_id()] = v;
		else
			ostk[(sp - RTX_TRACE_LSTK) * ostride + lane_id()] = v;
		sp++;
	};
	auto pop = [&]() -> uint32_t {
		sp--;
		return sp < RTX_TRACE_LSTK ? stk[sp * WAVE + lane_id()] : ostk[(sp - RTX_TRACE_LSTK) * ostride + lane_id()];
	};
	constexpr uint32_t K = (OCT == 8 || !RTX_W8_ORDER) ? 0u : (~(uint32_t)OCT & 7u);
	/* ob / inv: the ray's origin and inverse direction in the trees' frame, ob at parameter t0 of
	 * the world ray o / d (tf_shift; 0 unless the origin is far): boxes are tested against tbest - t0 */
	const f3 qs = ld3(S.w8qs), qo = ld3(S.w8qo);
	const f3 invq = mk3(inv.x / qs.x, inv.y / qs.y, inv.z / qs.z);
	const f3 oq = mk3((ob.x - qo.x) * qs.x, (ob.y - qo.y) * qs.y, (ob.z - qo.z) * qs.z);
	const f3 oi = mul3v(oq, invq);
	uint32_t node = 0, grp = 0;
	float gt = -INFINITY; /* RTX_TRACE_CULL: least entry distance of the group in grp (-inf: unknown) */
	constexpr bool T = RTX_TRACE_NEAR || RTX_TRACE_CULL;
	while (node != RTX_NONE) {
		W8Visit v;
		uint32_t nearp = 8;
		float tin = INFINITY;
		const uint32_t un = uni(node);
		if (RTX_TRACE_SCALAR && !ballot(node != un)) {
			if (T) {
				const W8VisitT r = w8_visit_st<OCT, K>(S.w8s + (size_t)un, invq, oi, tbest - t0);
				v = r.v;
				nearp = r.near;
				tin = r.tin;
			} else {
				v = w8_visit_s<OCT, K>(S.w8s + (size_t)un, invq, oi, tbest - t0);
			}
		} else {
			uint32_t w[16];
			const DW8 *N = S.w8 + (size_t)node;
#pragma unroll
			for (int k = 0; k < 4; k++) {
				const uint4 x = ldg4u((const uint32_t *)N + 4 * k);
				w[4 * k] = x.x;
				w[4 * k + 1] = x.y;
				w[4 * k + 2] = x.z;
				w[4 * k + 3] = x.w;
			}
			if (T) {
				const W8VisitT r = w8_visit_t<OCT, K>(w, invq, oi, tbest - t0);
				v = r.v;
				nearp = r.near;
				tin = r.tin;
			} else {
				v = w8_visit<OCT, K, false>(w, invq, oi, tbest - t0);
			}
		}
		if (COUNT && (!RTX_TRACE_EMPTYCOUNT || !v.hm))
			tc.nodes++;
		uint32_t lm = v.hm & ~v.io, im = v.hm & v.io;
		while (lm) {
			const uint32_t p = __builtin_ctz(lm);
			lm &= lm - 1;
			const char *pr = (const char *)(S.w8 + v.base + (p ^ K));
			const float4 a = ldg4(pr, 0), b = ldg4(pr, 16), c = ldg4(pr, 32);
			float t = 0.f;
			bool h;
			if ((__float_as_uint(c.w) >> 24) == RTX_SPHERE) {
				if (COUNT)
					tc.sph++;
				h = (!far || far_sphere_box(mk3(a.x, a.y, a.z), b.x, o, d, t0, tbest - t0)) && /* rtx_math.h */
				    hit_sphere(mk3(a.x, a.y, a.z), b.x, o, d, a.w, t);
			} else {
				if (COUNT)
					tc.tris++;
				h = hit_triangle(mk3(a.x, a.y, a.z), mk3(b.x, b.y, b.z), mk3(c.x, c.y, c.z), o, d, a.w, t);
			}
			if (h && t < tbest) {
				tbest = t;
				hid = __float_as_uint(ldg4(pr, 48).w);
			}
		}
		if (RTX_TRACE_CULL && tin > tbest) /* every hit inner child starts beyond the closest hit */
			im = 0;
		if (im) {
			const uint32_t p0 = (RTX_TRACE_NEAR && nearp < 8) ? nearp : (uint32_t)__builtin_ctz(im);
			node = v.base + (p0 ^ K);
			im &= ~(1u << p0);
			if (im) {
				if (grp)
					push(grp);
				grp = (v.base << 8) | im;
				gt = tin;
			}
		} else {
			if (RTX_TRACE_CULL && grp && gt > tbest) { /* the kept group starts beyond the closest hit */
				grp = sp ? pop() : 0u;
				gt = -INFINITY;
			}
			if (grp) {
				node = (grp >> 8) + (__builtin_ctz(grp) ^ K);
				grp &= grp - 1;
				if (!(grp & 0xFFu)) {
					grp = sp ? pop() : 0u;
					gt = -INFINITY;
				}
			} else {
				node = RTX_NONE;
			}
		}
	}
}

template <bool COUNT>
__device__ void trace_closest_w8(const DScene &S, uint32_t *stk, bool act, f3 o, f3 d, uint32_t inside, float &t_out,
				 uint32_t &hid_out, TraceCount &tc)
{
	float tbest = FLT_MAX;
	uint32_t hid = RTX_NONE;
	if (act && isnan3(d)) /* TIR / degenerate directions hit nothing */
		act = false;
	if (act && inside != RTX_NONE) {
		float t;
		bool h;
		if (inside & RTX_PLANE_BIT) {
			const DPlane &pl = S.planes[inside & ~RTX_PLANE_BIT];
			h = hit_plane(ld3(pl.n), pl.d, o, d, pl.eps, t);
		} else {
			const DPrim &pr = S.prims[inside];
			if ((__float_as_uint(pr.c[3]) >> 24) == RTX_SPHERE)
				h = hit_sphere(mk3(pr.a[0], pr.a[1], pr.a[2]), pr.b[0], o, d, pr.a[3], t);
			else
				h = hit_triangle(mk3(pr.a[0], pr.a[1], pr.a[2]), mk3(pr.b[0], pr.b[1], pr.b[2]),
						 mk3(pr.c[0], pr.c[1], pr.c[2]), o, d, pr.a[3], t);
		}
		if (h) {
			tbest = t;
			hid = inside;
			act = false;
		}
	}
	if (act) {
		for (uint32_t i = 0; i < S.num_planes; i++) {
			const DPlane &pl = S.planes[i];
			float t;
			if (COUNT)
				tc.pln++;
			if (hit_plane(ld3(pl.n), pl.d, o, d, pl.eps, t) && t < tbest) {
				tbest = t;
				hid = RTX_PLANE_BIT | i;
			}
		}
	}
	const u64 live = ballot(act);
	if (live) {
		/* the ray in the trees' frame (rtx_device.h DTreeFrame) for the box tests */
		const bool rot = S.tf.rotated != 0;
		float t0 = 0.f;
		f3 ob = rot ? tf_point(S.tf.r, S.tf.c, o) : o;
		const bool far = act && tf_far(ob, S.tf.cf, S.tf.rad);
		if (far) { /* a far origin (tf_shift), in any frame */
			ob = tf_shift(S.tf.r, S.tf.c, S.tf.cf, S.tf.rad, o, d, t0);
			if (COUNT)
				tc.far++;
		}
		const f3 inv = safe_inv_fast(rot ? tf_dir(S.tf.r, d) : d);
		/* the emitters the tree leaves out, one by one (as the reference's tree holds them, a far
		 * ray meets an emitter's box first: its world box from the origin shifted to t0 in double) */
		if (act && S.w8noemit) {
			for (uint32_t i = 0; i < S.num_emitters; i++) {
				const DEmitter &e = S.emitters[i];
				float t = 0.f;
				if (far && !world_box_at(e.wlo[0], e.whi[0], e.wlo[1], e.whi[1], e.wlo[2], e.whi[2], o, d, t0, 1.f, tbest - t0))
					continue;
				bool h;
				if (e.type == RTX_SPHERE)
					h = hit_sphere(ld3(e.p0), e.radius, o, d, e.eps, t);
				else
					h = hit_triangle(ld3(e.p0), ld3(e.e1), ld3(e.e2), o, d, e.eps, t);
				if (h && t < tbest) {
					tbest = t;
					hid = e.prim;
				}
			}
		}
		lds_u32 *ls = (lds_u32 *)stk;
		uint32_t *ostk = S.ostk + (size_t)blockIdx.x * WAVE;
		const size_t ostride = (size_t)gridDim.x * WAVE;
		const uint32_t oct = ((~__float_as_uint(inv.x)) >> 31) | (((~__float_as_uint(inv.y)) >> 31) << 1) |
				     (((~__float_as_uint(inv.z)) >> 31) << 2);
		const uint32_t lead = readlane(oct, (uint32_t)__ffsll((long long)live) - 1);
		const uint32_t sel = ballot(act & (oct != lead)) ? 8u : lead;
		const bool anyfar = ballot(far) != 0;
		if (act && anyfar) {
			closest_walk8<COUNT, 8, true>(S, ls, ostk, ostride, o, d, ob, inv, t0, far, tbest, hid, tc);
		} else if (act) {
			switch (sel) {
#define RTX_CWALK(K)                                                                           \
	case K:                                                                                    \
		closest_walk8<COUNT, K, false>(S, ls, ostk, ostride, o, d, ob, inv, t0, far, tbest, hid, tc); \
		break;
				RTX_CWALK(0) RTX_CWALK(1) RTX_CWALK(2) RTX_CWALK(3) RTX_CWALK(4) RTX_CWALK(5) RTX_CWALK(6)
				RTX_CWALK(7)
#undef RTX_CWALK
			default:
				closest_walk8<COUNT, 8, false>(S, ls, ostk, ostride, o, d, ob, inv, t0, far, tbest, hid, tc);
				break;
			}
		}
	}
	t_out = tbest;
	hid_out = hid;
}

/* the closest-hit walk of this scene: the 8-wide tree when built and chosen (DScene.trace_w8) */
template <bool COUNT>
__device__ __forceinline__ void trace_closest(const DScene &S, uint32_t *stk, bool act, f3 o, f3 d, uint32_t inside,
					      float &t_out, uint32_t &hid_out, TraceCount &tc)
{
	if (S.trace_w8)
		trace_closest_w8<COUNT>(S, stk, act, o, d, inside, t_out, hid_out, tc);
	else
		trace_closest_bvh2<COUNT>(S, stk, act, o, d, inside, t_out, hid_out, tc);
}

struct HitInfo {
	f3 p, n;
	float b;
	bool outside;
	uint32_t obj, mat;
	float eps;
};

/* hit record of hid for ray (o,d) at t (object.c sphere 254-265, triangle 356-365, plane 473-488) */
__device__ __forceinline__ HitInfo hit_info(const DScene &S, uint32_t hid, f3 o, f3 d, float t)
{
	HitInfo h;
	h.p = add3(mul3s(d, t), o);
	if (hid & RTX_PLANE_BIT) {
		const DPlane &pl = S.planes[hid & ~RTX_PLANE_BIT];
		const f3 n = ld3(pl.n);
		h.n = signbit(dot3(n, d)) ? n : mul3s(n, -1.f);
		h.obj = pl.obj;
		h.mat = pl.mat;
		h.eps = pl.eps;
	} else {
		const DPrim &pr = S.prims[hid];
		const uint32_t meta = __float_as_uint(pr.c[3]);
		if ((meta >> 24) == RTX_SPHERE)
			h.n = mul3s(sub3(add3(mul3s(d, t), o), mk3(pr.a[0], pr.a[1], pr.a[2])), 1.f / pr.b[0]);
		else
			h.n = mk3(pr.d[0], pr.d[1], pr.d[2]);
		h.obj = __float_as_uint(pr.b[3]);
		h.mat = meta & RTX_META_MAT;
		h.eps = pr.a[3];
	}
	h.b = dot3(h.n, d);
	h.outside = signbit(h.b);
	return h;
}

/* ------------------------------------------------------------------------ */
/* shade points                                                             */
/*  - GI parents live in an LDS table inside k_trace (SPW floats each)      */
/*  - every shade point with lights is emitted as a 96-byte record          */
/*    (6 x float4) for k_shadow:                                            */
/*      q0 = P, W.x   q1 = n, W.y   q2 = d, W.z   q3 = tex, mat             */
/*      q4 = obj, key_lo, key_hi, nl   q5 = slot, -, -, -                   */
/* ------------------------------------------------------------------------ */
#define SPW 16

struct GiParent {
	f3 p;
	float eps;
	f3 n;
	float delta;
	f3 w;
	uint32_t slot;
	uint32_t key_lo, key_hi, ngi, pad;
};

__device__ __forceinline__ void gp_store(float *tab, uint32_t k, const GiParent &g)
{
	float4 *q = (float4 *)(tab + k * SPW);
	q[0] = make_float4(g.p.x, g.p.y, g.p.z, g.eps);
	q[1] = make_float4(g.n.x, g.n.y, g.n.z, g.delta);
	q[2] = make_float4(g.w.x, g.w.y, g.w.z, __uint_as_float(g.slot));
	q[3] = make_float4(__uint_as_float(g.key_lo), __uint_as_float(g.key_hi), __uint_as_float(g.ngi), 0.f);
}

__device__ __forceinline__ GiParent gp_load(const float *tab, uint32_t k)
{
	const float4 *q = (const float4 *)(tab + k * SPW);
	const float4 a = q[0], b = q[1], c = q[2], e = q[3];
	GiParent g;
	g.p = mk3(a.x, a.y, a.z);
	g.eps = a.w;
	g.n = mk3(b.x, b.y, b.z);
	g.delta = b.w;
	g.w = mk3(c.x, c.y, c.z);
	g.slot = __float_as_uint(c.w);
	g.key_lo = __float_as_uint(e.x);
	g.key_hi = __float_as_uint(e.y);
	g.ngi = __float_as_uint(e.z);
	return g;
}

struct ShadePt {
	f3 p, n, d, w, tex;
	uint32_t mat, obj, key_lo, key_hi, nl, slot;
};

/* RTX_SP_FAR for a shade point far from the bounded objects (rtx_math.h tf_far), whose shadow
 * rays k_shadow then walks from the light end; the test k_shadow made per ray before round 6,
 * made once per point, in any frame */
__device__ __forceinline__ uint32_t sp_far(const DTreeFrame &tf, f3 p)
{
	const f3 ob = tf.rotated ? tf_point(tf.r, tf.c, p) : p;
	return tf_far(ob, tf.cf, tf.rad) ? RTX_SP_FAR : 0u;
}

__device__ __forceinline__ void spr_store(float4 *rec, const ShadePt &s)
{
	rec[0] = make_float4(s.p.x, s.p.y, s.p.z, s.w.x);
	rec[1] = make_float4(s.n.x, s.n.y, s.n.z, s.w.y);
	rec[2] = make_float4(s.d.x, s.d.y, s.d.z, s.w.z);
	rec[3] = make_float4(s.tex.x, s.tex.y, s.tex.z, __uint_as_float(s.mat));
	rec[4] = make_float4(__uint_as_float(s.obj), __uint_as_float(s.key_lo), __uint_as_float(s.key_hi),
			     __uint_as_float(s.nl));
	rec[5] = make_float4(__uint_as_float(s.slot), 0.f, 0.f, 0.f);
}


/* ------------------------------------------------------------------------ */
/* k_trace: per 8x8 tile, every cast_ray() of the tile's ray trees          */
/* ------------------------------------------------------------------------ */
struct TraceOut {
	float4 *staging; /* this wave's staging region */
	uint32_t cap;    /* records */
	uint32_t n;      /* records written for the current tile (uniform) */
	bool overflow;
};

/* append the lanes' shade points (has) to the staging region, order = lane order */
__device__ __forceinline__ void emit_sp(TraceOut &T, bool has, const ShadePt &s)
{
	const u64 m = ballot(has);
	if (!m)
		return;
	const uint32_t pos = T.n + mbcnt(m);
	if (has && pos < T.cap)
		spr_store(T.staging + (size_t)pos * SPREC, s);
	T.n += popc64(m);
	if (T.n > T.cap)
		T.overflow = true;
}

template <bool COUNT>
__device__ __forceinline__ void gi_batch(const DScene &S, const DParams &P, uint32_t total_lights, uint32_t *stk,
					 float *gp_tab, uint32_t *off, uint32_t ngi_mine, f3 &acc, TraceOut &T,
					 TraceCount &tc, u64 &n_closest)
{
	uint32_t total;
	const uint32_t ex = wave_excl_scan(ngi_mine, &total);
	if (total == 0)
		return;
	lds_sync();
	off[lane_id()] = ex;
	if (lane_id() == 0)
		off[WAVE] = total;
	lds_sync();
	for (uint32_t base = 0; base < total; base += WAVE) {
		const uint32_t idx = base + lane_id();
		const bool act = idx < total;
		const uint32_t h = act ? owner_of(off, idx) : 0u;
		const GiParent par = gp_load(gp_tab, h);
		const uint32_t s = idx - off[h];
		const uint64_t pkey = key_of(par.key_lo, par.key_hi);
		float u1, u2;
		draw(P, pkey, RTX_STREAM_GI, s, u1, u2);
		/* render.c:270-286: uniform hemisphere sample about n, weight delta * (n . dir) */
		const f3 dir = gi_direction(par.n, par.eps, u1, u2);
		const f3 kr = mul3s(par.w, par.delta * dot3(par.n, dir));
		const uint64_t ckey = rtx_key_child(pkey, RTX_CHILD_GI0 + s);
		float t;
		uint32_t hid;
		trace_closest<COUNT>(S, stk, act, par.p, dir, RTX_NONE, t, hid, tc);
		n_closest += popc64(ballot(act));
		const bool hit = act && hid != RTX_NONE;
		ShadePt cs = ShadePt();
		f3 cc = mk3(0.f, 0.f, 0.f);
		bool has = false;
		if (hit) {
			/* child cast_ray(..., 0 bounces): ke + direct light only (path mode has no ambient term) */
			const HitInfo hi = hit_info(S, hid, par.p, dir, t);
			const DMaterial &m = S.mats[hi.mat];
			const f3 w = mul3s(kr, att_factor(P, t));
			cc = mul3v(w, ld3(m.ke));
			cs.nl = hi.outside ? lights_for(S, total_lights, hi.obj) : 0u;
			has = cs.nl != 0;
			cs.p = hi.p;
			cs.n = hi.n;
			cs.d = dir;
			cs.w = w;
			cs.mat = hi.mat;
			cs.obj = hi.obj | (has ? sp_far(S.tf, hi.p) : 0u);
			cs.slot = par.slot;
			cs.tex = has ? texture_color(m, hi.p, P.u32conv) : mk3(0.f, 0.f, 0.f);
			cs.key_lo = (uint32_t)ckey;
			cs.key_hi = (uint32_t)(ckey >> 32);
		}
		route_add(acc, hit, par.slot, cc);
		emit_sp(T, has, cs);
		lds_sync();
	}
}

template <bool COUNT>
#ifndef RTX_TRACE_OCC
#define RTX_TRACE_OCC 6 /* waves per SIMD k_trace is register-capped for (80 VGPRs; with 9 LDS stack entries, 24 waves per CU) */
#endif
__global__ __launch_bounds__(WAVE, RTX_TRACE_OCC) void k_trace(DScene S, DFrame F, DParams P, float *__restrict__ rgb,
						float *__restrict__ zbuf, DTask *__restrict__ tasks, uint32_t task_cap,
						float4 *__restrict__ staging, uint32_t staging_cap,
						float4 *__restrict__ sp_out, uint32_t sp_cap, uint2 *__restrict__ tile_rec,
						uint32_t tile_begin, uint32_t tile_end, unsigned long long *__restrict__ ctr)
{
	extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
	float *gp_tab = (float *)lds_raw;
	uint32_t *off = (uint32_t *)(lds_raw + WAVE * SPW * 4);
	uint32_t *stk = (uint32_t *)(lds_raw + WAVE * SPW * 4 + 80 * 4);

	uint32_t total_lights = 0;
	for (uint32_t e = 0; e < S.num_emitters; e++)
		total_lights += S.emitters[e].num_lights;
	u64 n_closest = 0;
	TraceCount tc = { 0, 0, 0, 0, 0 };
	DTask *my_tasks = tasks + (size_t)blockIdx.x * task_cap;
	TraceOut T;
	T.staging = staging + (size_t)blockIdx.x * staging_cap * SPREC;
	T.cap = staging_cap;
	bool overflow = false, task_overflow = false, sp_overflow = false;

	for (;;) {
		uint32_t tile = 0;
		if (lane_id() == 0)
			tile = (uint32_t)atomicAdd(&ctr[RTX_C_TILE], 1ull);
		tile = uni(__shfl(tile, 0, WAVE)) + tile_begin;
		if (tile >= tile_end)
			break;
		const uint32_t g = P.tile_offset + tile * P.tile_stride;
		const uint32_t tx = g % P.tiles_x, ty = g / P.tiles_x;
		const uint32_t px = tx * RTX_TILE_W + (lane_id() & 7), py = ty * RTX_TILE_H + (lane_id() >> 3);
		const bool valid_px = px < F.width && py < F.height;
		T.n = 0;
		T.overflow = false;

		f3 acc = mk3(0.f, 0.f, 0.f);
		float zval = 0.f;

		/* primary ray (render.c:353-363): P = corner + row*vy, then += vx (col+1) times, sequentially */
		bool act = valid_px;
		f3 o = ld3(F.origin), d = mk3(0.f, 0.f, 1.f), kr = mk3(1.f, 1.f, 1.f);
		uint32_t rb = P.max_bounces, inside = RTX_NONE, slot = lane_id();
		uint64_t key = 0;
		bool primary = true;
		if (act) {
			f3 pp = add3(mul3s(ld3(F.step_y), (float)py), ld3(F.corner));
			const f3 sx = ld3(F.step_x);
			for (uint32_t c = 0; c <= px; c++)
				pp = add3(pp, sx);
			d = norm3(sub3(pp, o));
			key = rtx_key_pixel(P.seed, py * F.width + px);
		}
		uint32_t top = 0;
		for (;;) {
			float t;
			uint32_t hid;
			lds_sync();
			trace_closest<COUNT>(S, stk, act, o, d, inside, t, hid, tc);
			n_closest += popc64(ballot(act));
			const bool hit = act && hid != RTX_NONE;
			ShadePt sp = ShadePt();
			GiParent gp = GiParent();
			f3 cc = mk3(0.f, 0.f, 0.f);
			bool has = false, want_refl = false, want_refr = false;
			f3 rkr = mk3(0.f, 0.f, 0.f), rkt = rkr, rdir = rkr, tdir = rkr;
			if (hit) {
				const HitInfo h = hit_info(S, hid, o, d, t);
				const DMaterial &m = S.mats[h.mat];
				const f3 w = mul3s(kr, att_factor(P, t));
				f3 local = ld3(m.ke);
				if (P.gi == RTX_GI_AMBIENT)
					local = add3(local, mul3v(ld3(m.ka), ld3(S.ambient)));
				cc = mul3v(w, local);
				if (primary)
					zval = rb ? t : 0.f; /* render.c:304-305, 342 */
				if (rb) {
					if (inside != hid && (m.flags & RTX_MF_REFLECTIVE)) { /* render.c:308-317 */
						rkr = mul3v(kr, ld3(m.kr));
						if (P.min_intensity_sqr < magsqr3(rkr)) {
							want_refl = true;
							rdir = sub3(d, mul3s(h.n, 2.f * h.b));
						}
					}
					if (m.flags & RTX_MF_TRANSPARENT) { /* render.c:320-340 */
						rkt = mul3v(kr, ld3(m.kt));
						if (P.min_intensity_sqr < magsqr3(rkt)) {
							want_refr = true;
							tdir = refract_dir(d, h.n, h.b, h.outside, m.ior);
						}
					}
				}
				sp.nl = h.outside ? lights_for(S, total_lights, h.obj) : 0u;
				has = sp.nl != 0;
				sp.p = h.p;
				sp.n = h.n;
				sp.d = d;
				sp.w = w;
				sp.mat = h.mat;
				sp.obj = h.obj | (has ? sp_far(S.tf, h.p) : 0u);
				sp.slot = slot;
				sp.tex = has ? texture_color(m, h.p, P.u32conv) : mk3(0.f, 0.f, 0.f);
				sp.key_lo = (uint32_t)key;
				sp.key_hi = (uint32_t)(key >> 32);
				gp.p = h.p;
				gp.eps = h.eps;
				gp.n = h.n;
				gp.w = w;
				gp.slot = slot;
				gp.key_lo = sp.key_lo;
				gp.key_hi = sp.key_hi;
				gp.ngi = (P.gi == RTX_GI_PATH && rb && h.outside) ? (rb == P.max_bounces ? P.samples : 1u) : 0u;
				gp.delta = (rb == P.max_bounces) ? 1.f / (float)P.samples : 1.f;
			}
			route_add(acc, hit, slot, cc);
			emit_sp(T, has, sp);
			/* push reflection / refraction children (compacted, LIFO) */
			{
				const u64 mr = ballot(want_refl), mt = ballot(want_refr);
				const uint32_t nr = popc64(mr), nt = popc64(mt);
				if (nr + nt) {
					if (top + nr + nt > task_cap) {
						task_overflow = true;
					} else {
						const uint32_t pos_r = top + mbcnt(mr), pos_t = top + nr + mbcnt(mt);
						if (want_refl) {
							const uint64_t k2 = rtx_key_child(key, RTX_CHILD_REFLECT);
							DTask tk;
							tk.o[0] = sp.p.x; tk.o[1] = sp.p.y; tk.o[2] = sp.p.z;
							tk.d[0] = rdir.x; tk.d[1] = rdir.y; tk.d[2] = rdir.z;
							tk.kr[0] = rkr.x; tk.kr[1] = rkr.y; tk.kr[2] = rkr.z;
							tk.rb = rb - 1;
							tk.inside = RTX_NONE;
							tk.key_lo = (uint32_t)k2;
							tk.key_hi = (uint32_t)(k2 >> 32);
							tk.slot = slot;
							my_tasks[pos_r] = tk;
						}
						if (want_refr) {
							const uint64_t k2 = rtx_key_child(key, RTX_CHILD_REFRACT);
							DTask tk;
							tk.o[0] = sp.p.x; tk.o[1] = sp.p.y; tk.o[2] = sp.p.z;
							tk.d[0] = tdir.x; tk.d[1] = tdir.y; tk.d[2] = tdir.z;
							tk.kr[0] = rkt.x; tk.kr[1] = rkt.y; tk.kr[2] = rkt.z;
							tk.rb = rb - 1;
							tk.inside = hid;
							tk.key_lo = (uint32_t)k2;
							tk.key_hi = (uint32_t)(k2 >> 32);
							tk.slot = slot;
							my_tasks[pos_t] = tk;
						}
						top += nr + nt;
					}
				}
			}
			/* path-traced GI children of this batch's hits (render.c:238-288) */
			if (P.gi == RTX_GI_PATH) {
				lds_sync();
				if (hit)
					gp_store(gp_tab, lane_id(), gp);
				gi_batch<COUNT>(S, P, total_lights, stk, gp_tab, off, hit ? gp.ngi : 0u, acc, T, tc,
						n_closest);
			}
			if (top == 0)
				break;
			/* next batch: pop up to 64 tasks */
			__builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
			const uint32_t n = min(top, (uint32_t)WAVE);
			top -= n;
			act = lane_id() < n;
			primary = false;
			if (act) {
				const DTask tk = my_tasks[top + lane_id()];
				o = ld3(tk.o);
				d = ld3(tk.d);
				kr = ld3(tk.kr);
				rb = tk.rb;
				inside = tk.inside;
				key = key_of(tk.key_lo, tk.key_hi);
				slot = tk.slot;
			}
			__builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
		}
		/* local terms + z of the tile; light terms are added by k_accum */
		if (valid_px) {
			const size_t pix = (size_t)py * F.width + px;
			if (rgb) {
				rgb[pix * 3 + 0] = acc.x;
				rgb[pix * 3 + 1] = acc.y;
				rgb[pix * 3 + 2] = acc.z;
			}
			if (zbuf)
				zbuf[pix] = zval;
		}
		/* move the tile's shade points to the chunk's contiguous array */
		uint32_t n = T.n;
		uint32_t start = 0;
		if (T.overflow) {
			overflow = true;
			n = 0;
		}
		if (lane_id() == 0)
			start = n ? (uint32_t)atomicAdd(&ctr[RTX_C_SPCOUNT], (unsigned long long)n) : 0u;
		start = uni(__shfl(start, 0, WAVE));
		if ((uint64_t)start + n > sp_cap) {
			sp_overflow = true;
			n = 0;
		}
		__builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
		for (uint32_t i = lane_id(); i < n * SPREC; i += WAVE)
			sp_out[(size_t)start * SPREC + i] = T.staging[i];
		if (lane_id() == 0)
			tile_rec[tile - tile_begin] = make_uint2(start, n);
	}
	if (COUNT) {
		u64 a = tc.nodes, b = tc.tris, c = tc.sph, d2 = tc.pln, f = tc.far;
#pragma unroll
		for (int o2 = 32; o2 > 0; o2 >>= 1) {
			a += __shfl_xor(a, o2, WAVE);
			b += __shfl_xor(b, o2, WAVE);
			c += __shfl_xor(c, o2, WAVE);
			d2 += __shfl_xor(d2, o2, WAVE);
			f += __shfl_xor(f, o2, WAVE);
		}
		if (lane_id() == 0) {
			atomicAdd(&ctr[RTX_C_NODES], a);
			atomicAdd(&ctr[RTX_C_TRIS], b);
			atomicAdd(&ctr[RTX_C_SPHERES], c);
			atomicAdd(&ctr[RTX_C_PLANES], d2);
			atomicAdd(&ctr[RTX_C_FARC], f);
		}
	}
	if (lane_id() == 0) {
		atomicAdd(&ctr[RTX_C_CLOSEST], n_closest);
		if (overflow)
			atomicAdd(&ctr[RTX_C_OVERFLOW], 1ull);
		if (task_overflow)
			atomicAdd(&ctr[RTX_C_TASKOVERFLOW], 1ull);
		if (sp_overflow)
			atomicAdd(&ctr[RTX_C_SPOVERFLOW], 1ull);
	}
}

/* ------------------------------------------------------------------------ */
/* k_accum: one wave per tile adds its shade points' light terms to the     */
/* tile's pixels in emission order (deterministic, no float atomics)        */
/* ------------------------------------------------------------------------ */
__global__ __launch_bounds__(WAVE) void k_accum(DFrame F, DParams P, const uint2 *__restrict__ tile_rec,
						 const float4 *__restrict__ contrib, uint32_t tile_begin,
						 float *__restrict__ rgb)
{
	const uint32_t t = blockIdx.x;
	const uint2 rec = tile_rec[t];
	f3 acc = mk3(0.f, 0.f, 0.f);
	for (uint32_t base = 0; base < rec.y; base += WAVE) {
		const bool valid = base + lane_id() < rec.y;
		float4 c = make_float4(0.f, 0.f, 0.f, 0.f);
		if (valid)
			c = contrib[rec.x + base + lane_id()];
		route_add(acc, valid, valid ? __float_as_uint(c.w) : 0u, mk3(c.x, c.y, c.z));
	}
	const uint32_t g = P.tile_offset + (tile_begin + t) * P.tile_stride;
	const uint32_t px = (g % P.tiles_x) * RTX_TILE_W + (lane_id() & 7), py = (g / P.tiles_x) * RTX_TILE_H + (lane_id() >> 3);
	if (px < F.width && py < F.height) {
		const size_t pix = (size_t)py * F.width + px;
		rgb[pix * 3 + 0] += acc.x;
		rgb[pix * 3 + 1] += acc.y;
		rgb[pix * 3 + 2] += acc.z;
	}
}

__global__ void k_kat(int kind, uint32_t n, const float *__restrict__ in, float *__restrict__ out, int u32mode)
{
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n)
		return;
	const int wi = rtx_kat_in_width[kind], wo = rtx_kat_out_width[kind];
	const float *x = in + (size_t)i * wi;
	float *y = out + (size_t)i * wo;
	for (int k = 0; k < wo; k++)
		y[k] = 0.f;
	switch (kind) {
	case RTX_KAT_MOLLER: {
		float t = 0.f;
		bool h = hit_triangle(ld3(x + 6), ld3(x + 9), ld3(x + 12), ld3(x), ld3(x + 3), x[15], t);
		y[0] = h;
		y[1] = h ? t : 0.f;
	} break;
	case RTX_KAT_SPHERE: {
		float t = 0.f;
		f3 o = ld3(x), d = ld3(x + 3), c = ld3(x + 6);
		bool h = hit_sphere(c, x[9], o, d, x[10], t);
		y[0] = h;
		if (h) {
			y[1] = t;
			f3 n = mul3s(sub3(add3(mul3s(d, t), o), c), 1.f / x[9]);
			y[2] = n.x;
			y[3] = n.y;
			y[4] = n.z;
		}
	} break;
	case RTX_KAT_PLANE: {
		float t = 0.f;
		f3 o = ld3(x), d = ld3(x + 3), nn = ld3(x + 6);
		bool h = hit_plane(nn, x[9], o, d, x[10], t);
		y[0] = h;
		if (h) {
			y[1] = t;
			f3 n = signbit(dot3(nn, d)) ? nn : mul3s(nn, -1.f);
			y[2] = n.x;
			y[3] = n.y;
			y[4] = n.z;
		}
	} break;
	case RTX_KAT_SLAB: {
		float tmin = 0.f, tmax = 0.f;
		bool h = slab_ref(ld3(x + 6), ld3(x + 9), x[12], ld3(x), ld3(x + 3), tmin, tmax);
		y[0] = h;
		y[1] = h ? tmin : 0.f;
		y[2] = h ? tmax : 0.f;
	} break;
	case RTX_KAT_NOISE:
		y[0] = simplex3(x[0], x[1], x[2]);
		break;
	case RTX_KAT_TEXTURE: {
		DMaterial m;
		m.tex = (int)x[0];
		m.periodic = (int)x[1];
		for (int k = 0; k < 3; k++) {
			m.color[0][k] = x[2 + k];
			m.color[1][k] = x[5 + k];
		}
		m.scale = x[8];
		m.mortar = x[9];
		m.nfs = x[10];
		m.ns = x[11];
		m.fs = x[12];
		f3 c = texture_color(m, ld3(x + 13), u32mode);
		y[0] = c.x;
		y[1] = c.y;
		y[2] = c.z;
	} break;
	case RTX_KAT_SPH_LIGHT:
	case RTX_KAT_TRI_LIGHT: {
		DEmitter e;
		f3 p = mk3(0.f, 0.f, 0.f);
		float u1, u2;
		if (kind == RTX_KAT_SPH_LIGHT) {
			e.type = RTX_SPHERE;
			for (int k = 0; k < 3; k++)
				e.p0[k] = x[k];
			e.radius = x[3];
			p = ld3(x + 4);
			u1 = x[7];
			u2 = x[8];
		} else {
			e.type = RTX_TRIANGLE;
			for (int k = 0; k < 3; k++) {
				e.p0[k] = x[k];
				e.p1[k] = x[3 + k];
				e.p2[k] = x[6 + k];
			}
			u1 = x[9];
			u2 = x[10];
		}
		f3 l = light_point(e, p, u1, u2);
		y[0] = l.x;
		y[1] = l.y;
		y[2] = l.z;
	} break;
	case RTX_KAT_MORTON: {
		/* accel.c:72-88 (used by the reference's BVH build; kept for parity of the KAT suite) */
		uint32_t c = 0;
		for (int a = 0; a < 3; a++) {
			uint32_t v = (uint32_t)(1023.f * x[a]);
			v = (v * 0x00010001u) & 0xFF0000FFu;
			v = (v * 0x00000101u) & 0x0F00F00Fu;
			v = (v * 0x00000011u) & 0xC30C30C3u;
			v = (v * 0x00000005u) & 0x49249249u;
			c += v * (a == 0 ? 4u : a == 1 ? 2u : 1u);
		}
		y[0] = __uint_as_float(c);
	} break;
	case RTX_KAT_U32:
		y[0] = __uint_as_float(to_u32(x[0], RTX_U32_SAT));
		y[1] = __uint_as_float(to_u32(x[0], RTX_U32_WRAP));
		break;
	case RTX_KAT_GI_DIR: {
		f3 dd = gi_direction(ld3(x), x[3], x[4], x[5]);
		y[0] = dd.x;
		y[1] = dd.y;
		y[2] = dd.z;
	} break;
	case RTX_KAT_REFRACT: {
		f3 dd = ld3(x), nn = ld3(x + 3);
		float b = dot3(nn, dd);
		f3 r = refract_dir(dd, nn, b, signbit(b), x[6]);
		y[0] = r.x;
		y[1] = r.y;
		y[2] = r.z;
	} break;
	}
}

/* ------------------------------------------------------------------------ */
/* launchers (called from rtx_api.cpp)                                      */
/* ------------------------------------------------------------------------ */
extern "C" size_t rtx_trace_lds_bytes(uint32_t stack_size)
{
	size_t pad = 0;
#if RTX_MEASURE
	/* RTX_TRACE_LDS_PAD (measurement builds): extra bytes per wave, to read k_trace's occupancy slope */
	const char *e = getenv("RTX_TRACE_LDS_PAD");
	pad = e ? (size_t)atoi(e) : 0;
#endif
	const size_t lstk = stack_size < RTX_TRACE_LSTK ? stack_size : RTX_TRACE_LSTK;
	return (size_t)WAVE * SPW * 4 + 80 * 4 + lstk * WAVE * 4 + pad;
}

extern "C" hipError_t rtx_trace_occupancy(uint32_t stack_size, int *blocks_per_cu)
{
	return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, k_trace<false>, WAVE,
							     rtx_trace_lds_bytes(stack_size));
}

extern "C" hipError_t rtx_launch_trace(const DScene *S, const DFrame *F, const DParams *P, float *rgb, float *z,
				       DTask *tasks, uint32_t task_cap, float4 *staging, uint32_t staging_cap,
				       float4 *sp_out, uint32_t sp_cap, uint2 *tile_rec, uint32_t tile_begin,
				       uint32_t tile_end, unsigned long long *ctr, uint32_t waves, int count,
				       hipStream_t stream)
{
	const size_t lds = rtx_trace_lds_bytes(S->stack_size);
	if (count)
		hipLaunchKernelGGL(k_trace<true>, dim3(waves), dim3(WAVE), lds, stream, *S, *F, *P, rgb, z, tasks, task_cap,
				   staging, staging_cap, sp_out, sp_cap, tile_rec, tile_begin, tile_end, ctr);
	else
		hipLaunchKernelGGL(k_trace<false>, dim3(waves), dim3(WAVE), lds, stream, *S, *F, *P, rgb, z, tasks,
				   task_cap, staging, staging_cap, sp_out, sp_cap, tile_rec, tile_begin, tile_end, ctr);
	return hipGetLastError();
}

extern "C" hipError_t rtx_launch_accum(const DFrame *F, const DParams *P, const uint2 *tile_rec,
				       const float4 *contrib, uint32_t tile_begin, uint32_t ntiles, float *rgb,
				       hipStream_t stream)
{
	if (!ntiles || !rgb)
		return hipSuccess;
	hipLaunchKernelGGL(k_accum, dim3(ntiles), dim3(WAVE), 0, stream, *F, *P, tile_rec, contrib, tile_begin, rgb);
	return hipGetLastError();
}

extern "C" hipError_t rtx_launch_kat(int kind, uint32_t n, const float *in, float *out, int u32mode,
				     hipStream_t stream)
{
	hipLaunchKernelGGL(k_kat, dim3((n + 255) / 256), dim3(256), 0, stream, kind, n, in, out, u32mode);
	return hipGetLastError();
}

/* the code object of this file on the current device, loaded now (rtx_open) rather than at the
 * first launch inside an upload or a render */
extern "C" __attribute__((visibility("hidden"))) hipError_t rtx_load_trace(void)
{
	hipFuncAttributes a;
	return hipFuncGetAttributes(&a, (const void *)k_accum);
}
