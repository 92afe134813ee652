/*
 * MI355X (gfx950) kernels for C-Raytracer's trace/intersect/shade hot path.
 *
 * The reference's cast_ray() recursion (render.c:136-343) is evaluated as three
 * kernels per chunk of 8x8 pixel tiles, one wavefront per workgroup:
 *
 *  k_trace  (persistent; tiles from a device queue, one returning atomic each)
 *           every closest-hit query of the tile's ray trees: primaries, then
 *           reflection/refraction children from a per-wave LIFO task stack in
 *           HBM (__ballot/mbcnt compaction on push), and the path-GI samples
 *           of each batch flattened over (hit, sample) 64 at a time.  Per-lane
 *           BVH2 traversal with the stack in LDS ([entry][lane]).  Local terms
 *           (ke, ambient) go straight to the tile's pixels; every hit that sees
 *           lights becomes a 96-byte shade point, appended in a fixed order to
 *           a per-wave staging region and moved to the chunk's contiguous
 *           array at tile end.
 *  k_shadow (one wave per few shade points) direct lighting, the dominant
 *           work (95.9-99.6 % of all rays): (point, light) pairs flattened and
 *           traced 64 at a time as a PACKET - node and primitive indices are
 *           wave-uniform, every lane tests its own shadow ray, __ballot picks
 *           the children.  Shadow rays of one hit all aim at one small emitter,
 *           so packets stay coherent.  Per-point sums by deterministic
 *           segmented wave reductions.
 *  k_accum  (one wave per tile) adds the points' light terms to their pixels
 *           in emission order.
 *
 * No float atomics anywhere: a pixel's value is bit-identical whichever wave,
 * GPU or tile order renders it.
 */
#include <hip/hip_runtime.h>
#include <float.h>
#include <stdlib.h>

#include "rtx_kat.h"
#include "rtx_math.h"
#include "rtx_rng.h"

#define WAVE 64
/* shadow-walk build switches (measurement variants; defaults are the tuned choice) */
#ifndef RTX_SH_PF
#define RTX_SH_PF 1  /* touch the children's records before the current step's tests */
#endif
#ifndef RTX_SH_OCT
#define RTX_SH_OCT 1 /* specialise the box test on a packet-uniform direction octant */
#endif
#ifndef RTX_SH_PK
#define RTX_SH_PK 0  /* slab planes by packed FMA (v_pk_fma_f32): fewer VALU, measured 3% slower */
#endif
#ifndef RTX_DEBUG_NOWALK
#define RTX_DEBUG_NOWALK 0 /* measurement only: skip the BVH walk (per-packet overhead) */
#endif
#ifndef RTX_DEBUG_NOLEAF
#define RTX_DEBUG_NOLEAF 0 /* register-pressure experiments only */
#endif
#ifndef RTX_SH_FMA
#define RTX_SH_FMA 1 /* fused products in the shadow triangle test */
#endif
#ifndef RTX_SH_RAWMIN
#define RTX_SH_RAWMIN 1 /* segment-end min of the octant box test in asm (no canonicalise) */
#endif
#ifndef RTX_SH_MASK
#define RTX_SH_MASK 1 /* triangle any-hit decided on wave masks (no VGPR round trip) */
#endif
#ifndef RTX_SH_RCP
#define RTX_SH_RCP 1 /* any-hit triangle test with v_rcp_f32 instead of IEEE 1/a */
#endif
#ifndef RTX_SHADOW_OCC_R
#define RTX_SHADOW_OCC_R 6 /* waves/SIMD cap of the R-rays-per-lane walk (1: compiler's choice) */
#endif
#ifndef RTX_SHADOW_OCC_DEFAULT
#define RTX_SHADOW_OCC_DEFAULT 8
#endif


/* ------------------------------------------------------------------------ */
/* wave helpers                                                             */
/* ------------------------------------------------------------------------ */
typedef unsigned long long u64;
typedef uint32_t v16u __attribute__((ext_vector_type(16)));

__device__ __forceinline__ u64 ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }
__device__ __forceinline__ uint32_t popc64(u64 m) { return (uint32_t)__popcll(m); }
__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }
__device__ __forceinline__ uint32_t mbcnt(u64 m)
{
	return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint32_t readlane(uint32_t v, uint32_t l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ float readlanef(float v, uint32_t l)
{
	return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ bool lane_in(u64 m) { return (m >> lane_id()) & 1ull; }

/* deterministic butterfly sum: every lane gets the same total */
__device__ __forceinline__ float wave_sum(float v)
{
#pragma unroll
	for (int o = 32; o > 0; o >>= 1)
		v += __shfl_xor(v, o, WAVE);
	return v;
}

/* exclusive prefix sum over the wave; *tot = total (uniform) */
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v, uint32_t *tot)
{
	uint32_t x = v;
#pragma unroll
	for (int o = 1; o < WAVE; o <<= 1) {
		uint32_t y = __shfl_up(x, o, WAVE);
		if ((int)lane_id() >= o)
			x += y;
	}
	*tot = uni(__shfl(x, WAVE - 1, WAVE));
	return x - v;
}

/* largest k in [0,64) with off[k] <= idx, for off[0] = 0 <= idx < off[64] */
__device__ __forceinline__ uint32_t owner_of(const uint32_t *off, uint32_t idx)
{
	uint32_t lo = 0, hi = WAVE;
	while (hi - lo > 1) {
		uint32_t mid = (lo + hi) >> 1;
		if (off[mid] <= idx)
			lo = mid;
		else
			hi = mid;
	}
	return lo;
}

__device__ __forceinline__ void lds_sync()
{
	__builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
	__builtin_amdgcn_wave_barrier();
	__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

/* add c (per lane) into the accumulator of pixel slot `slot` (owned by lane `slot`), fixed order */
__device__ __forceinline__ void route_add(f3 &acc, bool valid, uint32_t slot, f3 c)
{
	u64 m = ballot(valid);
	if (!m)
		return;
	if (!ballot(valid && slot != lane_id())) {
		if (valid)
			acc = add3(acc, c);
		return;
	}
	const uint32_t s0 = readlane(slot, (uint32_t)__ffsll((long long)m) - 1);
	if (!ballot(valid && slot != s0)) {
		float sx = wave_sum(valid ? c.x : 0.f), sy = wave_sum(valid ? c.y : 0.f), sz = wave_sum(valid ? c.z : 0.f);
		if (lane_id() == s0)
			acc = add3(acc, mk3(sx, sy, sz));
		return;
	}
	while (m) {
		const uint32_t i = (uint32_t)__ffsll((long long)m) - 1;
		m &= m - 1;
		const uint32_t s = readlane(slot, i);
		const float x = readlanef(c.x, i), y = readlanef(c.y, i), z = readlanef(c.z, i);
		if (lane_id() == s)
			acc = add3(acc, mk3(x, y, z));
	}
}

__device__ __forceinline__ uint64_t key_of(uint32_t lo, uint32_t hi) { return ((uint64_t)hi << 32) | lo; }

__device__ __forceinline__ void draw(const DParams &P, uint64_t key, uint32_t stream, uint32_t idx, float &u1, float &u2)
{
	if (P.rng == RTX_RNG_CONST) {
		u1 = 0.5f;
		u2 = 0.5f;
	} else {
		rtx_draw2(key, stream, idx, &u1, &u2);
	}
}

__device__ __forceinline__ float att_factor(const DParams &P, float dist)
{
	if (P.attenuation == RTX_ATT_LIN)
		return 1.f / (P.att_offset + dist);
	if (P.attenuation == RTX_ATT_SQR) {
		float q = P.att_offset + dist;
		return 1.f / (q * q);
	}
	return 1.f;
}

/* lights a shade point on object `obj` samples: num_lights summed over emitters != obj (render.c:172-174) */
__device__ __forceinline__ uint32_t lights_for(const DScene &S, uint32_t total, uint32_t obj)
{
	uint32_t n = total;
	for (uint32_t e = 0; e < S.num_emitters; e++)
		if (S.emitters[e].obj == obj)
			n -= S.emitters[e].num_lights;
	return n;
}

/* ------------------------------------------------------------------------ */
/* closest hit: inside-object shortcut, planes, then BVH (render.c:118-147)  */
/* per-lane traversal, stack in LDS laid out [entry][lane]                  */
/* ------------------------------------------------------------------------ */
struct TraceCount {
	uint32_t nodes, tris, sph, pln;
};

template <bool COUNT>
__device__ void trace_closest(const DScene &S, uint32_t *stk, bool act, f3 o, f3 d, uint32_t inside, float &t_out,
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
		const f3 inv = safe_inv(d);
		const f3 oi = mul3v(o, inv);
		uint32_t ref = S.root_ref;
		uint32_t sp = 0;
		stk += lane_id();
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
						h = hit_sphere(mk3(a.x, a.y, a.z), b.x, o, d, a.w, t);
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
				ref = stk[--sp * WAVE];
			} else {
				const float4 *nd = (const float4 *)((const char *)S.nodes + (ref & RTX_REF_OFF));
				const float4 n0 = nd[0], n1 = nd[1], n2 = nd[2];
				const uint4 n3 = *(const uint4 *)(nd + 3);
				if (COUNT)
					tc.nodes++;
				float tn0, tn1;
				const bool h0 = slab(n0.x, n0.y, n0.z, n0.w, n1.x, n1.y, oi, inv, tbest, tn0) && tn0 < tbest;
				const bool h1 = slab(n1.z, n1.w, n2.x, n2.y, n2.z, n2.w, oi, inv, tbest, tn1) && tn1 < tbest;
				if (h0 && h1) {
					/* nearer child first; tie -> right first (accel.c:341-345) */
					const bool l_first = tn0 < tn1;
					stk[sp++ * WAVE] = l_first ? n3.y : n3.x;
					ref = l_first ? n3.x : n3.y;
				} else if (h0) {
					ref = n3.x;
				} else if (h1) {
					ref = n3.y;
				} else {
					if (sp == 0)
						break;
					ref = stk[--sp * WAVE];
				}
			}
		}
	}
	t_out = tbest;
	hid_out = hid;
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

#define SPREC 6 /* float4 per shade-point record */

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
			cs.obj = hi.obj;
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
__global__ __launch_bounds__(WAVE) void k_trace(DScene S, DFrame F, DParams P, float *__restrict__ rgb,
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
	TraceCount tc = { 0, 0, 0, 0 };
	DTask *my_tasks = tasks + (size_t)blockIdx.x * task_cap;
	TraceOut T;
	T.staging = staging + (size_t)blockIdx.x * staging_cap * SPREC;
	T.cap = staging_cap;
	bool overflow = false, sp_overflow = false;

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
				sp.obj = h.obj;
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
						overflow = true;
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
		u64 a = tc.nodes, b = tc.tris, c = tc.sph, d2 = tc.pln;
#pragma unroll
		for (int o2 = 32; o2 > 0; o2 >>= 1) {
			a += __shfl_xor(a, o2, WAVE);
			b += __shfl_xor(b, o2, WAVE);
			c += __shfl_xor(c, o2, WAVE);
			d2 += __shfl_xor(d2, o2, WAVE);
		}
		if (lane_id() == 0) {
			atomicAdd(&ctr[RTX_C_NODES], a);
			atomicAdd(&ctr[RTX_C_TRIS], b);
			atomicAdd(&ctr[RTX_C_SPHERES], c);
			atomicAdd(&ctr[RTX_C_PLANES], d2);
		}
	}
	if (lane_id() == 0) {
		atomicAdd(&ctr[RTX_C_CLOSEST], n_closest);
		if (overflow)
			atomicAdd(&ctr[RTX_C_OVERFLOW], 1ull);
		if (sp_overflow)
			atomicAdd(&ctr[RTX_C_SPOVERFLOW], 1ull);
	}
}

/* ------------------------------------------------------------------------ */
/* k_shadow: direct lighting (render.c:170-229) of shade points.            */
/* A wave takes `per_wave` consecutive shade points, flattens their         */
/* (point, light sample) pairs and walks the BVH with 64 shadow rays at a   */
/* time as a packet: node / primitive indices are wave-uniform (scalar      */
/* loads), each lane tests its own ray, __ballot picks the children.        */
/* ------------------------------------------------------------------------ */
struct ShadowCount {
	u64 nodes, tris, sph, pln, steps, psteps;
	u64 rnodes, rprims; /* per-ray need: inner nodes / leaf primitives under boxes the ray hits */
};

/* count mode: the rays of ballot b that hit the child `ref` would visit it in a ray-by-ray walk */
__device__ __forceinline__ void count_need(ShadowCount &sc, u64 b, uint32_t ref)
{
	if (ref & RTX_REF_LEAF)
		sc.rprims += (u64)popc64(b) * ((ref & RTX_REF_CNT) + 1);
	else
		sc.rnodes += popc64(b);
}

/* 64-byte BVH records are read through the constant address space: with a wave-uniform
 * address that is one s_load_dwordx16 into SGPRs, whatever the compiler can prove about
 * where the base pointer came from (the records are never written while a kernel runs) */
typedef const v16u __attribute__((address_space(4))) *crec_t;

__device__ __forceinline__ v16u rec_load(const char *recs, uint32_t off) { return *(crec_t)(recs + off); }

/* the same for other read-only scene tables indexed by wave-uniform values (s_load) */
template <typename T> __device__ __forceinline__ const __attribute__((address_space(4))) T *cptr(const T *p)
{
	return (const __attribute__((address_space(4))) T *)p;
}

/* prefetch: one dword of a record (s_load_dword), which brings its 64-byte line into the
 * scalar cache and L2 while this step computes.  Issued by inline asm so the compiler neither
 * sinks it nor waits for it; its destination SGPR stays live (hence untouched) until
 * consume(), which takes a field of the next record as an input and so sits behind that
 * record's lgkmcnt(0) wait, which has drained the touch too. */
__device__ __forceinline__ uint32_t touch(const char *recs, uint32_t off)
{
	uint32_t v;
	asm volatile("s_load_dword %0, %1, %2" : "=s"(v) : "s"(recs), "s"(off));
	return v;
}
__device__ __forceinline__ void consume(uint32_t a, uint32_t b, uint32_t dep)
{
	asm volatile("; consume %0 %1 %2" ::"s"(a), "s"(b), "s"(dep));
}
/* drain outstanding touches before their registers can be reused (walk exit) */
__device__ __forceinline__ void drain(uint32_t a, uint32_t b)
{
	asm volatile("s_waitcnt lgkmcnt(0)\n\t; drained %0 %1" ::"s"(a), "s"(b));
}

/* child-box test of the packet walk (the slab test of accel.c:112-158 on padded boxes).
 * OCT < 8: every live ray's direction lies in octant OCT (bit a set = inv[a] >= 0), so each
 * axis' entry plane is known at compile time and the per-axis min/max of `slab` drop out;
 * fma is monotone in the plane coordinate, so the answer is the same as slab()'s. */
typedef float f2v __attribute__((ext_vector_type(2)));

/* both slab planes of one axis by one packed FMA (v_pk_fma_f32): (lo, hi) * inv - o * inv */
__device__ __forceinline__ f2v slab_pair(uint32_t lo, uint32_t hi, float inv, float oi)
{
	const f2v p = { __uint_as_float(lo), __uint_as_float(hi) };
	const f2v m = { inv, inv }, c = { -oi, -oi };
	return RTX_SH_PK ? __builtin_elementwise_fma(p, m, c) : f2v{ fmaf(p.x, inv, -oi), fmaf(p.y, inv, -oi) };
}

template <int OCT>
__device__ __forceinline__ bool box_hit(const v16u &nd, const uint32_t b, f3 oi, f3 inv, float tlim)
{
	const f2v tx = slab_pair(nd[b], nd[b + 1], inv.x, oi.x);
	const f2v ty = slab_pair(nd[b + 2], nd[b + 3], inv.y, oi.y);
	const f2v tz = slab_pair(nd[b + 4], nd[b + 5], inv.z, oi.z);
	if (OCT == 8) {
		const float tn = fmaxf(fmaxf(fminf(tx.x, tx.y), fminf(ty.x, ty.y)), fmaxf(fminf(tz.x, tz.y), 0.f));
		const float tf = fminf(fminf(fmaxf(tx.x, tx.y), fmaxf(ty.x, ty.y)), fminf(fmaxf(tz.x, tz.y), tlim));
		return tn <= tf;
	}
	const float nx = (OCT & 1) ? tx.x : tx.y, fx = (OCT & 1) ? tx.y : tx.x;
	const float ny = (OCT & 2) ? ty.x : ty.y, fy = (OCT & 2) ? ty.y : ty.x;
	const float nz = (OCT & 4) ? tz.x : tz.y, fz = (OCT & 4) ? tz.y : tz.x;
	const float tn = fmaxf(fmaxf(nx, ny), fmaxf(nz, 0.f));
#if RTX_SH_RAWMIN
	/* min with the segment end in asm: tlim is a loop-carried value the compiler would
	 * canonicalise before every fminf (one extra VALU per node step); no NaN reaches here */
	float tf = fminf(fminf(fx, fy), fz);
	asm("v_min_f32 %0, %0, %1" : "+v"(tf) : "v"(tlim));
#else
	const float tf = fminf(fminf(fx, fy), fminf(fz, tlim));
#endif
	return tn <= tf;
}

/* moller_trumbore (object.c:422-441) as a branch-free any-hit test on (eps, tlim), with the
 * same accept set for finite inputs:
 *   reject |a| < eps;  reject u < 0, v < 0, u + v > 1 (u > 1 is implied);  accept eps < t < tlim.
 * Whenever t is finite, f = 1/a and u, v are finite too, so the three sign conditions fold into
 * one max3 compare and the t window into one min compare (a NaN or infinite t fails it).
 * 1/a by v_rcp_f32 (1 ulp): only the hit/miss decision is used. */
__device__ __forceinline__ f3 cross3_fma(f3 a, f3 b)
{
	return mk3(fmaf(a.y, b.z, -a.z * b.y), fmaf(a.z, b.x, -a.x * b.z), fmaf(a.x, b.y, -a.y * b.x));
}
__device__ __forceinline__ float dot3_fma(f3 a, f3 b) { return fmaf(a.x, b.x, fmaf(a.y, b.y, a.z * b.z)); }

__device__ __forceinline__ bool any_tri(f3 v0, f3 e1, f3 e2, f3 o, f3 d, float eps, float tlim)
{
	/* products fused (RTX_SH_FMA): 40 instead of 57 VALU; only hit decisions at exact
	 * edges can change, as with the 1-ulp reciprocal */
	const f3 h = RTX_SH_FMA ? cross3_fma(d, e2) : cross3(d, e2);
	const float a = RTX_SH_FMA ? dot3_fma(e1, h) : dot3(e1, h);
	const float f = RTX_SH_RCP ? __builtin_amdgcn_rcpf(a) : 1.f / a;
	const f3 s = sub3(o, v0);
	const float u = f * (RTX_SH_FMA ? dot3_fma(s, h) : dot3(s, h));
	const f3 q = RTX_SH_FMA ? cross3_fma(s, e1) : cross3(s, e1);
	const float v = f * (RTX_SH_FMA ? dot3_fma(d, q) : dot3(d, q));
	const float t = f * (RTX_SH_FMA ? dot3_fma(e2, q) : dot3(e2, q));
	const float out = fmaxf(fmaxf(-u, -v), (u + v) - 1.f); /* > 0: outside the triangle */
	return ((int)(fabsf(a) >= eps) & (int)(out <= 0.f) & (int)(fminf(t - eps, tlim - t) > 0.f)) != 0;
}

/* any_tri as a wave mask: each compare's ballot is its v_cmp result, ANDed on the scalar
 * unit (a per-lane bool would be materialised in a VGPR and compared back before the branch) */
__device__ __forceinline__ u64 any_tri_mask(f3 v0, f3 e1, f3 e2, f3 o, f3 d, float eps, float tlim)
{
	const f3 h = cross3_fma(d, e2);
	const float a = dot3_fma(e1, h);
	const float f = RTX_SH_RCP ? __builtin_amdgcn_rcpf(a) : 1.f / a;
	const f3 s = sub3(o, v0);
	const float u = f * dot3_fma(s, h);
	const f3 q = cross3_fma(s, e1);
	const float v = f * dot3_fma(d, q);
	const float t = f * dot3_fma(e2, q);
	const float out = fmaxf(fmaxf(-u, -v), (u + v) - 1.f);
	return ballot(fabsf(a) >= eps) & ballot(out <= 0.f) & ballot(fminf(t - eps, tlim - t) > 0.f);
}

/* per-lane select by a wave mask held in SGPRs: m's bit set -> b, else a */
__device__ __forceinline__ float msel(u64 m, float a, float b)
{
	float r;
	asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(m));
	return r;
}

/* one primitive of a leaf against the packet (accel.c:362-373): the target emitter skipped,
 * opaque hit -> the lane is blocked (tl = -1: no later test can hit it), transparent hit ->
 * li *= kt.  Returns true when a lane was blocked. */
template <bool COUNT>
__device__ __forceinline__ bool shadow_prim(const v16u &pr, const DMaterial *__restrict__ mats, f3 o, f3 d, float &tl,
					    uint32_t emit_u, uint32_t emit_obj, f3 &li, ShadowCount &sc)
{
	const uint32_t meta = pr[11], obj = pr[7];
	if (obj == emit_u)
		return false;
	const f3 a = mk3(__uint_as_float(pr[0]), __uint_as_float(pr[1]), __uint_as_float(pr[2]));
	bool h;
	if ((meta >> 24) == RTX_SPHERE) {
		if (COUNT)
			sc.sph += popc64(ballot(tl >= 0.f));
		if (COUNT)
			sc.psteps++;
		float t = 0.f;
		h = hit_sphere(a, __uint_as_float(pr[4]), o, d, __uint_as_float(pr[3]), t) & (t < tl);
	} else {
		if (COUNT)
			sc.tris += popc64(ballot(tl >= 0.f));
		if (COUNT)
			sc.psteps++;
		h = any_tri(a, mk3(__uint_as_float(pr[4]), __uint_as_float(pr[5]), __uint_as_float(pr[6])),
			    mk3(__uint_as_float(pr[8]), __uint_as_float(pr[9]), __uint_as_float(pr[10])), o, d,
			    __uint_as_float(pr[3]), tl);
	}
	if (emit_u == RTX_NONE) /* the packet's rays aim at different emitters */
		h = h & (obj != emit_obj);
	if (!ballot(h))
		return false;
	if (meta & RTX_META_TRANSPARENT) {
		const auto *m = cptr(mats) + (meta & RTX_META_MAT);
		const f3 kt = mk3(m->kt[0], m->kt[1], m->kt[2]);
		if (h)
			li = mul3v(li, kt);
		return false;
	}
	if (h)
		tl = -1.f;
	return true;
}

/* the walk's child decision, branch-free on the scalar unit (the compiler's version of the
 * same logic spends ~2x the SALU instructions, and the shared scalar unit is what the packet
 * walk saturates first).  Near child first for the packet's direction octant (order bit
 * `oct` of the node's order mask; any order is correct).  Returns the near child if its box
 * is hit by any live ray, else the far child if hit, else RTX_NONE (pop); when both are hit
 * the far child is pushed: lane sp of the VGPR stack <- far, sp += 1.  A miss writes NONE
 * into lane sp, above the stack top. */
#define RTX_NODE_STEP_ASM(OCTC)                                                                               \
	asm volatile("s_bitcmp1_b32 %[ord], %[oct]\n\t"                                                        \
		     "s_cselect_b32 %[rn], %[r0], %[r1]\n\t"                                                   \
		     "s_cselect_b32 %[rf], %[r1], %[r0]\n\t"                                                   \
		     "s_cselect_b64 %[bn], %[b0], %[b1]\n\t"                                                   \
		     "s_cselect_b64 %[bf], %[b1], %[b0]\n\t"                                                   \
		     "s_cmp_lg_u64 %[bf], 0\n\t"                                                               \
		     "s_cselect_b32 %[rf], %[rf], -1\n\t"                                                      \
		     "s_cmp_lg_u64 %[bn], 0\n\t"                                                               \
		     "s_cselect_b32 %[next], %[rn], %[rf]\n\t"                                                 \
		     "s_cselect_b32 %[push], %[rf], -1\n\t"                                                    \
		     "v_mov_b32 %[t], %[push]\n\t"                                                             \
		     "v_cmp_eq_u32 vcc, %[sp], %[lane]\n\t"                                                    \
		     "v_cndmask_b32 %[stk], %[stk], %[t], vcc\n\t"                                             \
		     "s_cmp_lg_u32 %[push], -1\n\t"                                                            \
		     "s_addc_u32 %[sp], %[sp], 0"                                                              \
		     : [next] "=&s"(next), [push] "=&s"(push), [rn] "=&s"(rn), [rf] "=&s"(rf), [bn] "=&s"(bn), \
		       [bf] "=&s"(bf), [t] "=&v"(t), [sp] "+s"(sp), [stk] "+v"(stk)                            \
		     : [b0] "s"(b0), [b1] "s"(b1), [r0] "s"(r0), [r1] "s"(r1), [ord] "s"(order), OCTC,         \
		       [lane] "v"(lane_id())                                                                   \
		     : "scc", "vcc")

template <int OCT>
__device__ __forceinline__ uint32_t node_step(u64 b0, u64 b1, uint32_t r0, uint32_t r1, uint32_t order, uint32_t oct,
					      uint32_t &sp, uint32_t &stk)
{
	uint32_t next, push, rn, rf, t;
	u64 bn, bf;
	if constexpr (OCT < 8) /* octant as an inline constant of s_bitcmp1_b32 */
		RTX_NODE_STEP_ASM([oct] "n"(OCT));
	else
		RTX_NODE_STEP_ASM([oct] "s"(oct));
	return next;
}

/* shadow_prim for a leaf of triangles only; tri_emit: some live ray aims at a triangle emitter
 * (else no triangle here can be the target light and the skip test drops out) */
template <bool COUNT>
__device__ __forceinline__ bool shadow_tri(const v16u &pr, const DMaterial *__restrict__ mats, f3 o, f3 d, float &tl,
					   bool tri_emit, uint32_t emit_obj, f3 &li, ShadowCount &sc)
{
	const uint32_t meta = pr[11];
	if (COUNT)
		sc.tris += popc64(ballot(tl >= 0.f));
	if (COUNT)
		sc.psteps++;
#if RTX_SH_MASK
	u64 hm = any_tri_mask(mk3(__uint_as_float(pr[0]), __uint_as_float(pr[1]), __uint_as_float(pr[2])),
			      mk3(__uint_as_float(pr[4]), __uint_as_float(pr[5]), __uint_as_float(pr[6])),
			      mk3(__uint_as_float(pr[8]), __uint_as_float(pr[9]), __uint_as_float(pr[10])), o, d,
			      __uint_as_float(pr[3]), tl);
	if (tri_emit)
		hm &= ballot(pr[7] != emit_obj);
	if (!hm)
		return false;
	if (meta & RTX_META_TRANSPARENT) {
		const auto *m = cptr(mats) + (meta & RTX_META_MAT);
		li = mk3(msel(hm, li.x, li.x * m->kt[0]), msel(hm, li.y, li.y * m->kt[1]), msel(hm, li.z, li.z * m->kt[2]));
		return false;
	}
	tl = msel(hm, tl, -1.f);
	return true;
#else
	bool h = any_tri(mk3(__uint_as_float(pr[0]), __uint_as_float(pr[1]), __uint_as_float(pr[2])),
			 mk3(__uint_as_float(pr[4]), __uint_as_float(pr[5]), __uint_as_float(pr[6])),
			 mk3(__uint_as_float(pr[8]), __uint_as_float(pr[9]), __uint_as_float(pr[10])), o, d,
			 __uint_as_float(pr[3]), tl);
	if (tri_emit)
		h = h & (pr[7] != emit_obj);
	if (!ballot(h))
		return false;
	if (meta & RTX_META_TRANSPARENT) {
		const auto *m = cptr(mats) + (meta & RTX_META_MAT);
		const f3 kt = mk3(m->kt[0], m->kt[1], m->kt[2]);
		if (h)
			li = mul3v(li, kt);
		return false;
	}
	if (h)
		tl = -1.f;
	return true;
#endif
}

/* is_light_blocked for one packet of shadow rays (accel.c:317-387): the 64 rays walk the BVH
 * together.  Node and primitive records are wave-uniform (one 64-byte s_load_dwordx16 each),
 * each lane tests its own ray, the ballots pick the children.  A lane's liveness is its
 * segment end tl (< 0: inactive or blocked), so no lane masks are carried; control stays on
 * a few scalar registers: the ref (record byte offset | leaf bits), the stack depth, and the
 * stack itself, one ref per lane of a VGPR (depth <= 63, checked at upload). */
template <bool COUNT, int OCT>
__device__ __forceinline__ void shadow_walk(const char *__restrict__ recs, const DMaterial *__restrict__ mats,
					    uint32_t root_ref, f3 o, f3 d, f3 inv, float &tl, uint32_t emit_u,
					    uint32_t emit_obj, bool tri_emit, uint32_t lead_oct, f3 &li, ShadowCount &sc)
{
	const f3 oi = mul3v(o, inv);
	const uint32_t oct = OCT < 8 ? (uint32_t)OCT : lead_oct;
	uint32_t ref = root_ref, sp = 0, stk = 0, pf0 = 0, pf1 = 0;
	if (COUNT)
		count_need(sc, ballot(tl >= 0.f), root_ref);
	for (;;) {
		const v16u rec = rec_load(recs, ref & RTX_REF_OFF);
		if (RTX_SH_PF)
			consume(pf0, pf1, rec[15]);
		uint32_t next = RTX_NONE; /* RTX_NONE: pop */
		if (!(ref & RTX_REF_LEAF)) {
			if (RTX_SH_PF) {
				pf0 = touch(recs, rec[12] & RTX_REF_OFF);
				pf1 = touch(recs, rec[13] & RTX_REF_OFF);
			}
			if (COUNT) {
				sc.nodes += popc64(ballot(tl >= 0.f));
				sc.steps++;
			}
			const u64 b0 = ballot(box_hit<OCT>(rec, 0, oi, inv, tl));
			const u64 b1 = ballot(box_hit<OCT>(rec, 6, oi, inv, tl));
			if (COUNT) {
				count_need(sc, b0, rec[12]);
				count_need(sc, b1, rec[13]);
			}
			next = node_step<OCT>(b0, b1, rec[12], rec[13], rec[14], oct, sp, stk);
		} else {
			const uint32_t off = ref & RTX_REF_OFF, cnt = (ref & RTX_REF_CNT) + 1;
			if (RTX_SH_PF) { /* the leaf's second primitive and the stack top (next pop) */
				pf0 = touch(recs, off + (cnt > 1 ? (uint32_t)sizeof(DNode) : 0u));
				pf1 = touch(recs, sp ? readlane(stk, sp - 1) & RTX_REF_OFF : off);
			}
			bool blk;
			if (ref & RTX_REF_SPH) {
				blk = shadow_prim<COUNT>(rec, mats, o, d, tl, emit_u, emit_obj, li, sc);
				for (uint32_t k = 1; k < cnt; k++)
					blk |= shadow_prim<COUNT>(rec_load(recs, off + k * (uint32_t)sizeof(DNode)), mats, o, d, tl,
								 emit_u, emit_obj, li, sc);
			} else {
				blk = shadow_tri<COUNT>(rec, mats, o, d, tl, tri_emit, emit_obj, li, sc);
				for (uint32_t k = 1; k < cnt; k++)
					blk |= shadow_tri<COUNT>(rec_load(recs, off + k * (uint32_t)sizeof(DNode)), mats, o, d, tl,
								tri_emit, emit_obj, li, sc);
			}
			if (blk && !ballot(tl >= 0.f))
				sp = 0; /* every ray of the packet is blocked: end the walk */
		}
		if (next == RTX_NONE) {
			if (sp == 0)
				break;
			next = readlane(stk, --sp);
		}
		ref = next;
	}
	if (RTX_SH_PF)
		drain(pf0, pf1);
}

/* ------------------------------------------------------------------------ */
/* ray-by-ray any-hit walk over the threaded quantised BVH (DQNode)         */
/* ------------------------------------------------------------------------ */
/* Measured on the benchmark frame (count mode): a 64-ray packet fetched 58 node records and
 * tested 27.6 primitives per ray, while each ray's own boxes cover only 7.6 inner nodes and
 * 2.2 primitives - deep in the tree the rays of one shade point part ways, and the packet
 * drags every ray through the union of their paths.  Here each lane walks alone: its node
 * index is its whole state (any-hit needs no order, so skip links replace the stack), a node
 * is one 16-byte vector load (quantised box + link), and lanes at different nodes cost only
 * their own steps.  The wave's cost is its longest ray, not the union of its rays.  With
 * per-lane loads the vector L1's tag rate is the scarce resource, hence one load per node. */
/* per-lane loads through the global address space (global_load, not flat_load: the pointers
 * come from LDS and the compiler cannot prove where they point) */
template <typename T> __device__ __forceinline__ const __attribute__((address_space(1))) T *gptr(const T *p)
{
	return (const __attribute__((address_space(1))) T *)p;
}
typedef float f4v __attribute__((ext_vector_type(4)));
/* 16-byte global load at byte offset off of p */
__device__ __forceinline__ float4 ldg4(const void *p, uint32_t off)
{
	const f4v v = *(const __attribute__((address_space(1))) f4v *)((const char *)p + off);
	return make_float4(v.x, v.y, v.z, v.w);
}

/* the slab test against a DQNode box, in the quantisation frame: the ray is transformed once
 * per walk (o' = (o - qo) * qs, inv' = inv / qs, oi = o' * inv'), so t = q * inv' - oi is the
 * world ray parameter and the test is box_hit's, with 16-bit integers for the planes (each
 * converted by one SDWA v_cvt_f32_u32 of its half-word).  The boxes are widened by a full
 * step on both sides, far more than the rounding of the transform. */
template <int OCT>
__device__ __forceinline__ bool box_hit_q(uint4 n, f3 oi, f3 inv, float tlim)
{
	const float tx0 = fmaf((float)(n.x & 0xFFFFu), inv.x, -oi.x), tx1 = fmaf((float)(n.x >> 16), inv.x, -oi.x);
	const float ty0 = fmaf((float)(n.y & 0xFFFFu), inv.y, -oi.y), ty1 = fmaf((float)(n.y >> 16), inv.y, -oi.y);
	const float tz0 = fmaf((float)(n.z & 0xFFFFu), inv.z, -oi.z), tz1 = fmaf((float)(n.z >> 16), inv.z, -oi.z);
	if (OCT == 8) {
		const float tn = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fmaxf(fminf(tz0, tz1), 0.f));
		const float tf = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fminf(fmaxf(tz0, tz1), tlim));
		return tn <= tf;
	}
	const float nx = (OCT & 1) ? tx0 : tx1, fx = (OCT & 1) ? tx1 : tx0;
	const float ny = (OCT & 2) ? ty0 : ty1, fy = (OCT & 2) ? ty1 : ty0;
	const float nz = (OCT & 4) ? tz0 : tz1, fz = (OCT & 4) ? tz1 : tz0;
	const float tn = fmaxf(fmaxf(nx, ny), fmaxf(nz, 0.f));
	float tf = fminf(fminf(fx, fy), fz);
	asm("v_min_f32 %0, %0, %1" : "+v"(tf) : "v"(tlim));
	return tn <= tf;
}

typedef uint32_t u4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ldg4u(const void *p)
{
	const u4v v = *(const __attribute__((address_space(1))) u4v *)p;
	return make_uint4(v.x, v.y, v.z, v.w);
}

/* one primitive record (a, b, c = its first 48 bytes) against this lane's shadow ray
 * (accel.c:362-373): the target emitter skipped; transparent hit -> li *= kt; opaque hit ->
 * true (blocked) */
template <bool COUNT>
__device__ __forceinline__ bool shadow_prim_ray(float4 a, float4 b, float4 c, const DMaterial *__restrict__ mats, f3 o,
						 f3 d, float tl, uint32_t emit_obj, f3 &li, uint32_t &ntri, uint32_t &nsph)
{
	const uint32_t meta = __float_as_uint(c.w), obj = __float_as_uint(b.w);
	if (obj == emit_obj)
		return false;
	bool h;
	if ((meta >> 24) == RTX_SPHERE) {
		if (COUNT)
			nsph++;
		float t = 0.f;
		h = hit_sphere(mk3(a.x, a.y, a.z), b.x, o, d, a.w, t) && t < tl;
	} else {
		if (COUNT)
			ntri++;
		h = any_tri(mk3(a.x, a.y, a.z), mk3(b.x, b.y, b.z), mk3(c.x, c.y, c.z), o, d, a.w, tl);
	}
	if (!h)
		return false;
	if (meta & RTX_META_TRANSPARENT) {
		const auto *m = gptr(mats) + (meta & RTX_META_MAT);
		li = mul3v(li, mk3(m->kt[0], m->kt[1], m->kt[2]));
		return false;
	}
	return true;
}

/* the quantised threaded BVH and its frame (rtx_device.h DQNode) */
struct QBvh {
	const DQNode *q;
	uint32_t n;
	f3 qo, qs;
	const uint4 *top;     /* the workgroup's LDS copy of the top records */
	const uint32_t *tend; /* ... and of the cut records' range ends */
	uint32_t nt;
};

/* LDS reads through generic pointers that point into LDS */
__device__ __forceinline__ uint4 lds4u(const void *p)
{
	const u4v v = *(const __attribute__((address_space(3))) u4v *)p;
	return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint32_t lds1u(const uint32_t *p)
{
	return *(const __attribute__((address_space(3))) uint32_t *)p;
}

/* The walk starts in the workgroup's LDS copy of the tree's top levels (DScene.top): a cut
 * record whose box is hit hands the lane to the DQNode array for the index range of its
 * children's subtrees, and the lane returns to the top copy at the next top record when the
 * range ends.  The nodes visited, and their order, are the plain threaded walk's.  Every
 * global node load costs a vector-L1 lookup per lane, the resource the walk saturates; the
 * top levels, which nearly every ray tests, come from LDS instead. */
template <bool COUNT, int OCT>
__device__ __forceinline__ void shadow_walk_ray(const QBvh &Q, const char *__restrict__ recs,
						const DMaterial *__restrict__ mats, f3 o, f3 d, f3 inv, float &tl,
						uint32_t emit_obj, f3 &li, ShadowCount &sc)
{
	const f3 invq = mk3(inv.x / Q.qs.x, inv.y / Q.qs.y, inv.z / Q.qs.z);
	const f3 oq = mk3((o.x - Q.qo.x) * Q.qs.x, (o.y - Q.qo.y) * Q.qs.y, (o.z - Q.qo.z) * Q.qs.z);
	const f3 oi = mul3v(oq, invq);
	const uint32_t nt = Q.nt;
	uint32_t t = tl >= 0.f ? 0u : nt, g = 0, ge = 0;
	uint32_t nnode = 0, nglob = 0, ntri = 0, nsph = 0;
	while (t < nt || g < ge) {
		const bool ing = g < ge;
		uint4 nd;
		if (ing)
			nd = ldg4u(Q.q + g);
		else
			nd = lds4u(Q.top + t);
		if (COUNT) {
			nnode++;
			nglob += ing ? 1u : 0u;
		}
		const bool hit = box_hit_q<OCT>(nd, oi, invq, tl);
		const uint32_t L = nd.w;
		if (L & RTX_REF_LEAF) {
			if (ing)
				g++;
			else
				t++;
			if (hit) {
				const char *p = recs + (L & RTX_REF_OFF);
				const uint32_t cnt = (L & RTX_REF_CNT) + 1;
				for (uint32_t k = 0; k < cnt; k++) {
					const char *pr = p + k * (uint32_t)sizeof(DNode);
					if (shadow_prim_ray<COUNT>(ldg4(pr, 0), ldg4(pr, 16), ldg4(pr, 32), mats, o, d, tl, emit_obj,
								   li, ntri, nsph)) {
						tl = -1.f;
						t = nt;
						ge = 0;
						break;
					}
				}
			}
		} else if (ing) {
			g = hit ? g + 1 : L >> 6;
		} else if (L & RTX_QTOP_CUT) {
			if (hit) {
				g = L >> 6;
				ge = lds1u(Q.tend + t);
			}
			t++;
		} else {
			t = hit ? t + 1 : L >> 6;
		}
	}
	if (COUNT) {
		uint32_t a = nnode, b = ntri, c = nsph, m = nnode, gq = nglob;
#pragma unroll
		for (int s = 32; s > 0; s >>= 1) {
			gq += __shfl_xor(gq, s, WAVE);
			a += __shfl_xor(a, s, WAVE);
			b += __shfl_xor(b, s, WAVE);
			c += __shfl_xor(c, s, WAVE);
			m = max(m, (uint32_t)__shfl_xor(m, s, WAVE));
		}
		sc.nodes += uni(a);
		sc.tris += uni(b);
		sc.sph += uni(c);
		sc.rnodes += uni(gq); /* box tests whose node came from the DQNode array, not the LDS top */
		sc.steps += uni(m); /* the wave's node steps: its longest ray */
		sc.psteps++;        /* walks */
	}
}


/* |v| of the light vector: v_sqrt_f32 (1 ulp) instead of the correctly rounded sqrt sequence
 * when RTX_SH_FASTSQRT; shadow-ray plane tests then also take t from v_rcp_f32. */
#ifndef RTX_SH_FASTSQRT
#define RTX_SH_FASTSQRT 0
#endif
__device__ __forceinline__ float sh_mag(f3 v)
{
	return RTX_SH_FASTSQRT ? __builtin_amdgcn_sqrtf(magsqr3(v)) : mag3(v);
}
__device__ __forceinline__ bool sh_hit_plane(f3 n, float dd, f3 o, f3 d, float eps, float &t)
{
	if (!RTX_SH_FASTSQRT)
		return hit_plane(n, dd, o, d, eps, t);
	const float a = dot3(n, d);
	if (fabsf(a) < eps)
		return false;
	t = (dd - dot3(n, o)) * __builtin_amdgcn_rcpf(a);
	return t > eps;
}

/* planes first (unbound_objects_is_light_blocked, object.c:183-197), then the BVH walk,
 * specialised on the packet's direction octant when all live rays share it.  Returns the
 * lane's blocked flag; li carries the transmittance product. */
template <bool COUNT>
__device__ __forceinline__ bool shadow_packet(const QBvh &Q, const char *__restrict__ recs,
					      const DMaterial *__restrict__ mats, const DPlane *__restrict__ planes,
					      uint32_t num_planes, uint32_t root_ref,
					      bool act, f3 o, f3 d, float dist, uint32_t emit_obj, bool emit_is_tri, f3 &li,
					      ShadowCount &sc)
{
	float tl = act ? dist : -1.f;
	for (uint32_t i = 0; i < num_planes; i++) { /* plane records are wave-uniform: s_load */
		const auto *pl = cptr(planes) + i;
		const auto *m = cptr(mats) + pl->mat;
		float t;
		const bool h = sh_hit_plane(mk3(pl->n[0], pl->n[1], pl->n[2]), pl->d, o, d, pl->eps, t) && t < dist && tl >= 0.f;
		if (m->flags & RTX_MF_TRANSPARENT) {
			if (h)
				li = mul3v(li, mk3(m->kt[0], m->kt[1], m->kt[2]));
		} else if (h) {
			tl = -1.f;
		}
	}
	if (COUNT)
		sc.pln += (u64)popc64(ballot(act)) * num_planes;
	const bool alive = tl >= 0.f;
	const u64 live = ballot(alive);
	if (!live || root_ref == RTX_EMPTY_REF)
		return act && !alive;
	const f3 inv = safe_inv_fast(d); /* boxes are padded 2e-6 relative: a 1-ulp 1/d keeps the test conservative */
	const uint32_t oct = ((~__float_as_uint(inv.x)) >> 31) | (((~__float_as_uint(inv.y)) >> 31) << 1) |
			     (((~__float_as_uint(inv.z)) >> 31) << 2);
	const uint32_t lead_lane = (uint32_t)__ffsll((long long)live) - 1;
	const uint32_t lead = readlane(oct, lead_lane), lead_emit = readlane(emit_obj, lead_lane);
	const uint32_t emit_u = ballot(alive & (emit_obj != lead_emit)) ? RTX_NONE : lead_emit;
	const bool tri_emit = ballot(alive & emit_is_tri) != 0;
	const uint32_t sel = (!RTX_SH_OCT || ballot(alive & (oct != lead))) ? 8u : lead;
	switch (sel) {
#if RTX_SH_RAY
		(void)emit_u;
		(void)tri_emit;
#define RTX_WALK(K)                                                                                                 \
	case K:                                                                                                           \
		shadow_walk_ray<COUNT, K>(Q, recs, mats, o, d, inv, tl, emit_obj, li, sc);                              \
		break;
#if RTX_SH_OCT
	RTX_WALK(0) RTX_WALK(1) RTX_WALK(2) RTX_WALK(3) RTX_WALK(4) RTX_WALK(5) RTX_WALK(6) RTX_WALK(7)
#endif
	default:
		shadow_walk_ray<COUNT, 8>(Q, recs, mats, o, d, inv, tl, emit_obj, li, sc);
		break;
#else
#define RTX_WALK(K)                                                                                                   \
	case K:                                                                                                           \
		shadow_walk<COUNT, K>(recs, mats, root_ref, o, d, inv, tl, emit_u, emit_obj, tri_emit, K, li, sc);           \
		break;
#if RTX_SH_OCT
	RTX_WALK(0) RTX_WALK(1) RTX_WALK(2) RTX_WALK(3) RTX_WALK(4) RTX_WALK(5) RTX_WALK(6) RTX_WALK(7)
#endif
	default:
		shadow_walk<COUNT, 8>(recs, mats, root_ref, o, d, inv, tl, emit_u, emit_obj, tri_emit, lead, li, sc);
		break;
#endif
#undef RTX_WALK
	}
	return act && tl < 0.f;
}

/* k_shadow arguments.  Lane 0 copies them to LDS; the packet loop re-reads them from there
 * after each walk (behind a compiler memory barrier), so none stays live in registers across
 * the traversal, which needs every SGPR it can get at 8 waves/SIMD. */
struct KShadow {
	const DNode *recs; /* BVH nodes, then primitives from record nnodes */
	const DQNode *qnodes; /* threaded quantised BVH (ray-by-ray walk) */
	float qo[3], qs[3];
	const uint32_t *top;  /* its top levels (rtx_device.h RTX_QTOP_CUT), copied to LDS per workgroup */
	uint32_t ntop;
	const DMaterial *mats;
	const DPlane *planes;
	const DEmitter *emitters;
	const float4 *sp;
	const uint32_t *perm; /* shade points in processing order (Morton-sorted), or null */
	float4 *contrib;
	unsigned long long *ctr;
	uint32_t nnodes, root_ref, num_planes, num_emitters, nq;
	uint32_t n_sp, per_wave, slot_b, slot_lg;
	int32_t rng, attenuation, reflection;
	float att_offset;
};

__device__ __forceinline__ void reread_barrier() { asm volatile("" ::: "memory"); }

/* a pointer read from LDS, made wave-uniform (SGPRs) so accesses through it stay scalar */
template <typename T> __device__ __forceinline__ T *unip(T *p)
{
	const uint64_t v = (uint64_t)p;
	return (T *)(((uint64_t)uni((uint32_t)(v >> 32)) << 32) | uni((uint32_t)v));
}

/* light_point (object.c:293-304) for the shadow kernel: on a sphere emitter the inclination and
 * azimuth are u * 2pi, so their sines and cosines come straight from the hardware's
 * revolution-scaled v_sin_f32 / v_cos_f32 instead of OCML's range-reduced sinf / cosf
 * (|error| ~1e-6 of the radius, far inside the frame tolerance; the KAT suite keeps checking the
 * exact light_point).  RTX_SH_FASTTRIG=0 restores the exact version here too. */
#ifndef RTX_SH_FASTTRIG
#define RTX_SH_FASTTRIG 1
#endif
/* 1/x in the shadow kernel's light sampling and attenuation: v_rcp_f32 (1 ulp) instead of the
 * IEEE division sequence when RTX_SH_FASTDIV (the shadow ray direction and the attenuated
 * intensity move by <= 1 ulp; the closest-hit path keeps IEEE division). */
#ifndef RTX_SH_FASTDIV
#define RTX_SH_FASTDIV 1
#endif
__device__ __forceinline__ float sh_rcp(float x) { return RTX_SH_FASTDIV ? __builtin_amdgcn_rcpf(x) : 1.f / x; }

__device__ __forceinline__ f3 light_point_sh(const DEmitter &e, f3 p, float u1, float u2)
{
	if (RTX_SH_FASTTRIG && e.type == RTX_SPHERE) {
		const f3 c = ld3(e.p0);
		const f3 nrm = sub3(c, p);
		const float si = __builtin_amdgcn_sinf(u1), ci = __builtin_amdgcn_cosf(u1);
		const float sa = __builtin_amdgcn_sinf(u2), ca = __builtin_amdgcn_cosf(u2);
		f3 ld = mk3(e.radius * ca * si, e.radius * sa * si, e.radius * ci);
		if (dot3(nrm, ld) != 0.f)
			ld = mul3s(ld, -1.f);
		return add3(c, ld);
	}
	return light_point(e, p, u1, u2);
}

/* direct-lighting terms of one unblocked light sample (render.c:199-228), read after the walk */
__device__ __forceinline__ f3 shade_light(const KShadow &ks, const float4 *rec, f3 ldir, f3 li, float ldist, float dsq)
{
	const float4 q1 = rec[1], q2 = rec[2], q3 = rec[3];
	const f3 n = mk3(q1.x, q1.y, q1.z), dir = mk3(q2.x, q2.y, q2.z);
	const float a = dot3(ldir, n);
	const int32_t att = (int32_t)uni((uint32_t)ks.attenuation);
	if (att == RTX_ATT_LIN)
		li = mul3s(li, sh_rcp(ks.att_offset + ldist));
	else if (att == RTX_ATT_SQR)
		li = mul3s(li, sh_rcp(ks.att_offset + dsq));
	const DMaterial &m = unip(ks.mats)[__float_as_uint(q3.w)];
	const f3 diff = mul3s(mul3v(mk3(q3.x, q3.y, q3.z), li), fmaxf(0.f, a));
	float sm;
	if ((int32_t)uni((uint32_t)ks.reflection) == RTX_BLINN) {
		sm = -dot3(n, norm3(add3(mul3s(ldir, -1.f), dir)));
	} else {
		sm = -dot3(sub3(mul3s(n, 2.f * a), ldir), dir);
	}
	const f3 spec = mul3s(mul3v(ld3(m.ks), li), fmaxf(0.f, powf(sm, m.shininess)));
	return add3(diff, spec);
}

/* one light sample per lane of the shade point `rec` (render.c:170-229): the light point of
 * sample idx (emitters in scene order, the hit object skipped), its shadow ray through the
 * packet walk, attenuation and Phong / Blinn.  Argument-block fields are read from LDS behind
 * reread barriers so none stays in registers across the walk. */
template <bool COUNT>
__device__ __forceinline__ f3 light_sample(const KShadow &ks, const float4 *rec, uint32_t idx, bool act,
					   ShadowCount &sc, const uint4 *top_q, const uint32_t *top_e)
{
	reread_barrier();
	const float4 q0 = rec[0], q4 = rec[4];
	const f3 p = mk3(q0.x, q0.y, q0.z);
	const uint32_t obj = __float_as_uint(q4.x);
	const DEmitter *emitters = unip(ks.emitters);
	const uint32_t num_emitters = uni(ks.num_emitters);
	uint32_t j = idx;
	uint32_t e = 0;
	for (; e < num_emitters; e++) {
		const uint32_t eo = emitters[e].obj, enl = emitters[e].num_lights;
		if (eo == obj)
			continue;
		if (j < enl)
			break;
		j -= enl;
	}
	if (e >= num_emitters)
		e = 0;
	const DEmitter &E = emitters[e];
	float u1 = 0.5f, u2 = 0.5f;
	if (uni(ks.rng) != RTX_RNG_CONST) /* the key already carries the seed (rtx_key_pixel) */
		rtx_draw2(key_of(__float_as_uint(q4.y), __float_as_uint(q4.z)), e, j, &u1, &u2);
#ifdef RTX_SH_STRAT /* measurement only: Morton-stratified light samples (packet coherence bound) */
	{
		const uint32_t m = j * 1024u / emitters[e].num_lights;
		uint32_t x = 0, y = 0;
		for (int b = 0; b < 5; b++) {
			x |= ((m >> (2 * b)) & 1u) << b;
			y |= ((m >> (2 * b + 1)) & 1u) << b;
		}
		u1 = (x + u1) * (1.f / 32.f);
		u2 = (y + u2) * (1.f / 32.f);
	}
#endif
	const f3 lp = light_point_sh(E, p, u1, u2);
	const f3 dv = sub3(lp, p);
	const float ldist = sh_mag(dv);
	const float dsq = magsqr3(dv);
	const f3 ldir = mul3s(dv, sh_rcp(ldist));
	f3 li = ld3(E.li);
	QBvh Q;
	Q.q = unip(ks.qnodes);
	Q.n = uni(ks.nq);
	Q.qo = mk3(ks.qo[0], ks.qo[1], ks.qo[2]);
	Q.qs = mk3(ks.qs[0], ks.qs[1], ks.qs[2]);
	Q.top = top_q;
	Q.tend = top_e;
	Q.nt = uni(ks.ntop);
	const bool blocked = shadow_packet<COUNT>(Q, (const char *)unip(ks.recs), unip(ks.mats), unip(ks.planes),
						  uni(ks.num_planes), RTX_DEBUG_NOWALK ? RTX_EMPTY_REF : uni(ks.root_ref),
						  act, p, ldir, ldist, E.obj, E.type == RTX_TRIANGLE, li, sc);
	reread_barrier();
	f3 contribution = mk3(0.f, 0.f, 0.f);
	if (act && !blocked)
		contribution = shade_light(ks, rec, ldir, li, ldist, dsq);
	return contribution;
}

/* All nl light samples of one shade point (single-point mode, >= 64 lights) with lane refill.
 * A 64-ray packet runs until its longest ray ends, so most lanes idle through the tail of
 * every packet.  Here a lane whose ray has ended takes the point's next unassigned sample
 * (render.c:170-229 per sample, as light_sample) once at least RTX_SH_REFILL lanes are idle
 * or none is walking, so the wave keeps walking until the point's samples run out.  Which
 * lane takes which sample depends only on the walk lengths, i.e. on the point: the per-lane
 * sums, and the point's result, stay deterministic and independent of scheduling. */
#ifndef RTX_SH_STREAM
#define RTX_SH_STREAM 0 /* > 0: stream single-point samples across points, batches of this many points */
#endif
#ifndef RTX_SH_REFILL
#define RTX_SH_REFILL 0
#endif
template <bool COUNT>
__device__ __forceinline__ f3 point_refill(const KShadow &ks, const float4 *rec, uint32_t nl, ShadowCount &sc,
					   const uint4 *top_q, const uint32_t *top_e)
{
	reread_barrier();
	const float4 q0 = rec[0], q4 = rec[4];
	const f3 p = mk3(q0.x, q0.y, q0.z);
	const uint32_t obj = __float_as_uint(q4.x);
	const uint32_t key_a = __float_as_uint(q4.y), key_b = __float_as_uint(q4.z);
	const uint32_t nt = uni(ks.ntop);
	const bool have_tree = uni(ks.root_ref) != RTX_EMPTY_REF && !RTX_DEBUG_NOWALK;
	f3 acc = mk3(0.f, 0.f, 0.f);
	f3 d = mk3(0.f, 0.f, 0.f), invq = d, oi = d, li = d;
	float tl = -1.f, ldist = 1.f, dsq = 1.f;
	uint32_t emit_obj = RTX_NONE, t = nt, g = 0, ge = 0;
	bool has = false; /* the lane holds a sample whose terms are not yet in acc */
	uint32_t next = 0; /* wave-uniform: the point's next unassigned sample */
	uint32_t nnode = 0, ntri = 0, nsph = 0, nsteps = 0;
	for (;;) {
		const bool walking = t < nt || g < ge;
		const u64 wl = ballot(walking);
		const uint32_t idle = (uint32_t)popc64(~wl);
		if (!wl || (idle >= RTX_SH_REFILL && next < nl)) {
			reread_barrier();
			/* finish this lane's ended sample, then take a new one */
			if (has && !walking) {
				if (tl >= 0.f)
					acc = add3(acc, shade_light(ks, rec, d, li, ldist, dsq));
				has = false;
			}
			const u64 want = ballot(!walking);
			const uint32_t idx = next + (uint32_t)__builtin_amdgcn_mbcnt_hi(
							   (uint32_t)(want >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)want, 0u));
			next = min(nl, next + (uint32_t)popc64(want));
			if (COUNT)
				sc.pln += (u64)popc64(ballot(!walking && idx < nl)) * uni(ks.num_planes);
			if (!walking && idx < nl) {
				const DEmitter *emitters = unip(ks.emitters);
				const uint32_t num_emitters = uni(ks.num_emitters);
				uint32_t j = idx, e = 0;
				for (; e < num_emitters; e++) {
					const uint32_t eo = emitters[e].obj, enl = emitters[e].num_lights;
					if (eo == obj)
						continue;
					if (j < enl)
						break;
					j -= enl;
				}
				if (e >= num_emitters)
					e = 0;
				const DEmitter &E = emitters[e];
				float u1 = 0.5f, u2 = 0.5f;
				if (uni(ks.rng) != RTX_RNG_CONST)
					rtx_draw2(key_of(key_a, key_b), e, j, &u1, &u2);
				const f3 lp = light_point_sh(E, p, u1, u2);
				const f3 dv = sub3(lp, p);
				ldist = sh_mag(dv);
				dsq = magsqr3(dv);
				d = mul3s(dv, sh_rcp(ldist));
				li = ld3(E.li);
				emit_obj = E.obj;
				tl = ldist;
				/* planes first (unbound_objects_is_light_blocked, object.c:183-197) */
				const DPlane *planes = unip(ks.planes);
				const uint32_t num_planes = uni(ks.num_planes);
				for (uint32_t i = 0; i < num_planes; i++) {
					const auto *pl = cptr(planes) + i;
					const auto *m = cptr(unip(ks.mats)) + pl->mat;
					float tp;
					const bool h = sh_hit_plane(mk3(pl->n[0], pl->n[1], pl->n[2]), pl->d, p, d, pl->eps, tp) &&
						       tp < ldist && tl >= 0.f;
					if (m->flags & RTX_MF_TRANSPARENT) {
						if (h)
							li = mul3v(li, mk3(m->kt[0], m->kt[1], m->kt[2]));
					} else if (h) {
						tl = -1.f;
					}
				}
				const f3 inv = safe_inv_fast(d);
				invq = mk3(inv.x / ks.qs[0], inv.y / ks.qs[1], inv.z / ks.qs[2]);
				const f3 oq = mk3((p.x - ks.qo[0]) * ks.qs[0], (p.y - ks.qo[1]) * ks.qs[1], (p.z - ks.qo[2]) * ks.qs[2]);
				oi = mul3v(oq, invq);
				t = (tl >= 0.f && have_tree) ? 0u : nt;
				g = 0;
				ge = 0;
				has = true;
			}
			if (!ballot(has))
				break;
			continue;
		}
		if (COUNT)
			nsteps++;
		if (walking) {
			const bool ing = g < ge;
			uint4 nd;
			if (ing)
				nd = ldg4u(unip(ks.qnodes) + g);
			else
				nd = lds4u(top_q + t);
			if (COUNT)
				nnode++;
			const bool hit = box_hit_q<8>(nd, oi, invq, tl);
			const uint32_t L = nd.w;
			if (L & RTX_REF_LEAF) {
				if (ing)
					g++;
				else
					t++;
				if (hit) {
					const char *pr = (const char *)unip(ks.recs) + (L & RTX_REF_OFF);
					const uint32_t cnt = (L & RTX_REF_CNT) + 1;
					for (uint32_t k = 0; k < cnt; k++, pr += sizeof(DNode)) {
						if (shadow_prim_ray<COUNT>(ldg4(pr, 0), ldg4(pr, 16), ldg4(pr, 32), unip(ks.mats), p, d, tl,
									   emit_obj, li, ntri, nsph)) {
							tl = -1.f;
							t = nt;
							ge = 0;
							break;
						}
					}
				}
			} else if (ing) {
				g = hit ? g + 1 : L >> 6;
			} else if (L & RTX_QTOP_CUT) {
				if (hit) {
					g = L >> 6;
					ge = lds1u(top_e + t);
				}
				t++;
			} else {
				t = hit ? t + 1 : L >> 6;
			}
		}
	}
	if (COUNT) {
		uint32_t a = nnode, b = ntri, c = nsph;
#pragma unroll
		for (int s = 32; s > 0; s >>= 1) {
			a += __shfl_xor(a, s, WAVE);
			b += __shfl_xor(b, s, WAVE);
			c += __shfl_xor(c, s, WAVE);
		}
		sc.nodes += uni(a);
		sc.tris += uni(b);
		sc.sph += uni(c);
		sc.steps += uni(nsteps);
		sc.psteps++;
	}
	return acc;
}

/* ------------------------------------------------------------------------ */
/* single-origin packets: R shadow rays per lane                            */
/* ------------------------------------------------------------------------ */
/* In single-point mode (>= 64 lights) every ray of a packet starts at the same shade point P.
 * Everything a node or a triangle contributes to a test that depends on P alone is then
 * wave-uniform: the box planes relative to P, and for Moller-Trumbore s = P - v0, q = s x e1,
 * e2 . q and e2 x s.  Each lane carries R rays (64*R per walk), so one record load, one set of
 * P-relative terms and one scalar child decision serve R times as many rays as the one-ray
 * walk; the per-ray work left is a few products and compares. */

/* box test from P-relative planes: dn / df = near / far plane minus P per axis for octant OCT
 * (OCT == 8: lo / hi minus P, order decided per lane).  (plane - P) is exact to half an ulp
 * and the boxes are padded 2e-6 relative, so the test stays conservative like box_hit's. */
template <int OCT>
__device__ __forceinline__ bool box_hit_so(f3 dn, f3 df, f3 inv, float tlim)
{
	const float ax = dn.x * inv.x, bx = df.x * inv.x;
	const float ay = dn.y * inv.y, by = df.y * inv.y;
	const float az = dn.z * inv.z, bz = df.z * inv.z;
	if (OCT == 8) {
		const float tn = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fmaxf(fminf(az, bz), 0.f));
		const float tf = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fminf(fmaxf(az, bz), tlim));
		return tn <= tf;
	}
	const float tn = fmaxf(fmaxf(ax, ay), fmaxf(az, 0.f));
	float tf = fminf(fminf(bx, by), bz);
	asm("v_min_f32 %0, %0, %1" : "+v"(tf) : "v"(tlim));
	return tn <= tf;
}

/* the P-relative planes of the child box at rec[b..b+5] = lo.x, hi.x, lo.y, hi.y, lo.z, hi.z */
template <int OCT>
__device__ __forceinline__ void box_planes_so(const v16u &nd, const uint32_t b, f3 o, f3 &dn, f3 &df)
{
	const float lx = __uint_as_float(nd[b]) - o.x, hx = __uint_as_float(nd[b + 1]) - o.x;
	const float ly = __uint_as_float(nd[b + 2]) - o.y, hy = __uint_as_float(nd[b + 3]) - o.y;
	const float lz = __uint_as_float(nd[b + 4]) - o.z, hz = __uint_as_float(nd[b + 5]) - o.z;
	if (OCT == 8) {
		dn = mk3(lx, ly, lz);
		df = mk3(hx, hy, hz);
		return;
	}
	dn = mk3((OCT & 1) ? lx : hx, (OCT & 2) ? ly : hy, (OCT & 4) ? lz : hz);
	df = mk3((OCT & 1) ? hx : lx, (OCT & 2) ? hy : ly, (OCT & 4) ? hz : lz);
}

/* moller_trumbore (object.c:422-441) with a shared origin, by the triple-product identities
 *   a = e1.(d x e2) = d.(e2 x e1),  u a = s.(d x e2) = d.(e2 x s),  v a = d.q,  t a = e2.q
 * (s = P - v0, q = s x e1): the per-ray part is three dot products.  Same accept set as
 * any_tri (|a| >= eps, u, v >= 0, u + v <= 1, eps < t < tlim). */
struct TriSO {
	f3 ca, cu, q;
	float tq;
};
__device__ __forceinline__ TriSO tri_so(f3 v0, f3 e1, f3 e2, f3 o)
{
	const f3 s = sub3(o, v0);
	TriSO T;
	T.ca = cross3_fma(e2, e1);
	T.cu = cross3_fma(e2, s);
	T.q = cross3_fma(s, e1);
	T.tq = dot3_fma(e2, T.q);
	return T;
}
__device__ __forceinline__ u64 any_tri_so_mask(const TriSO &T, f3 d, float eps, float tlim)
{
	const float a = dot3_fma(d, T.ca);
	const float f = __builtin_amdgcn_rcpf(a);
	const float u = f * dot3_fma(d, T.cu);
	const float v = f * dot3_fma(d, T.q);
	const float t = f * T.tq;
	const float out = fmaxf(fmaxf(-u, -v), (u + v) - 1.f);
	return ballot(fabsf(a) >= eps) & ballot(out <= 0.f) & ballot(fminf(t - eps, tlim - t) > 0.f);
}

/* keeps the per-ray tests of one record in sequence: the scheduler would otherwise interleave
 * all R rays' temporaries and run out of registers (other waves supply the parallelism) */
#ifndef RTX_SO_SCHED
#define RTX_SO_SCHED 1
#endif
#define RTX_SO_SERIAL()                                                                                             \
	do {                                                                                                            \
		if (RTX_SO_SCHED)                                                                                           \
			__builtin_amdgcn_sched_barrier(0);                                                                      \
	} while (0)

/* the packet of R rays per lane walking the BVH (shadow_walk with shared-origin tests).
 * Per-ray state in registers is only what every test reads: direction, its reciprocal and the
 * segment end.  The transmittance product li lives in LDS ([component][ray][lane]) and is
 * touched only on a transparent hit; emit_lds[ray][lane] is the index of the emitter the ray
 * aims at, read only when the packet's rays aim at different emitters (emit_u == RTX_NONE)
 * or at a triangle emitter (tri_emit). */
template <bool COUNT, int OCT, int R>
__device__ __forceinline__ void shadow_walk_so(const char *__restrict__ recs, const DMaterial *__restrict__ mats,
					       const DEmitter *__restrict__ emitters, uint32_t root_ref, f3 o,
					       const f3 (&d)[R], const f3 (&inv)[R], float (&tl)[R], float *li_lds,
					       uint32_t emit_u, const uint8_t *emit_lds, bool tri_emit, uint32_t lead_oct,
					       ShadowCount &sc)
{
	const uint32_t oct = OCT < 8 ? (uint32_t)OCT : lead_oct;
	uint32_t ref = root_ref, sp = 0, stk = 0, pf0 = 0, pf1 = 0;
	for (;;) {
		const v16u rec = rec_load(recs, ref & RTX_REF_OFF);
		if (RTX_SH_PF)
			consume(pf0, pf1, rec[15]);
		uint32_t next = RTX_NONE; /* RTX_NONE: pop */
		if (!(ref & RTX_REF_LEAF)) {
			if (RTX_SH_PF) {
				pf0 = touch(recs, rec[12] & RTX_REF_OFF);
				pf1 = touch(recs, rec[13] & RTX_REF_OFF);
			}
			if (COUNT) {
#pragma unroll
				for (int r = 0; r < R; r++)
					sc.nodes += popc64(ballot(tl[r] >= 0.f));
				sc.steps++;
			}
			u64 b0 = 0, b1 = 0;
			{
				f3 dn, df;
				box_planes_so<OCT>(rec, 0, o, dn, df);
#pragma unroll
				for (int r = 0; r < R; r++) {
					b0 |= ballot(box_hit_so<OCT>(dn, df, inv[r], tl[r]));
					RTX_SO_SERIAL();
				}
			}
			{
				f3 dn, df;
				box_planes_so<OCT>(rec, 6, o, dn, df);
#pragma unroll
				for (int r = 0; r < R; r++) {
					b1 |= ballot(box_hit_so<OCT>(dn, df, inv[r], tl[r]));
					RTX_SO_SERIAL();
				}
			}
			next = node_step<OCT>(b0, b1, rec[12], rec[13], rec[14], oct, sp, stk);
		} else {
			const uint32_t off = ref & RTX_REF_OFF, cnt = (ref & RTX_REF_CNT) + 1;
			if (RTX_SH_PF) { /* the leaf's second primitive and the stack top (next pop) */
				pf0 = touch(recs, off + (cnt > 1 ? (uint32_t)sizeof(DNode) : 0u));
				pf1 = touch(recs, sp ? readlane(stk, sp - 1) & RTX_REF_OFF : off);
			}
			bool blk = false;
			for (uint32_t k = 0; k < (RTX_DEBUG_NOLEAF ? 0u : cnt); k++) {
				const v16u pr = k ? rec_load(recs, off + k * (uint32_t)sizeof(DNode)) : rec;
				const uint32_t meta = pr[11], obj = pr[7];
				if (obj == emit_u)
					continue;
				const f3 a = mk3(__uint_as_float(pr[0]), __uint_as_float(pr[1]), __uint_as_float(pr[2]));
				const float eps = __uint_as_float(pr[3]);
				const bool sphere = (meta >> 24) == RTX_SPHERE;
				u64 hm[R], any = 0;
				if (COUNT)
					sc.psteps++;
				if (sphere) {
#pragma unroll
					for (int r = 0; r < R; r++) {
						if (COUNT)
							sc.sph += popc64(ballot(tl[r] >= 0.f));
						float t = 0.f;
						hm[r] = ballot(hit_sphere(a, __uint_as_float(pr[4]), o, d[r], eps, t) & (t < tl[r]));
						RTX_SO_SERIAL();
					}
				} else {
					const TriSO T = tri_so(a, mk3(__uint_as_float(pr[4]), __uint_as_float(pr[5]), __uint_as_float(pr[6])),
							       mk3(__uint_as_float(pr[8]), __uint_as_float(pr[9]), __uint_as_float(pr[10])), o);
#pragma unroll
					for (int r = 0; r < R; r++) {
						if (COUNT)
							sc.tris += popc64(ballot(tl[r] >= 0.f));
						hm[r] = any_tri_so_mask(T, d[r], eps, tl[r]);
						RTX_SO_SERIAL();
					}
				}
				if (sphere ? emit_u == RTX_NONE : tri_emit) {
#pragma unroll
					for (int r = 0; r < R; r++)
						hm[r] &= ballot(emitters[emit_lds[r * WAVE + lane_id()]].obj != obj);
				}
#pragma unroll
				for (int r = 0; r < R; r++)
					any |= hm[r];
				if (!any)
					continue;
				if (meta & RTX_META_TRANSPARENT) {
					const auto *m = cptr(mats) + (meta & RTX_META_MAT);
					const float k0 = m->kt[0], k1 = m->kt[1], k2 = m->kt[2];
#pragma unroll
					for (int r = 0; r < R; r++) {
						if (!hm[r])
							continue;
						float *l = li_lds + r * WAVE + lane_id();
						const float x = l[0], y = l[R * WAVE], z = l[2 * R * WAVE];
						l[0] = msel(hm[r], x, x * k0);
						l[R * WAVE] = msel(hm[r], y, y * k1);
						l[2 * R * WAVE] = msel(hm[r], z, z * k2);
					}
				} else {
#pragma unroll
					for (int r = 0; r < R; r++)
						tl[r] = msel(hm[r], tl[r], -1.f);
					blk = true;
				}
			}
			if (blk) {
				u64 alive = 0;
#pragma unroll
				for (int r = 0; r < R; r++)
					alive |= ballot(tl[r] >= 0.f);
				if (!alive)
					sp = 0; /* every ray of the packet is blocked: end the walk */
			}
		}
		if (next == RTX_NONE) {
			if (sp == 0)
				break;
			next = readlane(stk, --sp);
		}
		ref = next;
	}
	if (RTX_SH_PF)
		drain(pf0, pf1);
}

/* R light samples per lane of the shade point `rec`, indices base + r * 64 + lane (render.c:
 * 170-229), through one shared-origin walk.  Each lane adds its samples' contributions to acc
 * in index order, the same sequence of float additions as the one-ray packets. */
template <bool COUNT, int R>
__device__ __forceinline__ void light_chunk(const KShadow &ks, const float4 *rec, uint32_t base, uint32_t nl,
					    float *li_lds, uint8_t *emit_lds, f3 &acc, ShadowCount &sc)
{
	reread_barrier();
	const float4 q0 = rec[0], q4 = rec[4];
	const f3 p = mk3(q0.x, q0.y, q0.z);
	const uint32_t obj = __float_as_uint(q4.x);
	const DEmitter *emitters = unip(ks.emitters);
	const uint32_t num_emitters = uni(ks.num_emitters);
	const bool rng_const = uni(ks.rng) == RTX_RNG_CONST;
	f3 d[R], inv[R];
	float tl[R], ldist[R], dsq[R];
	u64 live = 0, tri_any = 0;
#pragma unroll
	for (int r = 0; r < R; r++) {
		const uint32_t idx = base + (uint32_t)r * WAVE + lane_id();
		const bool act = idx < nl;
		uint32_t j = idx, e = 0;
		for (; e < num_emitters; e++) {
			const uint32_t eo = emitters[e].obj, enl = emitters[e].num_lights;
			if (eo == obj)
				continue;
			if (j < enl)
				break;
			j -= enl;
		}
		if (e >= num_emitters)
			e = 0;
		const DEmitter &E = emitters[e];
		float u1 = 0.5f, u2 = 0.5f;
		if (!rng_const)
			rtx_draw2(key_of(__float_as_uint(q4.y), __float_as_uint(q4.z)), e, j, &u1, &u2);
		const f3 lp = light_point_sh(E, p, u1, u2);
		const f3 dv = sub3(lp, p);
		ldist[r] = sh_mag(dv);
		dsq[r] = magsqr3(dv);
		d[r] = mul3s(dv, sh_rcp(ldist[r]));
		float *l = li_lds + r * WAVE + lane_id();
		l[0] = E.li[0];
		l[R * WAVE] = E.li[1];
		l[2 * R * WAVE] = E.li[2];
		tl[r] = act ? ldist[r] : -1.f;
		emit_lds[r * WAVE + lane_id()] = (uint8_t)e;
		tri_any |= ballot(act & (E.type == RTX_TRIANGLE));
	}
	/* planes first (unbound_objects_is_light_blocked, object.c:183-197) */
	const DPlane *planes = unip(ks.planes);
	const uint32_t num_planes = uni(ks.num_planes);
	for (uint32_t i = 0; i < num_planes; i++) {
		const auto *pl = cptr(planes) + i;
		const auto *m = cptr(unip(ks.mats)) + pl->mat;
		const f3 pn = mk3(pl->n[0], pl->n[1], pl->n[2]);
		const bool transparent = (m->flags & RTX_MF_TRANSPARENT) != 0;
#pragma unroll
		for (int r = 0; r < R; r++) {
			float t;
			const bool h = sh_hit_plane(pn, pl->d, p, d[r], pl->eps, t) && t < ldist[r] && tl[r] >= 0.f;
			if (transparent) {
				if (h) {
					float *l = li_lds + r * WAVE + lane_id();
					l[0] = l[0] * m->kt[0];
					l[R * WAVE] = l[R * WAVE] * m->kt[1];
					l[2 * R * WAVE] = l[2 * R * WAVE] * m->kt[2];
				}
			} else if (h) {
				tl[r] = -1.f;
			}
		}
	}
	if (COUNT)
#pragma unroll
		for (int r = 0; r < R; r++)
			sc.pln += (u64)popc64(ballot(base + (uint32_t)r * WAVE + lane_id() < nl)) * num_planes;
	uint32_t oct[R];
	uint32_t lead_r = R, lead_lane = 0;
#pragma unroll
	for (int r = R - 1; r >= 0; r--) {
		inv[r] = safe_inv_fast(d[r]);
		oct[r] = ((~__float_as_uint(inv[r].x)) >> 31) | (((~__float_as_uint(inv[r].y)) >> 31) << 1) |
			 (((~__float_as_uint(inv[r].z)) >> 31) << 2);
		const u64 lv = ballot(tl[r] >= 0.f);
		live |= lv;
		if (lv) {
			lead_r = (uint32_t)r;
			lead_lane = (uint32_t)__ffsll((long long)lv) - 1;
		}
	}
	const uint32_t root_ref = uni(ks.root_ref);
	if (live && root_ref != RTX_EMPTY_REF && !RTX_DEBUG_NOWALK) {
		uint32_t lead = 0, lead_emit = 0;
#pragma unroll
		for (int r = 0; r < R; r++)
			if ((uint32_t)r == lead_r) {
				lead = readlane(oct[r], lead_lane);
				lead_emit = readlane(emit_lds[r * WAVE + lane_id()], lead_lane);
			}
		u64 mixed_oct = 0, mixed_emit = 0;
#pragma unroll
		for (int r = 0; r < R; r++) {
			const bool alive = tl[r] >= 0.f;
			mixed_oct |= ballot(alive & (oct[r] != lead));
			mixed_emit |= ballot(alive & ((uint32_t)emit_lds[r * WAVE + lane_id()] != lead_emit));
		}
		const uint32_t emit_u = mixed_emit ? RTX_NONE : uni(emitters[uni(lead_emit)].obj);
		const bool tri_emit = tri_any != 0;
		const uint32_t sel = (!RTX_SH_OCT || mixed_oct) ? 8u : lead;
		const char *recs = (const char *)unip(ks.recs);
		const DMaterial *mats = unip(ks.mats);
		switch (sel) {
#define RTX_WALK_SO(K)                                                                                              \
	case K:                                                                                                         \
		shadow_walk_so<COUNT, K, R>(recs, mats, emitters, root_ref, p, d, inv, tl, li_lds, emit_u, emit_lds,        \
					    tri_emit, K, sc);                                                               \
		break;
#if RTX_SH_OCT
			RTX_WALK_SO(0) RTX_WALK_SO(1) RTX_WALK_SO(2) RTX_WALK_SO(3) RTX_WALK_SO(4) RTX_WALK_SO(5) RTX_WALK_SO(6)
			RTX_WALK_SO(7)
#endif
		default:
			shadow_walk_so<COUNT, 8, R>(recs, mats, emitters, root_ref, p, d, inv, tl, li_lds, emit_u, emit_lds,
						    tri_emit, lead, sc);
			break;
#undef RTX_WALK_SO
		}
	}
	reread_barrier();
#pragma unroll
	for (int r = 0; r < R; r++) {
		const uint32_t idx = base + (uint32_t)r * WAVE + lane_id();
		f3 contribution = mk3(0.f, 0.f, 0.f);
		if (idx < nl && tl[r] >= 0.f) {
			const float *l = li_lds + r * WAVE + lane_id();
			contribution = shade_light(ks, rec, d[r], mk3(l[0], l[R * WAVE], l[2 * R * WAVE]), ldist[r], dsq[r]);
		}
		acc = add3(acc, contribution);
	}
}

/* Persistent workgroups of RTX_SH_NW waves.  A workgroup copies the threaded BVH's top levels
 * (DScene.top) to LDS once; then each wave takes per_wave shade points at a time from a global
 * queue (RTX_C_SPQUEUE), in processing (Morton) order, until the points run out.  The resident
 * waves so work on one compact region of the scene at a time, and no workgroup waits on a tail.
 * A point's result depends only on the point (its sums run inside one wave, in lane order), not
 * on which wave takes it. */
template <bool COUNT, int OCC, int R>
__global__ __launch_bounds__(WAVE * RTX_SH_NW, OCC) void k_shadow(KShadow ka)
{
	__shared__ uint4 top_q[RTX_TOP_MAX];             /* the top records (rtx_device.h RTX_QTOP_CUT) */
	__shared__ uint32_t top_e[RTX_TOP_MAX];          /* cut records: the DQNode index after the subtree */
	__shared__ KShadow ks_w[RTX_SH_NW];
	__shared__ float li_w[RTX_SH_NW][R > 1 ? 3 * R * WAVE : 1]; /* R > 1: each ray's light intensity x transmittance */
	__shared__ uint8_t emit_w[RTX_SH_NW][R > 1 ? R * WAVE : 1]; /* R > 1: the emitter each ray aims at */
	__shared__ uint32_t off_w[RTX_SH_NW][WAVE + 1]; /* first lane slot of each shade point, total */
	__shared__ uint32_t nls_w[RTX_SH_NW][WAVE];     /* shadow rays of each shade point */
	__shared__ uint32_t sid_w[RTX_SH_NW][WAVE];     /* each shade point's index in the record array */
	__shared__ float Ls_w[RTX_SH_NW][3][WAVE];      /* per shade point light sum, in packet order */
	const uint32_t ntop = ka.ntop;
	for (uint32_t i = threadIdx.x; i < ntop; i += WAVE * RTX_SH_NW) {
		top_q[i] = ldg4u(ka.top + 4 * i);
		top_e[i] = gptr(ka.top)[4 * ntop + i];
	}
	const uint32_t wv = uni(threadIdx.x / WAVE);
	if (lane_id() == 0)
		ks_w[wv] = ka;
	__syncthreads();
	KShadow &ks = ks_w[wv];
	float *li_lds = li_w[wv];
	uint8_t *emit_lds = emit_w[wv];
	uint32_t *off = off_w[wv], *nls = nls_w[wv], *sid = sid_w[wv];
	float(*Ls)[WAVE] = Ls_w[wv];
	ShadowCount sc = { 0, 0, 0, 0, 0, 0, 0, 0 };
	u64 rays_total = 0;
	for (;;) {
		reread_barrier();
		uint32_t j0 = 0;
		if (lane_id() == 0)
			j0 = (uint32_t)atomicAdd(unip(ks.ctr) + RTX_C_SPQUEUE, (unsigned long long)uni(ks.per_wave));
		j0 = readlane(j0, 0);
		const uint32_t n_sp = uni(ks.n_sp);
		if (j0 >= n_sp)
			break;
		const uint32_t cnt = min(uni(ks.per_wave), n_sp - j0);
		const bool own = lane_id() < cnt;
		const uint32_t *perm = unip(ks.perm);
		const uint32_t my_sid = own ? (perm ? perm[j0 + lane_id()] : j0 + lane_id()) : 0u;
		const uint32_t nl_mine = own ? __float_as_uint(unip(ks.sp)[(size_t)my_sid * SPREC + 4].w) : 0u;
		/* each point's samples occupy whole lane slots of B lanes (B = power of two), so a point's
		 * packet partial sums never depend on which other points share its wave: deterministic */
		uint32_t total;
		const uint32_t ex = wave_excl_scan((nl_mine + uni(ks.slot_b) - 1) >> uni(ks.slot_lg), &total);
		off[lane_id()] = ex;
		nls[lane_id()] = nl_mine;
		sid[lane_id()] = my_sid;
		Ls[0][lane_id()] = 0.f;
		Ls[1][lane_id()] = 0.f;
		Ls[2][lane_id()] = 0.f;
		if (lane_id() == 0)
			off[WAVE] = total;
		lds_sync();
		uint32_t nmin = own ? nl_mine : 0xFFFFFFFFu;
		#pragma unroll
		for (int o = 32; o > 0; o >>= 1)
			nmin = min(nmin, (uint32_t)__shfl_xor(nmin, o, WAVE));
		if (RTX_SH_STREAM && R == 1 && uni(ks.slot_b) == WAVE && uni(nmin) >= WAVE) {
			/* Streamed samples: the batch's points' samples, concatenated, fill packets of 64 lanes,
			 * so a point's last part-filled packet is shared with the next point (each has >= 64
			 * samples, so a packet spans at most two).  Lane s keeps the running sum of the samples
			 * i == s (mod 64) of the current point (acc) and of the next (accn), pulled from whichever
			 * lane computed them: the same additions in the same order as the unstreamed loop, so
			 * every point's sum is bit-identical to it. */
			uint32_t tot_s;
			const uint32_t so = wave_excl_scan(own ? nl_mine : 0u, &tot_s);
			uint32_t k = 0;
			f3 acc = mk3(0.f, 0.f, 0.f), accn = acc;
			for (uint32_t base = 0; base < tot_s; base += WAVE) {
				reread_barrier();
				const uint32_t g = base + lane_id();
				const bool act = g < tot_s;
				const bool has2 = k + 1 < cnt;
				const uint32_t s0 = readlane(so, k), s1 = has2 ? readlane(so, k + 1) : tot_s;
				const bool second = has2 && g >= s1;
				const uint32_t kl = second ? k + 1 : k;
				const float4 *rec = unip(ks.sp) + (size_t)sid[kl] * SPREC;
				const f3 c = light_sample<COUNT>(ks, rec, g - (second ? s1 : s0), act, sc, top_q, top_e);
				const bool in0 = act && !second, in1 = act && second;
				const int la = (int)((lane_id() + s0 - base) & (WAVE - 1));
				const int lb = (int)((lane_id() + s1 - base) & (WAVE - 1));
				acc.x += __shfl(in0 ? c.x : 0.f, la, WAVE);
				acc.y += __shfl(in0 ? c.y : 0.f, la, WAVE);
				acc.z += __shfl(in0 ? c.z : 0.f, la, WAVE);
				accn.x += __shfl(in1 ? c.x : 0.f, lb, WAVE);
				accn.y += __shfl(in1 ? c.y : 0.f, lb, WAVE);
				accn.z += __shfl(in1 ? c.z : 0.f, lb, WAVE);
				if (base + WAVE >= s1) { /* point k ends in this packet */
					const float sx = wave_sum(acc.x), sy = wave_sum(acc.y), sz = wave_sum(acc.z);
					if (lane_id() == 0) {
						Ls[0][k] = sx;
						Ls[1][k] = sy;
						Ls[2][k] = sz;
					}
					acc = accn;
					accn = mk3(0.f, 0.f, 0.f);
					k++;
				}
			}
			lds_sync();
		} else if (uni(ks.slot_b) == WAVE) {
			/* >= 64 lights: every packet is 64 samples of ONE shade point.  The point is wave-uniform
			 * (its record is read once per packet through one address, no owner search), each lane
			 * sums its samples over the point's packets, and one butterfly per point reduces them. */
			for (uint32_t k = 0; k < cnt; k++) {
				reread_barrier();
				const uint32_t nl = uni(nls[k]);
				const float4 *rec = unip(ks.sp) + (size_t)uni(sid[k]) * SPREC;
				f3 acc = mk3(0.f, 0.f, 0.f);
				if (R > 1) {
					for (uint32_t base = 0; base < nl; base += R * WAVE)
						light_chunk<COUNT, R>(ks, rec, base, nl, li_lds, emit_lds, acc, sc);
				} else if (RTX_SH_REFILL > 0) {
					acc = point_refill<COUNT>(ks, rec, nl, sc, top_q, top_e);
				} else {
					for (uint32_t base = 0; base < nl; base += WAVE) {
						const uint32_t idx = base + lane_id();
						acc = add3(acc, light_sample<COUNT>(ks, rec, idx, idx < nl, sc, top_q, top_e));
					}
				}
				const float sx = wave_sum(acc.x), sy = wave_sum(acc.y), sz = wave_sum(acc.z);
				if (lane_id() == 0) {
					Ls[0][k] = sx;
					Ls[1][k] = sy;
					Ls[2][k] = sz;
				}
			}
			lds_sync();
		} else if constexpr (R == 1) {
			/* fewer lights: several points share a packet, each in its own power-of-two lane slot */
			for (uint32_t base = 0;;) {
				reread_barrier();
				const uint32_t tot = uni(off[WAVE]), slot_b = uni(ks.slot_b), slot_lg = uni(ks.slot_lg);
				if (base >= tot)
					break;
				const uint32_t slot = base + (lane_id() >> slot_lg);
				const uint32_t k = slot < tot ? owner_of(off, slot) : 0u;
				const uint32_t idx = ((slot - off[k]) << slot_lg) + (lane_id() & (slot_b - 1));
				const bool act = slot < tot && idx < nls[k];
				const float4 *rec = unip(ks.sp) + (size_t)sid[k] * SPREC;
				const f3 contribution = light_sample<COUNT>(ks, rec, idx, act, sc, top_q, top_e);
				/* per-shade-point sums; lanes are ordered by k */
				const uint32_t t2 = uni(off[WAVE]), sb = uni(ks.slot_b), spp = WAVE / sb;
				const uint32_t last_slot_lane = (min(t2 - base, spp) - 1) * sb;
				const uint32_t k0 = readlane(k, 0), k1 = readlane(k, last_slot_lane);
				for (uint32_t kk = k0; kk <= k1; kk++) {
					const bool in = act && k == kk;
					if (!ballot(in))
						continue;
					const float sx = wave_sum(in ? contribution.x : 0.f);
					const float sy = wave_sum(in ? contribution.y : 0.f);
					const float sz = wave_sum(in ? contribution.z : 0.f);
					if (lane_id() == 0) {
						Ls[0][kk] += sx;
						Ls[1][kk] += sy;
						Ls[2][kk] += sz;
					}
				}
				lds_sync();
				base += spp;
			}
		}
		reread_barrier();
		if (own) {
			const float4 *my = unip(ks.sp) + (size_t)my_sid * SPREC;
			const float4 q0 = my[0], q1 = my[1], q2 = my[2], q5 = my[5];
			const f3 w = mk3(q0.w, q1.w, q2.w);
			const f3 c = mul3v(w, mk3(Ls[0][lane_id()], Ls[1][lane_id()], Ls[2][lane_id()]));
			unip(ks.contrib)[my_sid] = make_float4(c.x, c.y, c.z, q5.x);
		}
		uint32_t n_rays = own ? nls[lane_id()] : 0u;
#pragma unroll
		for (int o = 32; o > 0; o >>= 1)
			n_rays += __shfl_xor(n_rays, o, WAVE);
		rays_total += uni(n_rays);
	}
	if (lane_id() == 0) {
		unsigned long long *ctr = unip(ks.ctr);
		atomicAdd(&ctr[RTX_C_SHADOW], rays_total);
		if (COUNT) {
			atomicAdd(&ctr[RTX_C_SNODES], sc.nodes);
			atomicAdd(&ctr[RTX_C_STRIS], sc.tris);
			atomicAdd(&ctr[RTX_C_SSPHERES], sc.sph);
			atomicAdd(&ctr[RTX_C_SPLANES], sc.pln);
			atomicAdd(&ctr[RTX_C_SSTEPS], sc.steps);
			atomicAdd(&ctr[RTX_C_SPSTEPS], sc.psteps);
			atomicAdd(&ctr[RTX_C_SRNODES], sc.rnodes);
			atomicAdd(&ctr[RTX_C_SRTRIS], sc.rprims);
		}
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
	return (size_t)WAVE * SPW * 4 + 80 * 4 + (size_t)stack_size * WAVE * 4;
}

extern "C" size_t rtx_shadow_lds_bytes(uint32_t stack_size)
{
	(void)stack_size; /* static LDS only; the packet stack lives in a VGPR (depth <= 63, checked at upload) */
	return 0;
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

/* the persistent k_shadow grid: as many workgroups as are resident on the device at once (no
 * more than the work needs); the waves then share the shade points through RTX_C_SPQUEUE */
template <bool C, int O, int R> static void launch_shadow(const KShadow &ka, uint32_t nw, hipStream_t stream)
{
	static uint32_t slots = 0;
	if (!slots) {
		int dev = 0, cus = 0, per_cu = 0;
		if (hipGetDevice(&dev) != hipSuccess ||
		    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
		    hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void *>(&k_shadow<C, O, R>),
								 WAVE * RTX_SH_NW, 0) != hipSuccess)
			per_cu = 0;
		slots = per_cu > 0 && cus > 0 ? (uint32_t)(per_cu * cus) : 1024u;
	}
	const uint32_t need = (nw + RTX_SH_NW - 1) / RTX_SH_NW;
	hipLaunchKernelGGL((k_shadow<C, O, R>), dim3(need < slots ? need : slots), dim3(WAVE * RTX_SH_NW), 0, stream, ka);
}

extern "C" hipError_t rtx_launch_shadow(const DScene *S, const DParams *P, const float4 *sp, const uint32_t *perm,
					uint32_t n_sp, uint32_t per_wave, uint32_t slot_b, uint32_t rays_per_lane,
					float4 *contrib, unsigned long long *ctr, int count, hipStream_t stream)
{
	if (RTX_SH_STREAM && slot_b == WAVE && rays_per_lane == 1 && per_wave < RTX_SH_STREAM)
		per_wave = RTX_SH_STREAM; /* streamed samples: more points per batch, fewer part-filled packets */
	const uint32_t nw = (n_sp + per_wave - 1) / per_wave;
	if (!nw)
		return hipSuccess;
	if (!slot_b || (slot_b & (slot_b - 1)) || slot_b > WAVE || !per_wave || per_wave > WAVE || !rays_per_lane ||
	    rays_per_lane > 5 || (rays_per_lane > 1 && slot_b != WAVE))
		return hipErrorInvalidValue;
	if (S->num_top > RTX_TOP_MAX)
		return hipErrorInvalidValue;
	KShadow ka;
	ka.recs = S->nodes;
	ka.qnodes = S->qnodes;
	ka.top = S->top;
	ka.ntop = S->num_top;
	for (int a = 0; a < 3; a++) {
		ka.qo[a] = S->qo[a];
		ka.qs[a] = S->qs[a];
	}
	ka.nq = S->num_qnodes;
	ka.mats = S->mats;
	ka.planes = S->planes;
	ka.emitters = S->emitters;
	ka.sp = sp;
	ka.perm = perm;
	ka.contrib = contrib;
	ka.ctr = ctr;
	ka.nnodes = S->num_nodes;
	ka.root_ref = S->root_ref;
	ka.num_planes = S->num_planes;
	ka.num_emitters = S->num_emitters;
	ka.n_sp = n_sp;
	ka.per_wave = per_wave;
	ka.slot_b = slot_b;
	ka.slot_lg = (uint32_t)__builtin_ctz(slot_b);
	ka.rng = P->rng;
	ka.attenuation = P->attenuation;
	ka.reflection = P->reflection;
	ka.att_offset = P->att_offset;
	/* occupancy variant: RTX_SHADOW_OCC = 1 (compiler's choice), 6, 7 or 8 waves/SIMD (register caps) */
	static int occ = -1;
	if (occ < 0) {
		const char *e = getenv("RTX_SHADOW_OCC");
		occ = e ? atoi(e) : RTX_SHADOW_OCC_DEFAULT;
	}
#define RTX_LAUNCH_SHADOW(C, O, R) launch_shadow<C, O, R>(ka, nw, stream)
#define RTX_LAUNCH_SHADOW_R(C, O)                                                                                \
	switch (rays_per_lane) {                                                                                     \
	case 2: RTX_LAUNCH_SHADOW(C, O, 2); break;                                                                   \
	case 3: RTX_LAUNCH_SHADOW(C, O, 3); break;                                                                   \
	case 4: RTX_LAUNCH_SHADOW(C, O, 4); break;                                                                   \
	case 5: RTX_LAUNCH_SHADOW(C, O, 5); break;                                                                   \
	default: RTX_LAUNCH_SHADOW(C, O, 1); break;                                                                  \
	}
	if (count) {
		RTX_LAUNCH_SHADOW_R(true, 1);
	} else if (rays_per_lane > 1) {
		RTX_LAUNCH_SHADOW_R(false, RTX_SHADOW_OCC_R);
	} else if (occ == 8) {
		RTX_LAUNCH_SHADOW(false, 8, 1);
	} else if (occ == 7) {
		RTX_LAUNCH_SHADOW(false, 7, 1);
	} else if (occ == 6) {
		RTX_LAUNCH_SHADOW(false, 6, 1);
	} else {
		RTX_LAUNCH_SHADOW(false, 1, 1);
	}
#undef RTX_LAUNCH_SHADOW_R
#undef RTX_LAUNCH_SHADOW
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
