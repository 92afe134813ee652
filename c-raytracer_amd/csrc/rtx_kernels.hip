/*
 * MI355X (gfx950) kernels for C-Raytracer's trace/intersect/shade hot path.
 *
 * One persistent kernel, one wavefront per workgroup.  Each wave pulls 8x8
 * pixel tiles from a device-wide queue (one returning atomic per tile) and
 * evaluates the reference's cast_ray() ray tree (render.c:136-343) for all 64
 * pixels of the tile, iteratively instead of recursively:
 *
 *   batch   = up to 64 closest-hit rays, one per lane (primaries of the tile,
 *             then reflection/refraction children popped from the wave's task
 *             stack in HBM; __ballot/mbcnt compaction on push)
 *   trace   = per-lane BVH2 traversal, stack in LDS ([entry][lane], conflict-free)
 *   shade   = per-lane hit setup; local terms (ke, ambient) routed to the
 *             owning pixel's accumulator; children pushed; shade points (SP)
 *             written to an LDS table
 *   light   = the (SP, light sample) pairs of the batch flattened and processed
 *             64 at a time; each group of 64 shadow rays traverses the BVH as a
 *             PACKET: node/primitive indices are wave-uniform, so node records
 *             come in through scalar loads, every lane tests its own ray and
 *             __ballot picks the children to descend (the shadow rays of one
 *             hit all aim at the same emitter, so the packet is coherent).
 *             Per-SP sums by a deterministic segmented wave reduction.
 *   GI      = (SP, sample) pairs flattened the same way, traced per lane,
 *             their hits shaded and lit like any other batch.
 *
 * Everything a pixel receives is summed in a fixed order inside one wave, so
 * the image is bit-identical whichever wave, GPU or tile order renders it.
 */
#include <hip/hip_runtime.h>
#include <float.h>

#include "rtx_kat.h"
#include "rtx_math.h"
#include "rtx_rng.h"

#define WAVE 64

/* ------------------------------------------------------------------------ */
/* wave helpers                                                             */
/* ------------------------------------------------------------------------ */
typedef unsigned long long u64;

__device__ __forceinline__ u64 ballot(bool p) { return __ballot(p); }
__device__ __forceinline__ uint32_t popc64(u64 m) { return (uint32_t)__popcll(m); }
__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }
__device__ __forceinline__ uint32_t mbcnt(u64 m)
{
	return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ float unif(float v) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v))); }
__device__ __forceinline__ uint32_t readlane(uint32_t v, uint32_t l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ float readlanef(float v, uint32_t l)
{
	return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

/* deterministic butterfly sum: every lane gets the same total */
__device__ __forceinline__ float wave_sum(float v)
{
#pragma unroll
	for (int o = 32; o > 0; o >>= 1)
		v += __shfl_xor(v, o, WAVE);
	return v;
}

/* exclusive prefix sum of v over the wave; total returned via *tot (uniform) */
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

/* ------------------------------------------------------------------------ */
/* kernel-wide context                                                      */
/* ------------------------------------------------------------------------ */
struct Ctx {
	DScene S;
	DFrame F;
	DParams P;
	float *lds_sp_a;   /* 64 SP records */
	float *lds_sp_b;   /* 64 SP records (aliases the traversal stack) */
	uint32_t *off_a;   /* 65 offsets */
	uint32_t *off_b;
	uint32_t *pstk;    /* packet stack (wave-uniform) */
	uint32_t *stk;     /* per-lane stack [entry][lane] */
	uint32_t total_lights;
	/* counters (wave-uniform) */
	u64 n_closest, n_shadow, n_nodes, n_tris, n_spheres, n_planes;
};

#define SPW 24 /* floats per shade-point record (6 x float4) */

struct SP {
	f3 p;
	float eps;
	f3 n;
	uint32_t obj;
	f3 d;
	uint32_t mat;
	f3 w;
	uint32_t slot;
	f3 tex;
	uint32_t key_lo;
	float delta;
	uint32_t ngi;
	uint32_t nl;
	uint32_t key_hi;
};

__device__ __forceinline__ void sp_store(float *tab, uint32_t k, const SP &s)
{
	float4 *q = (float4 *)(tab + k * SPW);
	q[0] = make_float4(s.p.x, s.p.y, s.p.z, s.eps);
	q[1] = make_float4(s.n.x, s.n.y, s.n.z, __uint_as_float(s.obj));
	q[2] = make_float4(s.d.x, s.d.y, s.d.z, __uint_as_float(s.mat));
	q[3] = make_float4(s.w.x, s.w.y, s.w.z, __uint_as_float(s.slot));
	q[4] = make_float4(s.tex.x, s.tex.y, s.tex.z, __uint_as_float(s.key_lo));
	q[5] = make_float4(s.delta, __uint_as_float(s.ngi), __uint_as_float(s.nl), __uint_as_float(s.key_hi));
}

__device__ __forceinline__ SP sp_load(const float *tab, uint32_t k)
{
	const float4 *q = (const float4 *)(tab + k * SPW);
	float4 a = q[0], b = q[1], c = q[2], d = q[3], e = q[4], f = q[5];
	SP s;
	s.p = mk3(a.x, a.y, a.z);
	s.eps = a.w;
	s.n = mk3(b.x, b.y, b.z);
	s.obj = __float_as_uint(b.w);
	s.d = mk3(c.x, c.y, c.z);
	s.mat = __float_as_uint(c.w);
	s.w = mk3(d.x, d.y, d.z);
	s.slot = __float_as_uint(d.w);
	s.tex = mk3(e.x, e.y, e.z);
	s.key_lo = __float_as_uint(e.w);
	s.delta = f.x;
	s.ngi = __float_as_uint(f.y);
	s.nl = __float_as_uint(f.z);
	s.key_hi = __float_as_uint(f.w);
	return s;
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

/* lights an SP on object `obj` samples: sum of num_lights of the emitters != obj */
__device__ __forceinline__ uint32_t lights_for(const Ctx &C, uint32_t obj)
{
	uint32_t n = C.total_lights;
	for (uint32_t e = 0; e < C.S.num_emitters; e++)
		if (C.S.emitters[e].obj == obj)
			n -= C.S.emitters[e].num_lights;
	return n;
}

/* ------------------------------------------------------------------------ */
/* closest hit: planes, then BVH (render.c:118-124); per-lane traversal     */
/* ------------------------------------------------------------------------ */
template <bool COUNT>
__device__ void trace_closest(Ctx &C, bool act, f3 o, f3 d, uint32_t inside, float &t_out, uint32_t &hid_out,
			      uint32_t &nodes, uint32_t &tris, uint32_t &sph, uint32_t &pln)
{
	const DScene &S = C.S;
	float tbest = FLT_MAX;
	uint32_t hid = RTX_NONE;
	if (act && isnan3(d)) /* TIR / degenerate directions: no hit */
		act = false;
	/* inside-object shortcut (render.c:143-144) */
	if (act && inside != RTX_NONE) {
		float t;
		bool h;
		if (inside & RTX_PLANE_BIT) {
			const DPlane &pl = S.planes[inside & ~RTX_PLANE_BIT];
			h = hit_plane(ld3(pl.n), pl.d, o, d, pl.eps, t);
		} else {
			const DPrim &pr = S.prims[inside];
			uint32_t type = __float_as_uint(pr.c[3]) >> 24;
			if (type == RTX_SPHERE)
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
				pln++;
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
		uint32_t *stk = C.stk + lane_id();
		for (;;) {
			if (ref & RTX_LEAF_BIT) {
				uint32_t first = (ref >> 4) & 0x7FFFFFFu, cnt = (ref & 15u) + 1;
				for (uint32_t k = 0; k < cnt; k++) {
					const DPrim &pr = S.prims[first + k];
					float4 a = *(const float4 *)pr.a, b = *(const float4 *)pr.b, c = *(const float4 *)pr.c;
					uint32_t type = __float_as_uint(c.w) >> 24;
					float t;
					bool h;
					if (type == RTX_SPHERE) {
						if (COUNT)
							sph++;
						h = hit_sphere(mk3(a.x, a.y, a.z), b.x, o, d, a.w, t);
					} else {
						if (COUNT)
							tris++;
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
				const float4 *nd = (const float4 *)(S.nodes + ref);
				float4 n0 = nd[0], n1 = nd[1], n2 = nd[2];
				uint4 n3 = *(const uint4 *)(nd + 3);
				if (COUNT)
					nodes++;
				float tn0, tn1;
				bool h0 = slab(n0.x, n0.y, n0.z, n0.w, n1.x, n1.y, oi, inv, tbest, tn0) && tn0 < tbest;
				bool h1 = slab(n1.z, n1.w, n2.x, n2.y, n2.z, n2.w, oi, inv, tbest, tn1) && tn1 < tbest;
				if (h0 && h1) {
					/* nearer child first; tie -> right first (accel.c:341-345) */
					uint32_t nr = tn0 < tn1 ? n3.x : n3.y, fr = tn0 < tn1 ? n3.y : n3.x;
					stk[sp++ * WAVE] = fr;
					ref = nr;
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

/* ------------------------------------------------------------------------ */
/* shadow any-hit with transmittance (render.c:126-134, object.c:183-197,   */
/* accel.c:360-387) for one group of <= 64 rays, BVH walked as a packet.    */
/* ------------------------------------------------------------------------ */
template <bool COUNT>
__device__ void shadow_packet(Ctx &C, bool act, f3 o, f3 d, float dist, uint32_t emit_obj, f3 &li, bool &blocked)
{
	const DScene &S = C.S;
	blocked = false;
	if (act) {
		for (uint32_t i = 0; i < S.num_planes; i++) {
			const DPlane &pl = S.planes[i];
			float t;
			if (hit_plane(ld3(pl.n), pl.d, o, d, pl.eps, t) && t < dist) {
				const DMaterial &m = S.mats[pl.mat];
				if (m.flags & RTX_MF_TRANSPARENT)
					li = mul3v(li, ld3(m.kt));
				else {
					blocked = true;
					break;
				}
			}
		}
	}
	if (COUNT)
		C.n_planes += (u64)popc64(ballot(act)) * S.num_planes;
	u64 live = ballot(act && !blocked);
	if (!live || S.root_ref == RTX_EMPTY_REF)
		return;
	const f3 inv = safe_inv(d);
	const f3 oi = mul3v(o, inv);
	/* near-first order from the first live ray's direction signs */
	const uint32_t lead = (uint32_t)__ffsll((long long)live) - 1;
	const uint32_t dsign = uni(((d.x >= 0.f) ? 1u : 0u) | ((d.y >= 0.f) ? 2u : 0u) | ((d.z >= 0.f) ? 4u : 0u));
	const uint32_t dsgn = readlane(dsign, lead);
	uint32_t ref = S.root_ref;
	uint32_t sp = 0;
	for (;;) {
		if (ref & RTX_LEAF_BIT) {
			const uint32_t first = (ref >> 4) & 0x7FFFFFFu, cnt = (ref & 15u) + 1;
			for (uint32_t k = 0; k < cnt; k++) {
				const DPrim &pr = S.prims[first + k];
				const uint32_t meta = __float_as_uint(pr.c[3]);
				const uint32_t type = meta >> 24;
				const uint32_t obj = __float_as_uint(pr.b[3]);
				const bool mine = ((live >> lane_id()) & 1ull) && obj != emit_obj;
				float t;
				bool h = false;
				if (type == RTX_SPHERE) {
					if (COUNT)
						C.n_spheres += popc64(live);
					if (mine)
						h = hit_sphere(mk3(pr.a[0], pr.a[1], pr.a[2]), pr.b[0], o, d, pr.a[3], t);
				} else {
					if (COUNT)
						C.n_tris += popc64(live);
					if (mine)
						h = hit_triangle(mk3(pr.a[0], pr.a[1], pr.a[2]), mk3(pr.b[0], pr.b[1], pr.b[2]),
								 mk3(pr.c[0], pr.c[1], pr.c[2]), o, d, pr.a[3], t);
				}
				h = h && t < dist;
				if (ballot(h)) {
					const DMaterial &m = S.mats[meta & 0xFFFFFFu];
					if (m.flags & RTX_MF_TRANSPARENT) {
						if (h)
							li = mul3v(li, mk3(m.kt[0], m.kt[1], m.kt[2]));
					} else if (h) {
						blocked = true;
					}
				}
			}
			live = ballot(((live >> lane_id()) & 1ull) && !blocked);
			if (!live || sp == 0)
				break;
			ref = uni(C.pstk[--sp]);
		} else {
			const DNode &nd = S.nodes[ref];
			const bool me = (live >> lane_id()) & 1ull;
			float tn0, tn1;
			bool h0 = me && slab(nd.lo0x, nd.hi0x, nd.lo0y, nd.hi0y, nd.lo0z, nd.hi0z, oi, inv, dist, tn0);
			bool h1 = me && slab(nd.lo1x, nd.hi1x, nd.lo1y, nd.hi1y, nd.lo1z, nd.hi1z, oi, inv, dist, tn1);
			if (COUNT)
				C.n_nodes += popc64(live);
			const u64 b0 = ballot(h0), b1 = ballot(h1);
			if (b0 && b1) {
				const uint32_t ax = nd.axis & 3u;
				const bool pos = (dsgn >> ax) & 1u;
				const bool lg = (nd.axis >> 2) & 1u;
				const uint32_t nr = (pos != lg) ? nd.ref0 : nd.ref1;
				const uint32_t fr = (pos != lg) ? nd.ref1 : nd.ref0;
				if (lane_id() == 0)
					C.pstk[sp] = fr;
				sp++;
				ref = nr;
			} else if (b0) {
				ref = nd.ref0;
			} else if (b1) {
				ref = nd.ref1;
			} else {
				if (sp == 0)
					break;
				ref = uni(C.pstk[--sp]);
			}
		}
	}
}

/* ------------------------------------------------------------------------ */
/* direct lighting (render.c:170-229) for the shade points in `tab`:        */
/* returns, in the owner lane k, L_k = sum over its light samples of        */
/* (diffuse + specular) before the SP weight is applied.                    */
/* ------------------------------------------------------------------------ */
template <bool COUNT>
__device__ f3 direct_light(Ctx &C, const float *tab, uint32_t *off, uint32_t nl_mine)
{
	const DParams &P = C.P;
	f3 L = mk3(0.f, 0.f, 0.f);
	uint32_t total;
	uint32_t ex = wave_excl_scan(nl_mine, &total);
	if (total == 0)
		return L;
	off[lane_id()] = ex;
	if (lane_id() == 0)
		off[WAVE] = total;
	__builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
	__builtin_amdgcn_wave_barrier();
	__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
	C.n_shadow += total;
	for (uint32_t base = 0; base < total; base += WAVE) {
		const uint32_t idx = base + lane_id();
		const bool act = idx < total;
		/* owner SP: largest k with off[k] <= idx */
		uint32_t k = 0;
		if (act) {
			uint32_t lo = 0, hi = WAVE; /* off[lo] <= idx < off[hi] */
			while (hi - lo > 1) {
				uint32_t mid = (lo + hi) >> 1;
				if (off[mid] <= idx)
					lo = mid;
				else
					hi = mid;
			}
			k = lo;
		}
		f3 contrib = mk3(0.f, 0.f, 0.f);
		const SP s = sp_load(tab, k);
		uint32_t j = idx - off[k];
		/* (emitter, light) of this sample, emitters in scene order, skipping the hit object */
		uint32_t e = 0;
		for (; e < C.S.num_emitters; e++) {
			const DEmitter &E = C.S.emitters[e];
			if (E.obj == s.obj)
				continue;
			if (j < E.num_lights)
				break;
			j -= E.num_lights;
		}
		if (e >= C.S.num_emitters)
			e = 0;
		const DEmitter &E = C.S.emitters[e];
		float u1, u2;
		draw(P, key_of(s.key_lo, s.key_hi), e, j, u1, u2);
		const f3 lp = light_point(E, s.p, u1, u2);
		const f3 dv = sub3(lp, s.p);
		const float ldist = mag3(dv);
		const f3 ldir = mul3s(dv, 1.f / ldist);
		const float a = dot3(ldir, s.n);
		f3 li = ld3(E.li);
		bool blocked;
		shadow_packet<COUNT>(C, act, s.p, ldir, ldist, E.obj, li, blocked);
		if (act && !blocked) {
			if (P.attenuation == RTX_ATT_LIN)
				li = mul3s(li, 1.f / (P.att_offset + ldist));
			else if (P.attenuation == RTX_ATT_SQR)
				li = mul3s(li, 1.f / (P.att_offset + magsqr3(dv)));
			const DMaterial &m = C.S.mats[s.mat];
			f3 diff = mul3s(mul3v(s.tex, li), fmaxf(0.f, a));
			float sm;
			if (P.reflection == RTX_BLINN) {
				f3 h = norm3(add3(mul3s(ldir, -1.f), s.d));
				sm = -dot3(s.n, h);
			} else {
				f3 r = sub3(mul3s(s.n, 2.f * a), ldir);
				sm = -dot3(r, s.d);
			}
			f3 spec = mul3s(mul3v(ld3(m.ks), li), fmaxf(0.f, powf(sm, m.shininess)));
			contrib = add3(diff, spec);
		}
		/* segmented reduction: lanes are ordered by k */
		const uint32_t last = min(total - base, (uint32_t)WAVE) - 1;
		const uint32_t k0 = readlane(k, 0), k1 = readlane(k, last);
		for (uint32_t kk = k0; kk <= k1; kk++) {
			const bool in = act && k == kk;
			if (!ballot(in))
				continue;
			float sx = wave_sum(in ? contrib.x : 0.f);
			float sy = wave_sum(in ? contrib.y : 0.f);
			float sz = wave_sum(in ? contrib.z : 0.f);
			if (lane_id() == kk) {
				L.x += sx;
				L.y += sy;
				L.z += sz;
			}
		}
	}
	return L;
}

/* add c (per lane) into the accumulator of pixel slot `slot` (owned by lane slot), fixed order */
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

__device__ __forceinline__ void lds_sync()
{
	__builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
	__builtin_amdgcn_wave_barrier();
	__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

struct HitInfo {
	f3 p, n;
	float b;
	bool outside;
	uint32_t obj, mat;
	float eps;
};

/* hit record of hid for ray (o,d) at t: point, normal (object.c sphere 254-265, triangle 356-365, plane 473-488) */
__device__ __forceinline__ HitInfo hit_info(const DScene &S, uint32_t hid, f3 o, f3 d, float t)
{
	HitInfo h;
	h.p = add3(mul3s(d, t), o);
	if (hid & RTX_PLANE_BIT) {
		const DPlane &pl = S.planes[hid & ~RTX_PLANE_BIT];
		f3 n = ld3(pl.n);
		h.n = signbit(dot3(n, d)) ? n : mul3s(n, -1.f);
		h.obj = pl.obj;
		h.mat = pl.mat;
		h.eps = pl.eps;
	} else {
		const DPrim &pr = S.prims[hid];
		const uint32_t meta = __float_as_uint(pr.c[3]);
		if ((meta >> 24) == RTX_SPHERE) {
			f3 c = mk3(pr.a[0], pr.a[1], pr.a[2]);
			h.n = mul3s(sub3(add3(mul3s(d, t), o), c), 1.f / pr.b[0]);
		} else {
			h.n = mk3(pr.d[0], pr.d[1], pr.d[2]);
		}
		h.obj = __float_as_uint(pr.b[3]);
		h.mat = meta & 0xFFFFFFu;
		h.eps = pr.a[3];
	}
	h.b = dot3(h.n, d);
	h.outside = signbit(h.b);
	return h;
}

/* ------------------------------------------------------------------------ */
/* GI for the shade points of tab_a with ngi > 0 (render.c:238-288)         */
/* ------------------------------------------------------------------------ */
template <bool COUNT>
__device__ void gi_batch(Ctx &C, uint32_t ngi_mine, f3 &acc, uint32_t &lane_nodes, uint32_t &lane_tris,
			 uint32_t &lane_sph, uint32_t &lane_pln)
{
	const DParams &P = C.P;
	uint32_t total;
	uint32_t ex = wave_excl_scan(ngi_mine, &total);
	if (total == 0)
		return;
	lds_sync();
	C.off_a[lane_id()] = ex;
	if (lane_id() == 0)
		C.off_a[WAVE] = total;
	lds_sync();
	for (uint32_t base = 0; base < total; base += WAVE) {
		const uint32_t idx = base + lane_id();
		const bool act = idx < total;
		uint32_t h = 0;
		if (act) {
			uint32_t lo = 0, hi = WAVE;
			while (hi - lo > 1) {
				uint32_t mid = (lo + hi) >> 1;
				if (C.off_a[mid] <= idx)
					lo = mid;
				else
					hi = mid;
			}
			h = lo;
		}
		const SP par = sp_load(C.lds_sp_a, h);
		const uint32_t s = idx - C.off_a[h];
		const uint64_t pkey = key_of(par.key_lo, par.key_hi);
		float u1, u2;
		draw(P, pkey, RTX_STREAM_GI, s, u1, u2);
		const f3 dir = gi_direction(par.n, par.eps, u1, u2);
		const f3 kr = mul3s(par.w, par.delta * dot3(par.n, dir));
		const uint64_t ckey = rtx_key_child(pkey, RTX_CHILD_GI0 + s);
		/* child cast_ray(.., 0 bounces, no inside object) */
		float t;
		uint32_t hid;
		lds_sync();
		trace_closest<COUNT>(C, act, par.p, dir, RTX_NONE, t, hid, lane_nodes, lane_tris, lane_sph, lane_pln);
		C.n_closest += popc64(ballot(act));
		const bool hit = act && hid != RTX_NONE;
		SP cs = SP();
		f3 cc = mk3(0.f, 0.f, 0.f);
		uint32_t nl = 0;
		if (hit) {
			HitInfo hi = hit_info(C.S, hid, par.p, dir, t);
			const DMaterial &m = C.S.mats[hi.mat];
			const f3 w = mul3s(kr, att_factor(P, t));
			cc = mul3v(w, ld3(m.ke)); /* path mode: no ambient term */
			nl = hi.outside ? lights_for(C, hi.obj) : 0u;
			cs.p = hi.p;
			cs.eps = hi.eps;
			cs.n = hi.n;
			cs.obj = hi.obj;
			cs.d = dir;
			cs.mat = hi.mat;
			cs.w = w;
			cs.slot = par.slot;
			cs.tex = nl ? texture_color(m, hi.p, P.u32conv) : mk3(0.f, 0.f, 0.f);
			cs.key_lo = (uint32_t)ckey;
			cs.key_hi = (uint32_t)(ckey >> 32);
			cs.delta = 0.f;
			cs.ngi = 0;
			cs.nl = nl;
		}
		route_add(acc, hit, par.slot, cc);
		lds_sync();
		if (hit)
			sp_store(C.lds_sp_b, lane_id(), cs);
		lds_sync();
		f3 L = direct_light<COUNT>(C, C.lds_sp_b, C.off_b, nl);
		route_add(acc, nl != 0, cs.slot, mul3v(cs.w, L));
		lds_sync();
	}
}

/* ------------------------------------------------------------------------ */
/* the persistent render kernel                                             */
/* ------------------------------------------------------------------------ */
template <bool COUNT>
__global__ __launch_bounds__(WAVE) void k_render(DScene S, DFrame F, DParams P, float *__restrict__ rgb,
						 float *__restrict__ zbuf, DTask *__restrict__ tasks, uint32_t task_cap,
						 unsigned long long *__restrict__ ctr)
{
	extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
	Ctx C;
	C.S = S;
	C.F = F;
	C.P = P;
	{
		unsigned char *p = lds_raw;
		C.lds_sp_a = (float *)p;
		p += WAVE * SPW * 4;
		C.off_a = (uint32_t *)p;
		p += 80 * 4;
		C.off_b = (uint32_t *)p;
		p += 80 * 4;
		C.pstk = (uint32_t *)p;
		p += ((S.stack_size + 3) & ~3u) * 4;
		C.stk = (uint32_t *)p;
		C.lds_sp_b = (float *)p;
	}
	C.total_lights = 0;
	for (uint32_t e = 0; e < S.num_emitters; e++)
		C.total_lights += S.emitters[e].num_lights;
	C.n_closest = C.n_shadow = C.n_nodes = C.n_tris = C.n_spheres = C.n_planes = 0;
	uint32_t lane_nodes = 0, lane_tris = 0, lane_sph = 0, lane_pln = 0;
	DTask *my_tasks = tasks + (size_t)blockIdx.x * task_cap;
	uint32_t overflow = 0;

	for (;;) {
		uint32_t tile = 0;
		if (lane_id() == 0)
			tile = (uint32_t)atomicAdd(&ctr[RTX_C_TILE], 1ull);
		tile = uni(__shfl(tile, 0, WAVE));
		if (tile >= P.ntiles)
			break;
		const uint32_t g = P.tile_offset + tile * P.tile_stride;
		const uint32_t tx = g % P.tiles_x, ty = g / P.tiles_x;
		const uint32_t px = tx * RTX_TILE_W + (lane_id() & 7), py = ty * RTX_TILE_H + (lane_id() >> 3);
		const bool valid_px = px < F.width && py < F.height;

		f3 acc = mk3(0.f, 0.f, 0.f);
		float zval = 0.f;

		/* primary rays (render.c:353-363): P = corner + row*vy, then += vx (col+1) times */
		bool act = valid_px;
		f3 o = ld3(F.origin), d = mk3(0.f, 0.f, 1.f), kr = mk3(1.f, 1.f, 1.f);
		uint32_t rb = P.max_bounces, inside = RTX_NONE, slot = lane_id();
		uint64_t key = 0;
		bool primary = true;
		if (act) {
			f3 pp = add3(mul3s(ld3(F.step_y), (float)py), ld3(F.corner));
			for (uint32_t c = 0; c <= px; c++)
				pp = add3(pp, ld3(F.step_x));
			d = norm3(sub3(pp, o));
			key = rtx_key_pixel(P.seed, py * F.width + px);
		}
		uint32_t top = 0;
		for (;;) {
			/* ---- trace the batch ---- */
			float t;
			uint32_t hid;
			lds_sync();
			trace_closest<COUNT>(C, act, o, d, inside, t, hid, lane_nodes, lane_tris, lane_sph, lane_pln);
			C.n_closest += popc64(ballot(act));
			const bool hit = act && hid != RTX_NONE;
			/* ---- shade setup ---- */
			SP sp = SP();
			f3 cc = mk3(0.f, 0.f, 0.f);
			uint32_t nl = 0, ngi = 0;
			bool want_refl = false, want_refr = false;
			f3 rkr = mk3(0.f, 0.f, 0.f), rkt = mk3(0.f, 0.f, 0.f), rdir = mk3(0.f, 0.f, 0.f),
			   tdir = mk3(0.f, 0.f, 0.f);
			if (hit) {
				HitInfo h = hit_info(S, hid, o, d, t);
				const DMaterial &m = S.mats[h.mat];
				const f3 w = mul3s(kr, att_factor(P, t));
				f3 local = ld3(m.ke);
				if (P.gi == RTX_GI_AMBIENT)
					local = add3(local, mul3v(ld3(m.ka), ld3(S.ambient)));
				cc = mul3v(w, local);
				if (primary)
					zval = rb ? t : 0.f;
				if (rb) {
					if (inside != hid && (m.flags & RTX_MF_REFLECTIVE)) {
						rkr = mul3v(kr, ld3(m.kr));
						if (P.min_intensity_sqr < magsqr3(rkr)) {
							want_refl = true;
							rdir = sub3(d, mul3s(h.n, 2.f * h.b));
						}
					}
					if (m.flags & RTX_MF_TRANSPARENT) {
						rkt = mul3v(kr, ld3(m.kt));
						if (P.min_intensity_sqr < magsqr3(rkt)) {
							want_refr = true;
							tdir = refract_dir(d, h.n, h.b, h.outside, m.ior);
						}
					}
				}
				nl = h.outside ? lights_for(C, h.obj) : 0u;
				ngi = (P.gi == RTX_GI_PATH && rb && h.outside) ? (rb == P.max_bounces ? P.samples : 1u) : 0u;
				sp.p = h.p;
				sp.eps = h.eps;
				sp.n = h.n;
				sp.obj = h.obj;
				sp.d = d;
				sp.mat = h.mat;
				sp.w = w;
				sp.slot = slot;
				sp.tex = nl ? texture_color(m, h.p, P.u32conv) : mk3(0.f, 0.f, 0.f);
				sp.key_lo = (uint32_t)key;
				sp.key_hi = (uint32_t)(key >> 32);
				sp.delta = (rb == P.max_bounces) ? 1.f / (float)P.samples : 1.f;
				sp.ngi = ngi;
				sp.nl = nl;
			}
			route_add(acc, hit, slot, cc);
			if (primary && act)
				zval = hit ? zval : 0.f;
			/* ---- push reflection / refraction children (compacted) ---- */
			{
				const u64 mr = ballot(want_refl), mt = ballot(want_refr);
				const uint32_t nr = popc64(mr), nt = popc64(mt);
				if (nr + nt) {
					if (top + nr + nt > task_cap) {
						overflow = 1;
					} else {
						uint32_t pos_r = top + mbcnt(mr), pos_t = top + nr + mbcnt(mt);
						const uint64_t kref = rtx_key_child(key, RTX_CHILD_REFLECT);
						const uint64_t krft = rtx_key_child(key, RTX_CHILD_REFRACT);
						if (want_refl) {
							DTask tk;
							tk.o[0] = sp.p.x; tk.o[1] = sp.p.y; tk.o[2] = sp.p.z;
							tk.d[0] = rdir.x; tk.d[1] = rdir.y; tk.d[2] = rdir.z;
							tk.kr[0] = rkr.x; tk.kr[1] = rkr.y; tk.kr[2] = rkr.z;
							tk.rb = rb - 1;
							tk.inside = RTX_NONE;
							tk.key_lo = (uint32_t)kref;
							tk.key_hi = (uint32_t)(kref >> 32);
							tk.slot = slot;
							my_tasks[pos_r] = tk;
						}
						if (want_refr) {
							DTask tk;
							tk.o[0] = sp.p.x; tk.o[1] = sp.p.y; tk.o[2] = sp.p.z;
							tk.d[0] = tdir.x; tk.d[1] = tdir.y; tk.d[2] = tdir.z;
							tk.kr[0] = rkt.x; tk.kr[1] = rkt.y; tk.kr[2] = rkt.z;
							tk.rb = rb - 1;
							tk.inside = hid;
							tk.key_lo = (uint32_t)krft;
							tk.key_hi = (uint32_t)(krft >> 32);
							tk.slot = slot;
							my_tasks[pos_t] = tk;
						}
						top += nr + nt;
					}
				}
			}
			/* ---- direct light of the batch's shade points ---- */
			lds_sync();
			if (hit)
				sp_store(C.lds_sp_a, lane_id(), sp);
			lds_sync();
			{
				f3 L = direct_light<COUNT>(C, C.lds_sp_a, C.off_b, nl);
				route_add(acc, nl != 0, slot, mul3v(sp.w, L));
			}
			/* ---- path-traced GI children ---- */
			if (P.gi == RTX_GI_PATH)
				gi_batch<COUNT>(C, ngi, acc, lane_nodes, lane_tris, lane_sph, lane_pln);
			/* ---- next batch: pop up to 64 tasks (LIFO) ---- */
			if (top == 0)
				break;
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
		/* ---- write the tile ---- */
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
	}
	/* ---- counters ---- */
	if (COUNT) {
		u64 ln = lane_nodes, lt = lane_tris, ls = lane_sph, lp = lane_pln;
#pragma unroll
		for (int o2 = 32; o2 > 0; o2 >>= 1) {
			ln += __shfl_xor(ln, o2, WAVE);
			lt += __shfl_xor(lt, o2, WAVE);
			ls += __shfl_xor(ls, o2, WAVE);
			lp += __shfl_xor(lp, o2, WAVE);
		}
		C.n_nodes += ln;
		C.n_tris += lt;
		C.n_spheres += ls;
		C.n_planes += lp;
	}
	if (lane_id() == 0) {
		atomicAdd(&ctr[RTX_C_CLOSEST], C.n_closest);
		atomicAdd(&ctr[RTX_C_SHADOW], C.n_shadow);
		if (COUNT) {
			atomicAdd(&ctr[RTX_C_NODES], C.n_nodes);
			atomicAdd(&ctr[RTX_C_TRIS], C.n_tris);
			atomicAdd(&ctr[RTX_C_SPHERES], C.n_spheres);
			atomicAdd(&ctr[RTX_C_PLANES], C.n_planes);
		}
		if (overflow)
			atomicAdd(&ctr[RTX_C_OVERFLOW], 1ull);
	}
}

/* ------------------------------------------------------------------------ */
/* known-answer kernel (include/rtx_kat.h)                                  */
/* ------------------------------------------------------------------------ */
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
extern "C" size_t rtx_render_lds_bytes(uint32_t stack_size)
{
	size_t sp = (size_t)WAVE * SPW * 4;
	size_t stk = (size_t)stack_size * WAVE * 4;
	return sp + 2 * 80 * 4 + (((size_t)stack_size + 3) & ~3ull) * 4 + (stk > sp ? stk : sp);
}

extern "C" hipError_t rtx_launch_render(const DScene *S, const DFrame *F, const DParams *P, float *rgb, float *z,
					 DTask *tasks, uint32_t task_cap, unsigned long long *ctr, uint32_t waves,
					 int count, hipStream_t stream)
{
	size_t lds = rtx_render_lds_bytes(S->stack_size);
	if (count) {
		hipLaunchKernelGGL(k_render<true>, dim3(waves), dim3(WAVE), lds, stream, *S, *F, *P, rgb, z, tasks,
				   task_cap, ctr);
	} else {
		hipLaunchKernelGGL(k_render<false>, dim3(waves), dim3(WAVE), lds, stream, *S, *F, *P, rgb, z, tasks,
				   task_cap, ctr);
	}
	return hipGetLastError();
}

extern "C" hipError_t rtx_launch_kat(int kind, uint32_t n, const float *in, float *out, int u32mode,
				      hipStream_t stream)
{
	hipLaunchKernelGGL(k_kat, dim3((n + 255) / 256), dim3(256), 0, stream, kind, n, in, out, u32mode);
	return hipGetLastError();
}

extern "C" hipError_t rtx_render_occupancy(uint32_t stack_size, int *blocks_per_cu)
{
	size_t lds = rtx_render_lds_bytes(stack_size);
	return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, k_render<false>, WAVE, lds);
}
