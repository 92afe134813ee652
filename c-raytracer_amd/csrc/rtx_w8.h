/*
 * Device helpers shared by the walks of the 8-wide compressed BVH (rtx_device.h DW8 / DW8S):
 * the shadow any-hit walk (rtx_shadow.hip shadow_walk8) and the closest-hit walk
 * (rtx_trace.hip trace_closest_w8).  Both test a node's eight child boxes the same way
 * (accel.c:112-158's slab test, conservative on the quantised boxes), on the ray in the trees'
 * frame (rtx_device.h DTreeFrame).
 */
#ifndef RTX_W8_H
#define RTX_W8_H

#include <hip/hip_runtime.h>

#include "rtx_device.h"
#include "rtx_math.h"

/* ------------------------------------------------------------------------ */
/* loads                                                                    */
/* ------------------------------------------------------------------------ */
/* per-lane loads through the global address space (global_load, not flat_load: the pointers
 * come from LDS and the compiler cannot prove where they point) */
template <typename T> __device__ __forceinline__ const __attribute__((address_space(1))) T *gptr(const T *p)
{
	return (const __attribute__((address_space(1))) T *)p;
}
template <typename T> __device__ __forceinline__ __attribute__((address_space(1))) T *gptrw(T *p)
{
	return (__attribute__((address_space(1))) T *)p;
}
/* wave-uniform reads of read-only scene tables (s_load) */
template <typename T> __device__ __forceinline__ const __attribute__((address_space(4))) T *cptr(const T *p)
{
	return (const __attribute__((address_space(4))) T *)p;
}
typedef float f4v __attribute__((ext_vector_type(4)));
typedef uint32_t u4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 ldg4(const void *p, uint32_t off)
{
	const f4v v = *(const __attribute__((address_space(1))) f4v *)((const char *)p + off);
	return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint4 ldg4u(const void *p)
{
	const u4v v = *(const __attribute__((address_space(1))) u4v *)p;
	return make_uint4(v.x, v.y, v.z, v.w);
}
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
__device__ __forceinline__ void lds1st(uint32_t *p, uint32_t v) { *(__attribute__((address_space(3))) uint32_t *)p = v; }
/* a 32-bit LDS pointer (the lane stacks): one VGPR instead of a 64-bit generic pointer */
typedef __attribute__((address_space(3))) uint32_t lds_u32;

/* byte B of w as a float (v_cvt_f32_ubyteB) */
template <int B> __device__ __forceinline__ float ubyte(uint32_t w) { return (float)((w >> (8 * B)) & 0xFFu); }

/* the 8-bit mask m with bit i moved to bit i ^ K (K < 8 a compile-time constant) */
template <uint32_t K> __device__ __forceinline__ uint32_t perm_xor(uint32_t m)
{
	if (K & 1u)
		m = ((m & 0x55u) << 1) | ((m >> 1) & 0x55u);
	if (K & 2u)
		m = ((m & 0x33u) << 2) | ((m >> 2) & 0x33u);
	if (K & 4u)
		m = ((m & 0x0Fu) << 4) | ((m >> 4) & 0x0Fu);
	return m;
}

/* The slab test (accel.c:112-158) of child C of an 8-wide node (rtx_device.h DW8) on the segment
 * (0, tl): t = q8 * s + b per plane, with s = invq * 2^e and b = o * invq - oi the node frame's
 * scale and offset of the walk's ray transform (box_hit_q), so the same conservative grid test
 * on the box rounded outward to the node's 8-bit frame (KAT: RTX_KAT_BOX_Q8).  OCT < 8: every
 * live lane's direction lies in octant OCT, entry planes known at compile time; an empty slot
 * (lo 255 > hi 0) is then never hit. */
template <int OCT>
__device__ __forceinline__ bool w8_slab_tn(float lx, float hx, float ly, float hy, float lz, float hz, float tl, float &tn_out)
{
	if (OCT == 8) {
		const float tn = fmaxf(fmaxf(fminf(lx, hx), fminf(ly, hy)), fmaxf(fminf(lz, hz), 0.f));
		const float tf = fminf(fminf(fmaxf(lx, hx), fmaxf(ly, hy)), fminf(fmaxf(lz, hz), tl));
		tn_out = tn;
		return tn <= tf;
	}
	const float nx = (OCT & 1) ? lx : hx, fx = (OCT & 1) ? hx : lx;
	const float ny = (OCT & 2) ? ly : hy, fy = (OCT & 2) ? hy : ly;
	const float nz = (OCT & 4) ? lz : hz, fz = (OCT & 4) ? hz : lz;
	const float tn = fmaxf(fmaxf(nx, ny), fmaxf(nz, 0.f));
	float tf = fminf(fminf(fx, fy), fz);
	asm("v_min_f32 %0, %0, %1" : "+v"(tf) : "v"(tl));
	tn_out = tn;
	return tn <= tf;
}
template <int OCT>
__device__ __forceinline__ bool w8_slab(float lx, float hx, float ly, float hy, float lz, float hz, float tl)
{
	if (OCT == 8) {
		const float tn = fmaxf(fmaxf(fminf(lx, hx), fminf(ly, hy)), fmaxf(fminf(lz, hz), 0.f));
		const float tf = fminf(fminf(fmaxf(lx, hx), fmaxf(ly, hy)), fminf(fmaxf(lz, hz), tl));
		return tn <= tf;
	}
	const float nx = (OCT & 1) ? lx : hx, fx = (OCT & 1) ? hx : lx;
	const float ny = (OCT & 2) ? ly : hy, fy = (OCT & 2) ? hy : ly;
	const float nz = (OCT & 4) ? lz : hz, fz = (OCT & 4) ? hz : lz;
	const float tn = fmaxf(fmaxf(nx, ny), fmaxf(nz, 0.f));
	float tf = fminf(fminf(fx, fy), fz);
	asm("v_min_f32 %0, %0, %1" : "+v"(tf) : "v"(tl));
	return tn <= tf;
}
/* The same test (OCT < 8) as a word whose sign bit says "miss": with A the entry (max of the near
 * planes) and C the exit clipped to tl (min of the far planes and tl), the box is hit when
 * A <= C and C >= 0, i.e. when neither C - A nor C is negative.  Two full-rate VALU operations
 * (v_sub_f32, v_or_b32, which gfx950 dual-issues) replace v_max(0), v_cmp and v_cndmask, which it
 * does not (tools/dev/valu_rates.hip).  The two tests differ only where C or C - A is -0, a box
 * the ray touches at t = 0 alone, which holds no hit beyond the primitives' epsilon. */
template <int OCT>
__device__ __forceinline__ uint32_t w8_slab_miss(float lx, float hx, float ly, float hy, float lz, float hz, float tl)
{
	static_assert(OCT < 8, "octant-specialised only");
	const float nx = (OCT & 1) ? lx : hx, fx = (OCT & 1) ? hx : lx;
	const float ny = (OCT & 2) ? ly : hy, fy = (OCT & 2) ? hy : ly;
	const float nz = (OCT & 4) ? lz : hz, fz = (OCT & 4) ? hz : lz;
	const float a = fmaxf(fmaxf(nx, ny), nz);
	float c = fminf(fminf(fx, fy), fz);
	asm("v_min_f32 %0, %0, %1" : "+v"(c) : "v"(tl));
	return __float_as_uint(c - a) | __float_as_uint(c);
}
/* bit P of the miss word's sign (P < 8): v_lshrrev_b32 + v_and_b32, both dual-issued */
template <int P> __device__ __forceinline__ uint32_t w8_miss_bit(uint32_t m)
{
	return (m >> (31 - P)) & (1u << P);
}

template <int OCT, int C>
__device__ __forceinline__ bool w8_child(const uint32_t (&w)[16], f3 s, f3 b, float tl)
{
	constexpr int W = C >> 2, B = C & 3;
	return w8_slab<OCT>(fmaf(ubyte<B>(w[4 + W]), s.x, b.x), fmaf(ubyte<B>(w[6 + W]), s.x, b.x),
			    fmaf(ubyte<B>(w[8 + W]), s.y, b.y), fmaf(ubyte<B>(w[10 + W]), s.y, b.y),
			    fmaf(ubyte<B>(w[12 + W]), s.z, b.z), fmaf(ubyte<B>(w[14 + W]), s.z, b.z), tl);
}
/* the scalar-path copy (rtx_device.h DW8S): child C's plane offsets, ready floats (the same
 * values the conversions above produce, so the results are bit-identical), one s_load_dwordx8 */
typedef float f2v __attribute__((ext_vector_type(2)));
typedef float f8v __attribute__((ext_vector_type(8)));
template <int C> __device__ __forceinline__ f8v w8s_planes(const DW8S *n)
{
	return *(const __attribute__((address_space(4))) f8v *)&n->q[C][0];
}
/* one axis's two plane distances q * s + b: the SGPR pair in one v_pk_fma_f32 */
__device__ __forceinline__ f2v w8s_axis(float lo, float hi, float s, float b)
{
	const f2v q = { lo, hi }, sv = { s, s }, bv = { b, b };
	return __builtin_elementwise_fma(q, sv, bv);
}
template <int OCT, int C>
__device__ __forceinline__ bool w8_child_s(const DW8S *n, f3 s, f3 b, float tl)
{
	const f8v p = w8s_planes<C>(n);
	const f2v tx = w8s_axis(p[0], p[1], s.x, b.x), ty = w8s_axis(p[2], p[3], s.y, b.y), tz = w8s_axis(p[4], p[5], s.z, b.z);
	return w8_slab<OCT>(tx.x, tx.y, ty.x, ty.y, tz.x, tz.y, tl);
}

/* the node frame of an 8-wide node: per-axis scale s = invq * 2^e and offset b = o * invq - oi */
__device__ __forceinline__ void w8_frame(const uint32_t (&w)[16], f3 invq, f3 oi, f3 &s, f3 &b)
{
	s = mk3(ldexpf(invq.x, (int)((w[1] >> 16) & 15u)), ldexpf(invq.y, (int)((w[1] >> 20) & 15u)),
		ldexpf(invq.z, (int)((w[1] >> 24) & 15u)));
	b = mk3(fmaf((float)(w[0] & 0xFFFFu), invq.x, -oi.x), fmaf((float)(w[0] >> 16), invq.y, -oi.y),
		fmaf((float)(w[1] & 0xFFFFu), invq.z, -oi.z));
}

template <int OCT, int C>
__device__ __forceinline__ uint32_t w8_child_miss(const uint32_t (&w)[16], f3 s, f3 b, float tl)
{
	constexpr int W = C >> 2, B = C & 3;
	return w8_slab_miss<OCT>(fmaf(ubyte<B>(w[4 + W]), s.x, b.x), fmaf(ubyte<B>(w[6 + W]), s.x, b.x),
				 fmaf(ubyte<B>(w[8 + W]), s.y, b.y), fmaf(ubyte<B>(w[10 + W]), s.y, b.y),
				 fmaf(ubyte<B>(w[12 + W]), s.z, b.z), fmaf(ubyte<B>(w[14 + W]), s.z, b.z), tl);
}
#ifndef RTX_W8_SIGN
#define RTX_W8_SIGN 1 /* k_shadow's octant-specialised box tests through miss words (w8_slab_miss) */
#endif
/* hit mask of an 8-wide node's children in visit order: bit p for slot p ^ K */
template <int OCT, uint32_t K>
__device__ __forceinline__ uint32_t w8_hits(const uint32_t (&w)[16], f3 s, f3 b, float tl)
{
	if constexpr (OCT < 8 && RTX_W8_SIGN) {
		uint32_t m = w8_miss_bit<0 ^ K>(w8_child_miss<OCT, 0>(w, s, b, tl));
		m |= w8_miss_bit<1 ^ K>(w8_child_miss<OCT, 1>(w, s, b, tl));
		m |= w8_miss_bit<2 ^ K>(w8_child_miss<OCT, 2>(w, s, b, tl));
		m |= w8_miss_bit<3 ^ K>(w8_child_miss<OCT, 3>(w, s, b, tl));
		m |= w8_miss_bit<4 ^ K>(w8_child_miss<OCT, 4>(w, s, b, tl));
		m |= w8_miss_bit<5 ^ K>(w8_child_miss<OCT, 5>(w, s, b, tl));
		m |= w8_miss_bit<6 ^ K>(w8_child_miss<OCT, 6>(w, s, b, tl));
		m |= w8_miss_bit<7 ^ K>(w8_child_miss<OCT, 7>(w, s, b, tl));
		return m ^ 0xFFu;
	}
	uint32_t hm = 0;
	hm |= w8_child<OCT, 0>(w, s, b, tl) ? 1u << (0 ^ K) : 0u;
	hm |= w8_child<OCT, 1>(w, s, b, tl) ? 1u << (1 ^ K) : 0u;
	hm |= w8_child<OCT, 2>(w, s, b, tl) ? 1u << (2 ^ K) : 0u;
	hm |= w8_child<OCT, 3>(w, s, b, tl) ? 1u << (3 ^ K) : 0u;
	hm |= w8_child<OCT, 4>(w, s, b, tl) ? 1u << (4 ^ K) : 0u;
	hm |= w8_child<OCT, 5>(w, s, b, tl) ? 1u << (5 ^ K) : 0u;
	hm |= w8_child<OCT, 6>(w, s, b, tl) ? 1u << (6 ^ K) : 0u;
	hm |= w8_child<OCT, 7>(w, s, b, tl) ? 1u << (7 ^ K) : 0u;
	if (OCT == 8)
		hm &= w[3]; /* K = 0: slot order; the min/max form would turn an empty slot's box around */
	return hm;
}
#ifndef RTX_W8_SKIP
#define RTX_W8_SKIP 1 /* scalar path: branch over the empty slots (the slot mask is wave-uniform): scene5 k_shadow 557 -> 548 ms, scene6 2739 -> 2721 ms */
#endif
template <int OCT, uint32_t K, int C>
__device__ __forceinline__ uint32_t w8_hit_s(const DW8S *n, uint32_t w3, f3 s, f3 b, float tl)
{
	if (RTX_W8_SKIP && !((w3 >> C) & 1u))
		return 0u;
	if constexpr (OCT < 8 && RTX_W8_SIGN) { /* the divergent path's miss-word form: the same bits */
		const f8v p = w8s_planes<C>(n);
		const f2v tx = w8s_axis(p[0], p[1], s.x, b.x), ty = w8s_axis(p[2], p[3], s.y, b.y), tz = w8s_axis(p[4], p[5], s.z, b.z);
		const uint32_t m = w8_slab_miss<OCT>(tx.x, tx.y, ty.x, ty.y, tz.x, tz.y, tl);
		return w8_miss_bit<C ^ K>(m) ^ (1u << (C ^ K));
	}
	return w8_child_s<OCT, C>(n, s, b, tl) ? 1u << (C ^ K) : 0u;
}
template <int OCT, uint32_t K>
__device__ __forceinline__ uint32_t w8_hits_s(const DW8S *q, uint32_t w3, f3 s, f3 b, float tl)
{
	uint32_t hm = 0;
	hm |= w8_hit_s<OCT, K, 0>(q, w3, s, b, tl);
	hm |= w8_hit_s<OCT, K, 1>(q, w3, s, b, tl);
	hm |= w8_hit_s<OCT, K, 2>(q, w3, s, b, tl);
	hm |= w8_hit_s<OCT, K, 3>(q, w3, s, b, tl);
	hm |= w8_hit_s<OCT, K, 4>(q, w3, s, b, tl);
	hm |= w8_hit_s<OCT, K, 5>(q, w3, s, b, tl);
	hm |= w8_hit_s<OCT, K, 6>(q, w3, s, b, tl);
	hm |= w8_hit_s<OCT, K, 7>(q, w3, s, b, tl);
	if (OCT == 8 && !RTX_W8_SKIP)
		hm &= w3;
	return hm;
}

#ifndef RTX_W8_ORDER
#define RTX_W8_ORDER 1 /* closest hits (k_trace): visit hit children in the octant's slot order (0: plain slot order) */
#endif
#ifndef RTX_W8_SORDER
#define RTX_W8_SORDER 0 /* any-hit (k_shadow): the octant's slot order; plain slot order saves the mask permutes */
#endif

/* one 8-wide node visit's box tests: the hit mask in visit order and the node's masks */
struct W8Visit {
	uint32_t hm, base, io, to, nv;
};
template <int OCT, uint32_t K, bool UNI>
__device__ __forceinline__ W8Visit w8_visit(const uint32_t (&w)[16], f3 invq, f3 oi, float tl)
{
	f3 s, b;
	w8_frame(w, invq, oi, s, b);
	W8Visit v;
	v.hm = w8_hits<OCT, K>(w, s, b, tl);
	v.base = w[2] >> 8;
	v.io = perm_xor<K>(w[2] & 0xFFu);
	v.to = perm_xor<K>((w[3] >> 8) & 0xFFu);
	v.nv = w[3] & 0xFFu;
	if (UNI) /* keeps the two instances apart (the scalar one reads SGPR operands, no copies) */
		asm volatile("" ::: "memory");
	return v;
}

/* the same visit on the scalar-path copy (every walking lane at the node: SGPR operands) */
template <int OCT, uint32_t K>
__device__ __forceinline__ W8Visit w8_visit_s(const DW8S *n, f3 invq, f3 oi, float tl)
{
	typedef uint32_t u8v __attribute__((ext_vector_type(8)));
	const u8v p0 = *(const __attribute__((address_space(4))) u8v *)n; /* w0..w3, org */
	const uint32_t w1 = p0[1], w2 = p0[2], w3 = p0[3];
	const float org0 = __uint_as_float(p0[4]), org1 = __uint_as_float(p0[5]), org2 = __uint_as_float(p0[6]);
	const f3 s = mk3(ldexpf(invq.x, (int)((w1 >> 16) & 15u)), ldexpf(invq.y, (int)((w1 >> 20) & 15u)),
			 ldexpf(invq.z, (int)((w1 >> 24) & 15u)));
	const f3 b = mk3(fmaf(org0, invq.x, -oi.x), fmaf(org1, invq.y, -oi.y), fmaf(org2, invq.z, -oi.z));
	W8Visit v;
	v.hm = w8_hits_s<OCT, K>(n, w3, s, b, tl);
	v.base = w2 >> 8;
	v.io = perm_xor<K>(w2 & 0xFFu);
	v.to = perm_xor<K>((w3 >> 8) & 0xFFu);
	v.nv = w3 & 0xFFu;
	return v;
}

/* closest-hit visits (k_trace) with entry distances: besides the hit mask, the nearest hit inner
 * child (slot in visit order, or 8 for none) and the least entry distance of the hit inner
 * children (a lower bound for every sibling kept for later: RTX_TRACE_CULL drops a kept group
 * whose bound the closest hit so far has passed) */
struct W8VisitT {
	W8Visit v;
	uint32_t near;
	float tin;
};
template <int OCT, uint32_t K, int C, bool SC>
__device__ __forceinline__ void w8_child_t(const uint32_t *w, f3 s, f3 b, float tl, uint32_t io, uint32_t &hm, uint32_t &near,
					   float &tin)
{
	if (SC && RTX_W8_SKIP && !(((io >> 8) >> C) & 1u)) /* an empty slot (wave-uniform on the scalar path) */
		return;
	float t[6];
	if (SC) { /* w: the scalar-path copy (DW8S) */
		const f8v p = w8s_planes<C>((const DW8S *)w);
		const f2v tx = w8s_axis(p[0], p[1], s.x, b.x), ty = w8s_axis(p[2], p[3], s.y, b.y), tz = w8s_axis(p[4], p[5], s.z, b.z);
		t[0] = tx.x, t[1] = tx.y, t[2] = ty.x, t[3] = ty.y, t[4] = tz.x, t[5] = tz.y;
	} else {
		constexpr int W = C >> 2, B = C & 3;
		t[0] = fmaf(ubyte<B>(w[4 + W]), s.x, b.x), t[1] = fmaf(ubyte<B>(w[6 + W]), s.x, b.x);
		t[2] = fmaf(ubyte<B>(w[8 + W]), s.y, b.y), t[3] = fmaf(ubyte<B>(w[10 + W]), s.y, b.y);
		t[4] = fmaf(ubyte<B>(w[12 + W]), s.z, b.z), t[5] = fmaf(ubyte<B>(w[14 + W]), s.z, b.z);
	}
	float tn;
	const bool h = w8_slab_tn<OCT>(t[0], t[1], t[2], t[3], t[4], t[5], tl, tn) && (OCT != 8 || ((io >> 8) >> C) & 1u);
	hm |= h ? 1u << (C ^ K) : 0u;
	const bool in = h && ((io >> C) & 1u);
	near = (in && tn < tin) ? (uint32_t)(C ^ K) : near;
	tin = (in && tn < tin) ? tn : tin;
}
template <int OCT, uint32_t K, bool SC>
__device__ __forceinline__ void w8_hits_t(const uint32_t *w, f3 s, f3 b, float tl, uint32_t io, W8VisitT &r)
{
	uint32_t hm = 0, near = 8;
	float tin = INFINITY;
	w8_child_t<OCT, K, 0, SC>(w, s, b, tl, io, hm, near, tin);
	w8_child_t<OCT, K, 1, SC>(w, s, b, tl, io, hm, near, tin);
	w8_child_t<OCT, K, 2, SC>(w, s, b, tl, io, hm, near, tin);
	w8_child_t<OCT, K, 3, SC>(w, s, b, tl, io, hm, near, tin);
	w8_child_t<OCT, K, 4, SC>(w, s, b, tl, io, hm, near, tin);
	w8_child_t<OCT, K, 5, SC>(w, s, b, tl, io, hm, near, tin);
	w8_child_t<OCT, K, 6, SC>(w, s, b, tl, io, hm, near, tin);
	w8_child_t<OCT, K, 7, SC>(w, s, b, tl, io, hm, near, tin);
	r.v.hm = hm;
	r.near = near;
	r.tin = tin;
}
/* io argument: inner-child mask (bits 0-7, slot order) | slot mask << 8 (generic octant only) */
template <int OCT, uint32_t K>
__device__ __forceinline__ W8VisitT w8_visit_t(const uint32_t (&w)[16], f3 invq, f3 oi, float tl)
{
	f3 s, b;
	w8_frame(w, invq, oi, s, b);
	W8VisitT r;
	w8_hits_t<OCT, K, false>(w, s, b, tl, (w[2] & 0xFFu) | ((w[3] & 0xFFu) << 8), r);
	r.v.base = w[2] >> 8;
	r.v.io = perm_xor<K>(w[2] & 0xFFu);
	r.v.to = perm_xor<K>((w[3] >> 8) & 0xFFu);
	r.v.nv = w[3] & 0xFFu;
	return r;
}
template <int OCT, uint32_t K>
__device__ __forceinline__ W8VisitT w8_visit_st(const DW8S *n, f3 invq, f3 oi, float tl)
{
	typedef uint32_t u8v __attribute__((ext_vector_type(8)));
	const u8v p0 = *(const __attribute__((address_space(4))) u8v *)n; /* w0..w3, org */
	const uint32_t w1 = p0[1], w2 = p0[2], w3 = p0[3];
	const f3 s = mk3(ldexpf(invq.x, (int)((w1 >> 16) & 15u)), ldexpf(invq.y, (int)((w1 >> 20) & 15u)),
			 ldexpf(invq.z, (int)((w1 >> 24) & 15u)));
	const f3 b = mk3(fmaf(__uint_as_float(p0[4]), invq.x, -oi.x), fmaf(__uint_as_float(p0[5]), invq.y, -oi.y),
			 fmaf(__uint_as_float(p0[6]), invq.z, -oi.z));
	W8VisitT r;
	w8_hits_t<OCT, K, true>((const uint32_t *)n, s, b, tl, (w2 & 0xFFu) | ((w3 & 0xFFu) << 8), r);
	r.v.base = w2 >> 8;
	r.v.io = perm_xor<K>(w2 & 0xFFu);
	r.v.to = perm_xor<K>((w3 >> 8) & 0xFFu);
	r.v.nv = w3 & 0xFFu;
	return r;
}

#endif
