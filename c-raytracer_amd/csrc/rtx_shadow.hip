/*
 * k_shadow: direct lighting of every shade point (render.c:170-229) on gfx950.
 *
 * Shadow rays are 95.9-99.6 % of the reference's rays (is_light_blocked,
 * render.c:126-134 -> object.c:183-197 + accel.c:360-387).  Each (shade point,
 * light sample) pair is one lane: the lane samples its light point, tests the
 * unbound planes, walks the BVH for any opaque blocker (multiplying the
 * transmittance of transparent ones), then evaluates Phong / Blinn.
 *
 * The walk: every lane walks its own shadow ray over the 8-wide compressed BVH
 * (rtx_device.h DW8, shadow_walk8): one 64-byte node per step, eight box tests
 * per memory round trip, pending siblings as (base, slot mask) groups in a
 * register, an LDS lane stack and HBM below it (any depth).  A step whose walking
 * lanes share one node reads it through the scalar cache; other steps read the
 * tree's top three levels from the workgroup's LDS copy (DScene.w8top) and the
 * rest from memory.  Small scenes (the whole threaded BVH2 fits the LDS top copy)
 * may walk the threaded BVH2 instead (shadow_walk: one 16-byte record per step,
 * no stack, read from LDS), and tiny ones test their few objects one by one
 * (DScene.lin, no walk).  The walks test boxes in the tree's frame (DScene.tf:
 * the rotation the uploader chose for the leaf boxes) and primitives in world
 * space.  The emitter and material records of a one-point packet are read
 * through the scalar cache.
 *
 * Scheduling: persistent workgroups; each wave takes `per_wave` shade points at
 * a time from a global queue in Morton order of their position (rtx_sort.hip),
 * so the resident waves share one compact region of the tree in L2.  A point's
 * samples fill whole power-of-two lane slots and its sum runs inside one wave
 * in lane order, so its result does not depend on which wave takes it.
 */
#include <hip/hip_runtime.h>
#include <float.h>
#include <stdlib.h>

#include "rtx_kat.h"
#include "rtx_quant.h"
#include "rtx_wave.h"
#include "rtx_w8.h"

#ifndef RTX_DEBUG_NOWALK
#define RTX_DEBUG_NOWALK 0 /* measurement only: skip the BVH walk (everything else in k_shadow stays) */
#endif
#ifndef RTX_DEBUG_NOLEAF
#define RTX_DEBUG_NOLEAF 0 /* measurement only: the walk tests no leaf (wrong images; the cost of the leaf tests) */
#endif
#ifndef RTX_SH_FASTSQRT
#define RTX_SH_FASTSQRT 1 /* the shadow ray's length from v_sqrt_f32 (1 ulp) instead of the correctly rounded sequence */
#endif
#ifndef RTX_SH_OCT
#define RTX_SH_OCT 1 /* walks specialised on a wave-uniform direction octant */
#endif
#ifndef RTX_SH_FASTPOW
#define RTX_SH_FASTPOW 1 /* specular powf from v_log_f32 / v_exp_f32 (sh_pow) */
#endif
#ifndef RTX_SH_FARLIN
#define RTX_SH_FARLIN 0 /* far shade points: objects tested one by one are culled by their world boxes first */
#endif
#ifndef RTX_SH_SPILL_UNI
#define RTX_SH_SPILL_UNI 1 /* the lane-stack spill area addressed from a wave-uniform base */
#endif
#ifndef RTX_SH_RECAFTER
#define RTX_SH_RECAFTER 1 /* several points per packet: the record address formed again after the walk */
#endif
#ifndef RTX_SH_SPUNI
#define RTX_SH_SPUNI 1 /* >= 64 lights: the shade-point record through scalar loads */
#endif
#ifndef RTX_SHADOW_OCC_DEFAULT
#define RTX_SHADOW_OCC_DEFAULT 8 /* waves per SIMD the walk is register-capped for */
#endif
#ifndef RTX_SHADOW_OCC_SLOT
#define RTX_SHADOW_OCC_SLOT RTX_SHADOW_OCC_DEFAULT /* the same for the lane-slot kernel */
#endif
/* light_point (object.c:293-304) in k_shadow: a sphere light's inclination and azimuth are
 * u * 2pi, so their sines and cosines come from the revolution-scaled v_sin_f32 / v_cos_f32
 * instead of OCML's range-reduced sinf / cosf.  KAT: RTX_KAT_SPH_LIGHT_SH, <= 4e-6 of the
 * radius.  RTX_SH_FASTTRIG=0 restores the exact light_point. */
#ifndef RTX_SH_FASTTRIG
#define RTX_SH_FASTTRIG 1
#endif
/* 1/x in light sampling and attenuation: v_rcp_f32 (1 ulp) instead of the IEEE division
 * sequence (the closest-hit path keeps IEEE division).  RTX_SH_FASTDIV=0 restores it. */
#ifndef RTX_SH_FASTDIV
#define RTX_SH_FASTDIV 1
#endif

/* ------------------------------------------------------------------------ */
/* intersection tests of the any-hit walk                                   */
/* ------------------------------------------------------------------------ */
/* The slab test (accel.c:112-158) against a DQNode box, in the quantisation frame: the ray is
 * transformed once per walk (o' = (o - qo) * qs, inv' = inv / qs, oi = o' * inv'), so
 * t = q * inv' - oi is the world ray parameter, with the 16-bit plane coordinates converted by
 * one SDWA v_cvt_f32_u32 each.  OCT < 8: every live lane's direction lies in octant OCT (bit a
 * set: inv[a] >= 0), so each axis' entry plane is known at compile time.  The boxes are
 * widened by one quantisation step on both sides, far more than the transform's rounding, so
 * the test is conservative (KAT: RTX_KAT_BOX_Q). */
template <int OCT> __device__ __forceinline__ bool box_hit_q(uint4 n, f3 oi, f3 inv, float tlim, float &tn_out);
template <int OCT> __device__ __forceinline__ bool box_hit_q(uint4 n, f3 oi, f3 inv, float tlim)
{
	float tn;
	return box_hit_q<OCT>(n, oi, inv, tlim, tn);
}
template <int OCT> __device__ __forceinline__ bool box_hit_q(uint4 n, f3 oi, f3 inv, float tlim, float &tn_out)
{
	const float tx0 = fmaf((float)(n.x & 0xFFFFu), inv.x, -oi.x), tx1 = fmaf((float)(n.x >> 16), inv.x, -oi.x);
	const float ty0 = fmaf((float)(n.y & 0xFFFFu), inv.y, -oi.y), ty1 = fmaf((float)(n.y >> 16), inv.y, -oi.y);
	const float tz0 = fmaf((float)(n.z & 0xFFFFu), inv.z, -oi.z), tz1 = fmaf((float)(n.z >> 16), inv.z, -oi.z);
	if (OCT == 8) {
		const float tn = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fmaxf(fminf(tz0, tz1), 0.f));
		const float tf = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fminf(fmaxf(tz0, tz1), tlim));
		tn_out = tn;
		return tn <= tf;
	}
	const float nx = (OCT & 1) ? tx0 : tx1, fx = (OCT & 1) ? tx1 : tx0;
	const float ny = (OCT & 2) ? ty0 : ty1, fy = (OCT & 2) ? ty1 : ty0;
	const float nz = (OCT & 4) ? tz0 : tz1, fz = (OCT & 4) ? tz1 : tz0;
	const float tn = fmaxf(fmaxf(nx, ny), fmaxf(nz, 0.f));
	/* min with the segment end in asm: tlim is loop-carried and the compiler would
	 * canonicalise it before every fminf; no NaN reaches here */
	float tf = fminf(fminf(fx, fy), fz);
	asm("v_min_f32 %0, %0, %1" : "+v"(tf) : "v"(tlim));
	tn_out = tn;
	return tn <= tf;
}

/* moller_trumbore (object.c:422-441) as a branch-free any-hit test on (eps, tlim), with the
 * same accept set for finite inputs:
 *   reject |a| < eps;  reject u < 0, v < 0, u + v > 1 (u > 1 is implied);  accept eps < t < tlim.
 * Whenever t is finite, f = 1/a and u, v are finite too, so the three sign conditions fold into
 * one max3 compare and the t window into one min compare (a NaN or infinite t fails it).
 * Products are fused and 1/a comes from v_rcp_f32 (1 ulp): only hit/miss decisions at exact
 * edges can differ from the IEEE test (KAT: RTX_KAT_ANY_TRI). */
__device__ __forceinline__ f3 cross3_fma(f3 a, f3 b)
{
	return mk3(fmaf(a.y, b.z, -a.z * b.y), fmaf(a.z, b.x, -a.x * b.z), fmaf(a.x, b.y, -a.y * b.x));
}
__device__ __forceinline__ float dot3_fma(f3 a, f3 b) { return fmaf(a.x, b.x, fmaf(a.y, b.y, a.z * b.z)); }

__device__ __forceinline__ bool any_tri(f3 v0, f3 e1, f3 e2, f3 o, f3 d, float eps, float tlim)
{
	const f3 h = cross3_fma(d, e2);
	const float a = dot3_fma(e1, h);
	const float f = __builtin_amdgcn_rcpf(a);
	const f3 s = sub3(o, v0);
	const float u = f * dot3_fma(s, h);
	const f3 q = cross3_fma(s, e1);
	const float v = f * dot3_fma(d, q);
	const float t = f * dot3_fma(e2, q);
	const float out = fmaxf(fmaxf(-u, -v), (u + v) - 1.f); /* > 0: outside the triangle */
	return ((int)(fabsf(a) >= eps) & (int)(out <= 0.f) & (int)(fminf(t - eps, tlim - t) > 0.f)) != 0;
}

/* ------------------------------------------------------------------------ */
/* one shadow ray per lane                                                  */
/* ------------------------------------------------------------------------ */
struct ShadowCount {
	u64 boxes;     /* box tests (records stepped through), summed over lanes */
	u64 gboxes;    /* ... of which from the DQNode array (not the LDS top) */
	u64 tris, sph; /* primitive tests */
	u64 pln;       /* plane tests */
	u64 steps;     /* walk-loop iterations of the waves (a wave runs until its longest ray ends) */
	u64 walks;     /* wave walks (64 rays each) */
	u64 lrounds;   /* 8-wide walk: wave iterations of the leaf loops (immediate and deferred) */
	u64 unif;      /* 8-wide walk: wave steps with one node for all walking lanes (scalar path) */
	u64 far;       /* rays from far shade points, walked from the light end (RTX_SP_FAR) */
	u64 spills;    /* 8-wide walk: lane-stack pushes beyond the LDS entries (to DScene.w8spill in HBM) */
	u64 clear;     /* rays of packets the cone cull let skip the walk (cone_clear) */
};

/* one primitive record (a, b, c = its first 48 bytes) against this lane's shadow ray
 * (accel.c:362-373): the target emitter skipped; transparent hit -> li *= kt; opaque hit ->
 * true (blocked) */
template <bool COUNT>
__device__ __forceinline__ bool shadow_prim(float4 a, float4 b, float4 c, const DMaterial *__restrict__ mats, f3 o, f3 d,
					    float tl, uint32_t emit_obj, f3 &li, uint32_t &ntri, uint32_t &nsph)
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

/* every primitive of the leaf with ref L, in order, its records REC bytes apart from p (64-byte
 * DPrims for the BVH2 walk, 48-byte triangle records for the wide walk); true at the first
 * opaque hit */
template <bool COUNT, uint32_t REC>
__device__ __forceinline__ bool shadow_leaf(uint32_t L, const char *__restrict__ p, const DMaterial *__restrict__ mats, f3 o,
					    f3 d, float tl, uint32_t emit_obj, f3 &li, uint32_t &ntri, uint32_t &nsph)
{
	const uint32_t cnt = (L & RTX_REF_CNT) + 1;
	for (uint32_t k = 0; k < cnt; k++) {
		const char *pr = p + k * REC;
		if (shadow_prim<COUNT>(ldg4(pr, 0), ldg4(pr, 16), ldg4(pr, 32), mats, o, d, tl, emit_obj, li, ntri, nsph))
			return true;
	}
	return false;
}

/* the trees of the shadow walks and their 16-bit frame (rtx_device.h DQNode, DW8) */
struct QBvh {
	const DQNode *q;
	f3 qo, qs, qsi; /* qsi = 1 / qs (IEEE, per component) */
	const uint4 *top;     /* the workgroup's LDS copy of the top records */
	const uint32_t *tend; /* ... and of the cut records' range ends */
	uint32_t nt;          /* top records */
	const DW8 *w8;        /* the 8-wide BVH (rtx_device.h DW8), WALK_W8 */
	const DW8S *w8s;      /* ... its nodes' scalar-path copies */
	const uint4 *t8;      /* the workgroup's LDS copy of its entries [0, nt8) (top levels) */
	uint32_t nt8;
	uint32_t *spill;      /* the lane-stack entries from lstk on, [entry][grid lane] (w8_spill_at) */
	uint32_t wv;          /* this wave's index in its workgroup */
	uint32_t lstk;        /* lane-stack entries in LDS (<= RTX_W8_STACK) */
	lds_u32 *stk;         /* the wave's LDS stacks of sibling groups: lane l's entry k at stk[k * WAVE + l]
	                       * (RTX_W8_LANEADDR 0: this lane's, entry k at stk[k * WAVE]) */
	lds_u32 *tq;          /* WALK_W8: the LDS queues of deferred leaf groups, likewise */
	bool sph;             /* WALK_W8: the tree holds spheres (DScene.w8sph) */
};

/* the shadow walks k_shadow instantiates */
enum { WALK_BVH2 = 0, WALK_W8 = 2 }; /* the RTX_WALK_* values */

/* is_light_blocked's BVH part (accel.c:360-387) for this lane's ray.  The walk starts in the
 * workgroup's LDS copy of the tree's top levels: a cut record whose box is hit hands the lane
 * to the DQNode array for the index range of its children's subtrees, and the lane returns to
 * the top copy at the next top record when the range ends.  tl < 0 on entry: inactive lane.
 * On an opaque hit tl becomes -1. */
template <bool COUNT, int OCT>
__device__ __forceinline__ void shadow_walk(const QBvh &Q, const char *__restrict__ recs, const DMaterial *__restrict__ mats,
					    f3 o, f3 d, f3 ob, f3 inv, float &tl, uint32_t emit_obj, f3 &li, ShadowCount &sc)
{
	const f3 invq = mk3(inv.x * Q.qsi.x, inv.y * Q.qsi.y, inv.z * Q.qsi.z);
	const f3 oq = mk3((ob.x - Q.qo.x) * Q.qs.x, (ob.y - Q.qo.y) * Q.qs.y, (ob.z - Q.qo.z) * Q.qs.z);
	const f3 oi = mul3v(oq, invq);
	const uint32_t nt = Q.nt;
	uint32_t t = tl >= 0.f ? 0u : nt, g = 0, ge = 0;
	uint32_t nbox = 0, nglob = 0, ntri = 0, nsph = 0, nstep = 0;
	while (t < nt || g < ge) {
		const bool ing = g < ge;
		uint4 nd;
		if (ing)
			nd = ldg4u(Q.q + g);
		else
			nd = lds4u(Q.top + t);
		if (COUNT) {
			nbox++;
			nglob += ing ? 1u : 0u;
		}
		const bool hit = box_hit_q<OCT>(nd, oi, invq, tl);
		const uint32_t L = nd.w;
		if (L & RTX_REF_LEAF) {
			if (ing)
				g++;
			else
				t++;
			if (hit && shadow_leaf<COUNT, sizeof(DPrim)>(L, recs + (L & RTX_REF_OFF), mats, o, d, tl, emit_obj, li, ntri, nsph)) {
				tl = -1.f;
				t = nt;
				ge = 0;
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
	if (COUNT)
		nstep = nbox;
	if (COUNT) {
		uint32_t a = nbox, b = ntri, c = nsph, gq = nglob;
#pragma unroll
		for (int s = 32; s > 0; s >>= 1) {
			a += __shfl_xor(a, s, WAVE);
			b += __shfl_xor(b, s, WAVE);
			c += __shfl_xor(c, s, WAVE);
			gq += __shfl_xor(gq, s, WAVE);
			nstep = max(nstep, (uint32_t)__shfl_xor(nstep, s, WAVE));
		}
		sc.boxes += uni(a);
		sc.gboxes += uni(gq);
		sc.tris += uni(b);
		sc.sph += uni(c);
		sc.steps += uni(nstep);
		sc.walks++;
	}
}

/* is_light_blocked's BVH part (accel.c:360-387) over the 8-wide BVH (rtx_device.h DW8): one
 * 64-byte node per step (four 16-byte loads, or its DW8S copy through scalar loads when every live lane is at
 * the node), eight box tests.  Hit children are taken in the octant's visit order (slot p ^ K):
 *  - opaque leaf slots are tested at once (an opaque hit ends the ray);
 *  - transparent leaf slots (tmask) can only multiply the transmittance, so their tests are
 *    deferred: the lane keeps them as leaf groups (base << 8 | mask) in a register and an LDS
 *    queue of RTX_W8_TQ, and the wave runs a round of deferred tests only when at least
 *    RTX_W8_DEFER lanes hold some (or a queue is full, or no lane has node work left), so a
 *    round tests many lanes' primitives instead of a few;
 *  - the first hit inner child is visited next and the rest are kept as one group in a
 *    register, the older groups in the lane's LDS stack (entries from Q.lstk on in HBM,
 *    Q.spill), at most one per level, so any depth walks.
 * tl < 0 on entry: inactive lane.  On an opaque hit tl becomes -1. */
#ifndef RTX_SH_OWNINC
#define RTX_SH_OWNINC 1 /* a slot's point found from the lane's previous one (off[] is nondecreasing) */
#endif
#ifndef RTX_SH_SLOTFOLD
#define RTX_SH_SLOTFOLD 1 /* slot sums folded by lane 0 from LDS (k_shadow's several-points-per-packet path) */
#endif
#ifndef RTX_W8_TOP
#define RTX_W8_TOP 1 /* divergent steps read the tree's top levels (DScene.w8top entries) from an LDS copy */
#endif
#ifndef RTX_W8_TQ
#define RTX_W8_TQ 4 /* deferred leaf groups per lane in LDS (besides the one in a register) */
#endif
#ifndef RTX_W8_TRIONLY
#define RTX_W8_TRIONLY 1 /* leaf tests of a tree without spheres skip the sphere case (DScene.w8sph) */
#endif
#ifndef RTX_W8_LANEADDR
#define RTX_W8_LANEADDR 2 /* the lane-stack / queue LDS addresses formed from lane_id() at each access (no per-lane
                           * address register live across the walk, which the allocator spilled to scratch) */
#endif
#define W8_LN (LA ? lane_id() : 0u)
#ifndef RTX_W8_LEAF2
#define RTX_W8_LEAF2 1 /* a round of opaque leaf tests takes two of a lane's hit leaf slots */
#endif
#ifndef RTX_W8_DEFER2
#define RTX_W8_DEFER2 1 /* a round of deferred transparent-leaf tests takes two of a lane's queued leaves */
#endif
#ifndef RTX_W8_DEFER
#define RTX_W8_DEFER 64 /* lanes holding deferred leaf tests that trigger a round of them (16 / 32 / 48 / 64: 613 / 601 / 598 / 594 ms) */
#endif
/* a deferred leaf test: the transparent primitive at entry pr (rtx_device.h DW8 leaf entry,
 * whose 4th float4 holds its material's kt) against this lane's shadow ray; a hit multiplies
 * the transmittance (accel.c:370-377) */
template <bool COUNT, bool SPH>
__device__ __forceinline__ void w8_defer_test(const char *pr, f3 o, f3 d, float tl, f3 &li, uint32_t &ntri, uint32_t &nsph)
{
	const float4 a = ldg4(pr, 0), b = ldg4(pr, 16), c = ldg4(pr, 32);
	bool h;
	if (SPH && (__float_as_uint(c.w) >> 24) == RTX_SPHERE) {
		if (COUNT)
			nsph++;
		float t = 0.f;
		h = hit_sphere(mk3(a.x, a.y, a.z), b.x, o, d, a.w, t) && t < tl;
	} else {
		if (COUNT)
			ntri++;
		h = any_tri(mk3(a.x, a.y, a.z), mk3(b.x, b.y, b.z), mk3(c.x, c.y, c.z), o, d, a.w, tl);
	}
	if (h) {
		const float4 kt = ldg4(pr, 48);
		li = mul3v(li, mk3(kt.x, kt.y, kt.z));
	}
}

/* an opaque leaf test: does the primitive at entry pr block this lane's shadow ray?  (no
 * emitter or transparency cases: the 8-wide tree marks its leaves when built from host records).
 * SPH false: the tree holds no spheres (DScene.w8sph), the test is the triangle's alone */
template <bool COUNT, bool SPH>
__device__ __forceinline__ bool w8_opaque_test(const char *pr, f3 o, f3 d, float tl, uint32_t &ntri, uint32_t &nsph)
{
	const float4 a = ldg4(pr, 0), b = ldg4(pr, 16), c = ldg4(pr, 32);
	if (SPH && (__float_as_uint(c.w) >> 24) == RTX_SPHERE) {
		if (COUNT)
			nsph++;
		float t = 0.f;
		return hit_sphere(mk3(a.x, a.y, a.z), b.x, o, d, a.w, t) && t < tl;
	}
	if (COUNT)
		ntri++;
	return any_tri(mk3(a.x, a.y, a.z), mk3(b.x, b.y, b.z), mk3(c.x, c.y, c.z), o, d, a.w, tl);
}

/* lane-stack entry k (>= Q.lstk) of this lane in HBM, [entry][grid lane]: its address formed where
 * it is used, from the launch's constant block size, the workgroup's and wave's indices and
 * lane_id() (volatile asm, so nothing of it is hoisted into the packet's set-up: round 5's
 * per-lane spill pointer and round 6's first stride / lane-offset pair were computed per packet
 * and spilled to scratch there, one 12-byte scratch store per lane and packet) */
__device__ __forceinline__ uint32_t *w8_spill_at(const QBvh &Q, uint32_t k)
{
	constexpr uint32_t B = WAVE * RTX_SH_NW; /* k_shadow's block size (rtx_launch_shadow) */
	return Q.spill + ((size_t)(k - Q.lstk) * ((size_t)gridDim.x * B) + (size_t)blockIdx.x * B + Q.wv * WAVE + lane_id());
}

/* the visit order of hit children: plain slot order (RTX_W8_SORDER 0), front to back from the
 * shade point (1), or front to back from the light (2) */
template <int OCT> __device__ __forceinline__ constexpr uint32_t w8_sorder()
{
	return (OCT == 8 || !RTX_W8_SORDER) ? 0u : RTX_W8_SORDER == 2 ? ((uint32_t)OCT & 7u) : (~(uint32_t)OCT & 7u);
}

/* one lane's 8-wide any-hit walk: the node it is at (RTX_NONE: no node work), the kept sibling
 * group and the stack depth below it, the deferred transparent-leaf group and the queue depth */
struct W8Walk {
	uint32_t node, grp, sp, tgrp, tn;
};
/* the walk's counters (COUNT instances) */
struct W8Ctr {
	uint32_t nbox, ntri, nsph, nstep, nlr, nun, nspill;
};

/* this lane's opaque leaf hits lm (visit order) in the block at base, tested in turn: does one
 * block the ray?  (the wave's lanes in step, a lane leaving at its first blocking hit) */
template <bool COUNT, bool SPH, uint32_t K>
__device__ __forceinline__ bool w8_opaque_leaves(const DW8 *w8, uint32_t lm, uint32_t base, f3 o, f3 d, float tl, W8Ctr &c)
{
	while (lm) {
		const uint32_t p = __builtin_ctz(lm);
		lm &= lm - 1;
		if (RTX_W8_LEAF2) {
			/* two of the lane's hit leaves per round (the same tests in the same order, half the
			 * rounds: a Menger face's two triangles share a box in the rotated frame, so a lane that
			 * meets one meets both) */
			const bool two = lm != 0;
			const uint32_t q = two ? __builtin_ctz(lm) : p;
			lm &= lm - 1;
			if (w8_opaque_test<COUNT, SPH>((const char *)(w8 + base + (p ^ K)), o, d, tl, c.ntri, c.nsph))
				return true;
			if (two && w8_opaque_test<COUNT, SPH>((const char *)(w8 + base + (q ^ K)), o, d, tl, c.ntri, c.nsph))
				return true;
			continue;
		}
		if (w8_opaque_test<COUNT, SPH>((const char *)(w8 + base + (p ^ K)), o, d, tl, c.ntri, c.nsph))
			return true;
	}
	return false;
}

/* One iteration of the 8-wide any-hit walk for the wave: a round of deferred transparent-leaf
 * tests, or one node step with its opaque leaf tests (see shadow_walk8).  wk / hd: this lane has
 * node work / deferred tests; walking / holding: their ballots (at least one lane has one).  o / d: the
 * world ray; invq / oi: its inverse direction and origin term in the tree's 16-bit frame. */
template <bool COUNT, int OCT, bool LA>
__device__ __forceinline__ void w8_iter(const QBvh &Q, f3 o, f3 d, f3 invq, f3 oi, float &tl, f3 &li, W8Walk &w, W8Ctr &c,
					bool wk, bool hd, u64 walking, u64 holding)
{
	constexpr uint32_t K = w8_sorder<OCT>();
	lds_u32 *stk = Q.stk, *tq = Q.tq;
	if (!walking || popc64(holding) >= RTX_W8_DEFER || ballot(w.tn == RTX_W8_TQ)) {
		/* a round of deferred transparent-leaf tests */
		if (COUNT)
			c.nlr++;
		if (hd) {
			const char *pr = (const char *)(Q.w8 + (w.tgrp >> 8) + (__builtin_ctz(w.tgrp) ^ K));
			w.tgrp &= w.tgrp - 1;
			if (!(w.tgrp & 0xFFu))
				w.tgrp = w.tn ? tq[--w.tn * WAVE + W8_LN] : 0u;
			/* RTX_W8_DEFER2: the lane's next queued leaf in the same round (the transmittance
			 * products in the same order) */
			const char *pr2 = nullptr;
			if (RTX_W8_DEFER2 && w.tgrp) {
				pr2 = (const char *)(Q.w8 + (w.tgrp >> 8) + (__builtin_ctz(w.tgrp) ^ K));
				w.tgrp &= w.tgrp - 1;
				if (!(w.tgrp & 0xFFu))
					w.tgrp = w.tn ? tq[--w.tn * WAVE + W8_LN] : 0u;
			}
			if (!RTX_W8_TRIONLY || Q.sph) {
				w8_defer_test<COUNT, true>(pr, o, d, tl, li, c.ntri, c.nsph);
				if (RTX_W8_DEFER2 && pr2)
					w8_defer_test<COUNT, true>(pr2, o, d, tl, li, c.ntri, c.nsph);
			} else {
				w8_defer_test<COUNT, false>(pr, o, d, tl, li, c.ntri, c.nsph);
				if (RTX_W8_DEFER2 && pr2)
					w8_defer_test<COUNT, false>(pr2, o, d, tl, li, c.ntri, c.nsph);
			}
		}
		return;
	}
	uint32_t lm = 0, base = 0; /* this step's opaque leaf hits (visit order) and their block */
	if (wk) {
		const uint32_t un = uni(w.node);
		W8Visit v;
		if (!ballot(w.node != un)) {
			/* every walking lane is at one node: its scalar-path copy through the scalar cache,
			 * the planes as SGPR float operands (no vector-memory address / data cycles) */
			v = w8_visit_s<OCT, K>(Q.w8s + (size_t)un, invq, oi, tl);
		} else {
			uint32_t wd[16];
			if (w.node < Q.nt8) { /* a top-level node: the workgroup's LDS copy (no texture-path traffic) */
#pragma unroll
				for (int k = 0; k < 4; k++) {
					const uint4 x = lds4u(Q.t8 + 4 * w.node + k);
					wd[4 * k] = x.x;
					wd[4 * k + 1] = x.y;
					wd[4 * k + 2] = x.z;
					wd[4 * k + 3] = x.w;
				}
			} else {
				const DW8 *N = Q.w8 + (size_t)w.node;
#pragma unroll
				for (int k = 0; k < 4; k++) {
					const uint4 x = ldg4u((const uint32_t *)N + 4 * k);
					wd[4 * k] = x.x;
					wd[4 * k + 1] = x.y;
					wd[4 * k + 2] = x.z;
					wd[4 * k + 3] = x.w;
				}
			}
			v = w8_visit<OCT, K, false>(wd, invq, oi, tl);
		}
		const uint32_t hm = v.hm;
		base = v.base;
		lm = RTX_DEBUG_NOLEAF ? 0u : hm & ~v.io & ~v.to;
		uint32_t im = hm & v.io;
		const uint32_t dm = RTX_DEBUG_NOLEAF ? 0u : hm & v.to;
		if (COUNT) {
			c.nstep++;
			c.nbox += popc64(v.nv);
			c.nun += ballot(w.node != uni(w.node)) ? 0u : 1u;
		}
		if (dm) { /* transparent leaves: deferred */
			const uint32_t g = (base << 8) | dm;
			if (w.tgrp)
				tq[w.tn++ * WAVE + W8_LN] = g;
			else
				w.tgrp = g;
		}
		/* the next node (a lane the opaque leaves below block drops it again) */
		if (im) {
			w.node = base + (__builtin_ctz(im) ^ K);
			im &= im - 1;
			if (im) {
				if (w.grp) {
					if (w.sp < Q.lstk)
						stk[w.sp * WAVE + W8_LN] = w.grp;
					else {
						*gptrw(w8_spill_at(Q, w.sp)) = w.grp;
						if (COUNT)
							c.nspill++;
					}
					w.sp++;
				}
				w.grp = (base << 8) | im;
			}
		} else if (w.grp) {
			w.node = (w.grp >> 8) + (__builtin_ctz(w.grp) ^ K);
			w.grp &= w.grp - 1;
			if (!(w.grp & 0xFFu)) {
				w.grp = 0;
				if (w.sp) {
					w.sp--;
					w.grp = w.sp < Q.lstk ? stk[w.sp * WAVE + W8_LN]
							      : *gptr(w8_spill_at(Q, w.sp));
				}
			}
		} else {
			w.node = RTX_NONE;
		}
	}
	/* opaque leaves, at once (an opaque hit ends the ray): the tree marks every leaf slot (built
	 * from the primitive records, emitters left out), each lane tests its own.  (Dealing the
	 * wave's tests over its lanes with ds_permute, one round for all, measured slower on scene6:
	 * 2834 vs 2806 ms, every dealt job tested without the early break) */
	if (!ballot(lm != 0))
		return;
	if (COUNT) {
		uint32_t r = 0;
		for (uint32_t m = lm;; m &= m - 1) {
			if (!ballot(m != 0))
				break;
			if (RTX_W8_LEAF2)
				m &= m - 1;
			r++;
		}
		c.nlr += r;
	}
	const bool blocked = (!RTX_W8_TRIONLY || Q.sph) ? w8_opaque_leaves<COUNT, true, K>(Q.w8, lm, base, o, d, tl, c)
							  : w8_opaque_leaves<COUNT, false, K>(Q.w8, lm, base, o, d, tl, c);
	if (blocked) { /* the queue too: a full queue left behind would keep the wave in deferred rounds */
		tl = -1.f;
		w.node = RTX_NONE;
		w.tgrp = 0;
		w.tn = 0;
	}
}

/* the walk's counters summed over the wave into sc (walks: wave walks of 64 lane slots) */
template <bool COUNT> __device__ __forceinline__ void w8_count(W8Ctr c, ShadowCount &sc, uint32_t walks)
{
	if (!COUNT)
		return;
	uint32_t a = c.nbox, bb = c.ntri, cc = c.nsph, nstep = c.nstep, nun = c.nun, nlr = c.nlr, nsp = c.nspill;
#pragma unroll
	for (int k = 32; k > 0; k >>= 1) {
		a += __shfl_xor(a, k, WAVE);
		nsp += __shfl_xor(nsp, k, WAVE);
		bb += __shfl_xor(bb, k, WAVE);
		cc += __shfl_xor(cc, k, WAVE);
		nstep = max(nstep, (uint32_t)__shfl_xor(nstep, k, WAVE));
		nun = max(nun, (uint32_t)__shfl_xor(nun, k, WAVE));
		nlr = max(nlr, (uint32_t)__shfl_xor(nlr, k, WAVE));
	}
	sc.boxes += uni(a);
	sc.gboxes += uni(a);
	sc.lrounds += uni(nlr);
	sc.unif += uni(nun);
	sc.spills += uni(nsp);
	sc.tris += uni(bb);
	sc.sph += uni(cc);
	sc.steps += uni(nstep);
	sc.walks += walks;
}

template <bool COUNT, int OCT, bool LA>
__device__ __forceinline__ void shadow_walk8(const QBvh &Q, const DMaterial *__restrict__ mats, f3 o, f3 d, f3 ob, f3 inv,
					     float &tl, uint32_t emit_obj, f3 &li, ShadowCount &sc)
{
	/* the ray in the tree's 16-bit frame: ob / inv are its origin and inverse direction in the
	 * tree's rotated frame (shadow_query), o / d the world ray the primitives are tested with */
	const f3 invq = mk3(inv.x * Q.qsi.x, inv.y * Q.qsi.y, inv.z * Q.qsi.z);
	const f3 oq = mk3((ob.x - Q.qo.x) * Q.qs.x, (ob.y - Q.qo.y) * Q.qs.y, (ob.z - Q.qo.z) * Q.qs.z);
	const f3 oi = mul3v(oq, invq);
	W8Walk w = { tl >= 0.f ? 0u : RTX_NONE, 0u, 0u, 0u, 0u };
	W8Ctr c = { 0u, 0u, 0u, 0u, 0u, 0u, 0u };
	for (;;) {
		/* the lane's two conditions once, as lane masks the branches below reuse */
		const bool wk = w.node != RTX_NONE, hd = w.tgrp != 0;
		const u64 walking = ballot(wk);
		const u64 holding = ballot(hd);
		if (!(walking | holding))
			break;
		w8_iter<COUNT, OCT, LA>(Q, o, d, invq, oi, tl, li, w, c, wk, hd, walking, holding);
	}
	w8_count<COUNT>(c, sc, 1u);
}

/* is_light_blocked (render.c:126-134): planes first (unbound_objects_is_light_blocked,
 * object.c:183-197), then the BVH walk, specialised on the direction octant when every live
 * lane shares it.  Returns the lane's blocked flag; li carries the transmittance product. */
/* hit_plane(...) && t < dist (object.c:473-488 and is_light_blocked's plane test) with the
 * quotient t = num / a as num * v_rcp_f32(a) (within 2 ulp of the IEEE quotient, like the
 * light points of RTX_SH_FASTTRIG): the decisions differ from the IEEE test only for a t within
 * 2 ulp of the plane's epsilon or of the light sample's distance */
#ifndef RTX_SH_PLANE_RCP
#define RTX_SH_PLANE_RCP 1
#endif
__device__ __forceinline__ bool plane_blocks(f3 n, float dd, f3 o, f3 d, float eps, float dist)
{
	float t;
	if (!RTX_SH_PLANE_RCP)
		return hit_plane(n, dd, o, d, eps, t) && t < dist;
	const float a = dot3(n, d);
	if (!(fabsf(a) >= eps)) /* hit_plane's fabsf(a) < eps (a NaN misses there too) */
		return false;
	t = (dd - dot3(n, o)) * __builtin_amdgcn_rcpf(a);
	return t > eps && t < dist;
}

template <bool COUNT, int WALK, bool LA>
__device__ __forceinline__ bool shadow_query(const QBvh &Q, const char *__restrict__ recs, const DMaterial *__restrict__ mats,
					     const DPlane *__restrict__ planes, uint32_t num_planes, const DEmitter *__restrict__ lin,
					     uint32_t num_lin, bool have_tree, const DTreeFrame &tf, bool act, bool far, f3 o, f3 d,
					     float dist, uint32_t emit_obj, f3 &li, ShadowCount &sc)
{
	float tl = act ? dist : -1.f;
	for (uint32_t i = 0; i < num_planes; i++) { /* plane records are wave-uniform: s_load */
		const auto *pl = cptr(planes) + i;
		const bool h = plane_blocks(mk3(pl->n[0], pl->n[1], pl->n[2]), pl->d, o, d, pl->eps, dist) && tl >= 0.f;
		if (pl->transparent) {
			if (h)
				li = mul3v(li, mk3(pl->kt[0], pl->kt[1], pl->kt[2]));
		} else if (h) {
			tl = -1.f;
		}
	}
	/* objects tested one by one like the planes, records wave-uniform (s_load): the emitters other
	 * than the one sampled when the 8-wide tree leaves them out (rtx_device.h DW8), or every bounded
	 * object of a tiny scene (DScene.lin), in object order */
	for (uint32_t i = 0; i < num_lin; i++) {
		const auto *e = cptr(lin) + i;
		if (e->obj == emit_obj || !(tl >= 0.f))
			continue;
		/* a far shade point: the object's world box first, from the light end like the walk */
		if (RTX_SH_FARLIN == 1 && far &&
		    !world_box_at(e->wlo[0], e->whi[0], e->wlo[1], e->whi[1], e->wlo[2], e->whi[2], o, d, dist, -1.f, dist))
			continue;
		bool h;
		if (e->type == RTX_SPHERE) {
			float t = 0.f;
			h = (RTX_SH_FARLIN != 2 || !far ||
			     world_box_at(e->wlo[0], e->whi[0], e->wlo[1], e->whi[1], e->wlo[2], e->whi[2], o, d, 0.f, 1.f, dist)) &&
			    hit_sphere(mk3(e->p0[0], e->p0[1], e->p0[2]), e->radius, o, d, e->eps, t) && t < tl;
		} else {
			h = any_tri(mk3(e->p0[0], e->p0[1], e->p0[2]), mk3(e->e1[0], e->e1[1], e->e1[2]),
				    mk3(e->e2[0], e->e2[1], e->e2[2]), o, d, e->eps, tl);
		}
		if (h) {
			if (e->transparent)
				li = mul3v(li, mk3(e->kt[0], e->kt[1], e->kt[2]));
			else
				tl = -1.f;
		}
	}
	if (COUNT)
		sc.pln += (u64)popc64(ballot(act)) * num_planes;
	const bool alive = tl >= 0.f;
	const u64 live = ballot(alive);
	if (!live || !have_tree)
		return act && !alive;
	/* the ray in the trees' frame (rtx_device.h DTreeFrame): origin ob, direction db.  A shade point
	 * far from the bounded objects (a plane point far out, rtx_math.h tf_far; k_trace marks its
	 * record RTX_SP_FAR): the walk runs the segment from its other end, the light point, x' formed
	 * in double there; the same boxes meet the segment [0, dist] from either end, and the
	 * primitives are still tested from o along d.  In every frame: the world trees' slab test
	 * rounds at 2^-24 |o| too. */
	f3 ob = o, db = d;
	if (uni(tf.rotated)) {
		float r[3][3], c[3];
#pragma unroll
		for (int i = 0; i < 3; i++) {
			c[i] = __uint_as_float(uni(__float_as_uint(tf.c[i])));
#pragma unroll
			for (int j = 0; j < 3; j++)
				r[i][j] = __uint_as_float(uni(__float_as_uint(tf.r[i][j])));
		}
		ob = tf_point(r, c, o);
		db = tf_dir(r, d);
		if (far) {
			ob = tf_point_at(r, c, o, d, dist);
			db = mk3(-db.x, -db.y, -db.z);
		}
	} else if (far) {
		ob = tf_world_at(o, d, dist);
		db = mk3(-d.x, -d.y, -d.z);
	}
	if (COUNT)
		sc.far += (u64)popc64(ballot(alive && far));
	const f3 inv = safe_inv_fast(db); /* boxes are padded 2e-6 relative: a 1-ulp 1/d keeps the test conservative */
	const uint32_t oct = ((~__float_as_uint(inv.x)) >> 31) | (((~__float_as_uint(inv.y)) >> 31) << 1) |
			     (((~__float_as_uint(inv.z)) >> 31) << 2);
	const uint32_t lead = readlane(oct, (uint32_t)__ffsll((long long)live) - 1);
	const uint32_t sel = (!RTX_SH_OCT || ballot(alive & (oct != lead))) ? 8u : lead;
	switch (sel) {
#define RTX_WALK(K)                                                                            \
	case K:                                                                                \
		if (WALK == WALK_W8)                                                           \
			shadow_walk8<COUNT, K, LA>(Q, mats, o, d, ob, inv, tl, emit_obj, li, sc); \
		else                                                                           \
			shadow_walk<COUNT, K>(Q, recs, mats, o, d, ob, inv, tl, emit_obj, li, sc); \
		break;
		RTX_WALK(0) RTX_WALK(1) RTX_WALK(2) RTX_WALK(3) RTX_WALK(4) RTX_WALK(5) RTX_WALK(6) RTX_WALK(7)
#undef RTX_WALK
	default:
		if (WALK == WALK_W8)
			shadow_walk8<COUNT, 8, LA>(Q, mats, o, d, ob, inv, tl, emit_obj, li, sc);
		else
			shadow_walk<COUNT, 8>(Q, recs, mats, o, d, ob, inv, tl, emit_obj, li, sc);
		break;
	}
	return act && tl < 0.f;
}

/* ------------------------------------------------------------------------ */
/* light sampling and shading                                               */
/* ------------------------------------------------------------------------ */
/* k_shadow arguments.  Lane 0 copies them to LDS; the loops re-read them from there behind a
 * compiler memory barrier, so none stays live in registers across the walk. */
struct KShadow {
	const DPrim *prims;   /* primitive records (DQNode leaf refs are byte offsets from `recs`) */
	const char *recs;     /* base of the record array the leaf refs point into */	const DQNode *qnodes; /* threaded quantised BVH */
const DW8 *w8;        /* 8-wide compressed BVH (WALK_W8 instances; qo / qs / qsi are then its frame) */
	const DW8S *w8s;      /* its nodes' scalar-path copies */
	uint32_t *w8spill;    /* lane-stack spill area, [entry][grid lane] */
	uint32_t w8lstk;      /* lane-stack entries in LDS */
	uint32_t w8top;       /* entries of the 8-wide tree's top levels, copied to LDS per workgroup (DScene.w8top) */
	uint32_t w8sph;       /* the 8-wide tree holds spheres (DScene.w8sph) */
	const DEmitter *lin;  /* objects shadow_query tests one by one: the emitters the 8-wide tree leaves out,
	                       * or every bounded object of a tiny scene (no tree walk) */
	uint32_t num_lin;
	float qo[3], qs[3], qsi[3];
	DTreeFrame tf;        /* the trees' frame (their boxes are in it) */
	const uint32_t *top; /* its top levels (rtx_device.h RTX_QTOP_CUT), copied to LDS per workgroup */
	uint32_t ntop;
	const DMaterial *mats;
	const DPlane *planes;
	const DEmitter *emitters;
	const float4 *sp;
	const uint32_t *perm; /* shade points in processing (Morton) order, or null */
	float4 *contrib;
	unsigned long long *ctr;
	uint32_t have_tree, num_planes, num_emitters;
	uint32_t n_sp, per_wave, slot_b, slot_lg;
	int32_t rng, attenuation, reflection;
	float att_offset;
	const float4 *cull;   /* DScene.cull: the 8-wide tree's second-level bounding spheres (cone_clear) */
	uint32_t num_cull;    /* 0: no cull (RTX_OPT_SHADOW_CULL off, or no such tree) */
	uint32_t cull_slots;  /* the lane-slot path culls too (RTX_OPT_SHADOW_CULL 2) */
};

__device__ __forceinline__ void reread_barrier() { asm volatile("" ::: "memory"); }

/* a pointer read from LDS, made wave-uniform (SGPRs) so accesses through it stay scalar */
template <typename T> __device__ __forceinline__ T *unip(T *p)
{
	const uint64_t v = (uint64_t)p;
	return (T *)(((uint64_t)uni((uint32_t)(v >> 32)) << 32) | uni((uint32_t)v));
}

__device__ __forceinline__ float sh_rcp(float x) { return RTX_SH_FASTDIV ? __builtin_amdgcn_rcpf(x) : 1.f / x; }

/* light_point (object.c:293-304, 403-419) as k_shadow evaluates it (RTX_SH_FASTTRIG) */
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

/* field k of a shade-point record: UNI (>= 64 lights, the record is wave-uniform) through
 * scalar loads, else per lane */
template <bool UNI> __device__ __forceinline__ float4 sp_field(const float4 *rec, int k)
{
	if (UNI) {
		const auto *r = (const __attribute__((address_space(4))) f4v *)rec;
		const f4v v = r[k];
		return make_float4(v.x, v.y, v.z, v.w);
	}
	return ldg4(rec, 16 * k);
}

/* powf(x, y) of the specular term (render.c:224, fmaxf(0, powf(specular_mul, shininess))).
 * RTX_SH_FASTPOW: exp2(y * log2|x|) from v_log_f32 / v_exp_f32, with powf's y = 0 -> 1 and its
 * sign rule for x < 0 (odd integer y negative, even positive, otherwise NaN, which fmaxf
 * turns into 0).  Relative error about |y log2 x| * 2^-24 (< 2e-6 for results above 1e-9). */
__device__ __forceinline__ float sh_pow(float x, float y)
{
	if (!RTX_SH_FASTPOW)
		return powf(x, y);
	if (y == 0.f)
		return 1.f;
	const float ax = fabsf(x);
	const bool den = ax < 1.17549435e-38f; /* v_log_f32 flushes denormal inputs: scale by 2^32 */
	const float lx = __builtin_amdgcn_logf(den ? ax * 4294967296.f : ax) - (den ? 32.f : 0.f);
	const float r = __builtin_amdgcn_exp2f(y * lx);
	if (!(x < 0.f))
		return r;
	if (rintf(y) != y)
		return __builtin_nanf("");
	const float h = 0.5f * y; /* exact; an integer iff y is even */
	return rintf(h) != h ? -r : r;
}

/* the attenuation factor of a light sample at distance ldist (render.c:217-222), formed before
 * the walk so one float, not ldist and dsq, lives across it (the product with the transmittance
 * after the walk is the same operation in the same order) */
__device__ __forceinline__ float sample_att(const KShadow &ks, float ldist, float dsq)
{
	const int32_t att = (int32_t)uni((uint32_t)ks.attenuation);
	if (att == RTX_ATT_LIN)
		return sh_rcp(ks.att_offset + ldist);
	if (att == RTX_ATT_SQR)
		return sh_rcp(ks.att_offset + dsq);
	return 1.f;
}

/* direct-lighting terms of one unblocked light sample (render.c:199-228), read after the walk */
template <bool UNI>
__device__ __forceinline__ f3 shade_light(const KShadow &ks, const float4 *rec, f3 ldir, f3 li, float attf)
{
	const float4 q1 = sp_field<UNI>(rec, 1), q2 = sp_field<UNI>(rec, 2), q3 = sp_field<UNI>(rec, 3);
	const f3 n = mk3(q1.x, q1.y, q1.z), dir = mk3(q2.x, q2.y, q2.z);
	const float a = dot3(ldir, n);
	if ((int32_t)uni((uint32_t)ks.attenuation) != RTX_ATT_NONE)
		li = mul3s(li, attf);
	f3 ks3;
	float shin;
	if (UNI) { /* the material of a wave-uniform record: scalar reads */
		const auto &m = cptr(unip(ks.mats))[__float_as_uint(q3.w)];
		ks3 = mk3(m.ks[0], m.ks[1], m.ks[2]);
		shin = m.shininess;
	} else {
		const DMaterial &m = unip(ks.mats)[__float_as_uint(q3.w)];
		ks3 = ld3(m.ks);
		shin = m.shininess;
	}
	const f3 diff = mul3s(mul3v(mk3(q3.x, q3.y, q3.z), li), fmaxf(0.f, a));
	float sm;
	if ((int32_t)uni((uint32_t)ks.reflection) == RTX_BLINN)
		sm = -dot3(n, norm3(add3(mul3s(ldir, -1.f), dir)));
	else
		sm = -dot3(sub3(mul3s(n, 2.f * a), ldir), dir);
	const f3 spec = mul3s(mul3v(ks3, li), fmaxf(0.f, sh_pow(sm, shin)));
	return add3(diff, spec);
}

/* the light point of sample j of emitter number e, E (object.c:293-304, 403-419: stratified per
 * the rng mode), its shadow ray's direction and length, and the sample's intensity */
__device__ __forceinline__ void emitter_sample(const KShadow &ks, const DEmitter &E, uint32_t e, uint32_t j, uint32_t ka, uint32_t kb,
					       f3 p, f3 &ldir, float &ldist, float &dsq, f3 &li)
{
	float u1 = 0.5f, u2 = 0.5f;
	if (uni(ks.rng) != RTX_RNG_CONST) /* the key already carries the seed (rtx_key_pixel) */
		rtx_draw2(key_of(ka, kb), e, j, &u1, &u2);
	if (uni(ks.rng) == RTX_RNG_STRAT) /* stratum j of the emitter's lights (IEEE, as the oracle) */
		u1 = ((float)j + u1) / (float)E.num_lights;
	const f3 lp = light_point_sh(E, p, u1, u2);
	const f3 dv = sub3(lp, p);
	dsq = magsqr3(dv);
	ldist = RTX_SH_FASTSQRT ? __builtin_amdgcn_sqrtf(dsq) : sqrtf(dsq); /* mag3(dv) */
	ldir = mul3s(dv, sh_rcp(ldist));
	li = ld3(E.li);
}

/* an emitter record read through the scalar cache (every lane reads the same one) */
__device__ __forceinline__ DEmitter emitter_uni(const DEmitter *e)
{
	uint32_t w[sizeof(DEmitter) / 4];
	const auto *W = cptr((const uint32_t *)e);
#pragma unroll
	for (int i = 0; i < (int)(sizeof(DEmitter) / 4); i++)
		w[i] = W[i];
	DEmitter E;
	__builtin_memcpy(&E, w, sizeof(E));
	return E;
}

/* the shadow walks' view of the trees (QBvh) from the kernel arguments and the workgroup's LDS */
template <int WALK>
__device__ __forceinline__ QBvh make_qbvh(const KShadow &ks, const uint4 *top_q, const uint32_t *top_e, lds_u32 *stk,
					  const uint4 *t8, uint32_t wv)
{
	QBvh Q;
	Q.q = unip(ks.qnodes);
	Q.qo = mk3(ks.qo[0], ks.qo[1], ks.qo[2]);
	Q.qs = mk3(ks.qs[0], ks.qs[1], ks.qs[2]);
	Q.qsi = mk3(ks.qsi[0], ks.qsi[1], ks.qsi[2]);
	Q.top = top_q;
	Q.tend = top_e;
	Q.nt = uni(ks.ntop);
	Q.w8 = WALK == WALK_W8 ? unip(ks.w8) : nullptr;
	Q.w8s = WALK == WALK_W8 ? unip(ks.w8s) : nullptr;
	Q.t8 = t8;
	Q.nt8 = (WALK == WALK_W8 && RTX_W8_TOP) ? min(uni(ks.w8top), (uint32_t)RTX_W8_TOP_MAX) : 0u;
	Q.spill = WALK == WALK_W8 ? unip(ks.w8spill) : nullptr;
	Q.wv = wv;
	Q.lstk = uni(ks.w8lstk);
	Q.sph = uni(ks.w8sph) != 0;
	Q.stk = stk;
	Q.tq = stk + RTX_W8_STACK * WAVE;
	return Q;
}

/* The cone cull of a packet of one shade point's samples of one emitter: every shadow ray of the
 * packet runs from p to a point of the emitter, so it lies in the cone from p around the emitter's
 * bounding sphere (below), cut at the sphere's far side.  Lane k tests the bounding sphere k of the 8-wide tree's second level
 * (DScene.cull, world space): centre distance t along the axis, e off it; the sphere misses the
 * cone when e cos(a) - t sin(a) > r or it lies wholly before p or beyond the light.  r is padded
 * by 2e-5 of the coordinates' and distances' magnitudes, far above the rays' float rounding, so a
 * clear packet is one whose walks could reach no primitive: skipping them changes no bit of the
 * image (test_gpu_cone_cull_is_invisible).  True when no lane's sphere meets the cone. */
__device__ __forceinline__ bool cone_clear(const KShadow &ks, const DEmitter &E, f3 p)
{
	const uint32_t n = uni(ks.num_cull);
	if (!n)
		return false;
	/* the emitter's bounding sphere: a sphere light itself (its light points are c + ld with |ld|
	 * the radius to a few ulp, light_point_sh), a triangle's circumscribing sphere about its
	 * centroid (its light points lie in it); padded by 1e-4 of the radius and 1e-6 of |c| */
	f3 lc;
	float lr;
	if (E.type == RTX_SPHERE) {
		lc = ld3(E.p0);
		lr = E.radius;
	} else {
		const f3 a = ld3(E.p0), b = ld3(E.p1), c = ld3(E.p2);
		lc = mul3s(add3(add3(a, b), c), 1.f / 3.f);
		lr = sqrtf(fmaxf(fmaxf(magsqr3(sub3(a, lc)), magsqr3(sub3(b, lc))), magsqr3(sub3(c, lc))));
	}
	lr = lr * 1.0001f + 1e-6f * fmaxf(fmaxf(fabsf(lc.x), fabsf(lc.y)), fabsf(lc.z));
	const f3 ax0 = sub3(lc, p);
	const float L = sqrtf(magsqr3(ax0));
	if (!(L > 1.01f * lr)) /* the point at or inside the light's sphere: no cone */
		return false;
	const f3 ax = mul3s(ax0, 1.f / L);
	const float sn = lr / L, cs = sqrtf(fmaxf(0.f, 1.f - sn * sn));
	const float mag = fmaxf(fmaxf(fabsf(p.x), fabsf(p.y)), fabsf(p.z)) + fmaxf(fmaxf(fabsf(lc.x), fabsf(lc.y)), fabsf(lc.z));
	bool meets = false;
	const uint32_t k = lane_id();
	if (k < n) {
		const float4 sp = ldg4((const char *)(unip(ks.cull) + k), 0);
		const f3 v = sub3(mk3(sp.x, sp.y, sp.z), p);
		const float vv = magsqr3(v), t = dot3(v, ax);
		const float e = sqrtf(fmaxf(0.f, vv - t * t));
		const float br = sp.w + 2e-5f * (mag + sqrtf(vv) + L + lr);
		meets = vv <= br * br || (t >= -br && t <= L + lr + br && e * cs - t * sn <= br);
	}
	return !ballot(meets);
}

/* the emitters (bit e, e < 64) whose cone from shade point p meets no top-level box of the tree:
 * formed once per point of the wave-uniform path, before its packets (a far point: none) */
__device__ __forceinline__ u64 cone_mask(const KShadow &ks, f3 p, bool far)
{
	if (!uni(ks.num_cull) || far)
		return 0ull;
	const DEmitter *emitters = unip(ks.emitters);
	const uint32_t ne = min(uni(ks.num_emitters), 64u);
	u64 m = 0ull;
	for (uint32_t e = 0; e < ne; e++)
		if (cone_clear(ks, emitter_uni(emitters + e), p))
			m |= 1ull << e;
	return m;
}

/* The lane-slot path's cone mask (RTX_SH_SLOTCULL): each lane tests its own point's cones (emitters
 * e < 8) against every sphere in turn, the sphere and the emitter read through the scalar cache;
 * bit e set when no sphere meets.  A packet whose every live lane is clear for its emitter skips
 * the walk, as a clear point's packets do on the wave-uniform path. */
#ifndef RTX_SH_SLOTCULL
#define RTX_SH_SLOTCULL 1
#endif
__device__ __forceinline__ uint32_t cone_mask_lane(const KShadow &ks, f3 p, bool own)
{
	const uint32_t n = uni(ks.num_cull);
	if (!n)
		return 0u;
	const DEmitter *emitters = unip(ks.emitters);
	const uint32_t ne = min(uni(ks.num_emitters), 8u);
	const float4 *cull = unip(ks.cull);
	uint32_t m = 0u;
	for (uint32_t e = 0; e < ne; e++) {
		const DEmitter E = emitter_uni(emitters + e);
		f3 lc;
		float lr;
		if (E.type == RTX_SPHERE) {
			lc = ld3(E.p0);
			lr = E.radius;
		} else {
			const f3 a = ld3(E.p0), b = ld3(E.p1), c = ld3(E.p2);
			lc = mul3s(add3(add3(a, b), c), 1.f / 3.f);
			lr = sqrtf(fmaxf(fmaxf(magsqr3(sub3(a, lc)), magsqr3(sub3(b, lc))), magsqr3(sub3(c, lc))));
		}
		lr = lr * 1.0001f + 1e-6f * fmaxf(fmaxf(fabsf(lc.x), fabsf(lc.y)), fabsf(lc.z));
		const f3 ax0 = sub3(lc, p);
		const float L = sqrtf(magsqr3(ax0));
		bool meets = !own || !(L > 1.01f * lr);
		if (ballot(!meets)) {
			const f3 ax = mul3s(ax0, 1.f / L);
			const float sn = lr / L, cs = sqrtf(fmaxf(0.f, 1.f - sn * sn));
			const float mag = fmaxf(fmaxf(fabsf(p.x), fabsf(p.y)), fabsf(p.z)) + fmaxf(fmaxf(fabsf(lc.x), fabsf(lc.y)), fabsf(lc.z));
			for (uint32_t k = 0; k < n && ballot(!meets); k++) {
				const auto *q = (const __attribute__((address_space(4))) f4v *)(cull + k);
				const f4v sp = *q;
				const f3 v = sub3(mk3(sp.x, sp.y, sp.z), p);
				const float vv = magsqr3(v), t = dot3(v, ax);
				const float e2 = sqrtf(fmaxf(0.f, vv - t * t));
				const float br = sp.w + 2e-5f * (mag + sqrtf(vv) + L + lr);
				meets = meets || vv <= br * br || (t >= -br && t <= L + lr + br && e2 * cs - t * sn <= br);
			}
		}
		if (!meets)
			m |= 1u << e;
	}
	return m;
}

/* one light sample per lane of the shade point `rec` (render.c:170-229): the light point of
 * sample idx (emitters in scene order, the hit object skipped), its shadow ray, attenuation
 * and Phong / Blinn.  Argument-block fields are read from LDS behind reread barriers. */
template <bool COUNT, int WALK, bool UNI, bool LA, bool SC = false>
__device__ __forceinline__ f3 light_sample(const KShadow &ks, const float4 *rec_uni, uint32_t sidv, uint32_t idx, bool act, ShadowCount &sc,
					   const uint4 *top_q, const uint32_t *top_e, lds_u32 *stk, const uint4 *t8, uint32_t wv,
					   const uint32_t *cmask, uint32_t lclr = 0u)
{
	reread_barrier();
	/* the shade point's record: wave-uniform (UNI), or this lane's record sidv, whose address is
	 * formed again after the walk (the asm below) so only the 32-bit index lives across it: the
	 * 64-bit address did, and the allocator spilled it to scratch around the generic-octant walk,
	 * one store per packet (scene6: 43 GB of WRITE_SIZE per frame) */
	const float4 *rec = UNI ? rec_uni : unip(ks.sp) + (size_t)sidv * SPREC;
	const float4 q0 = sp_field<UNI && RTX_SH_SPUNI>(rec, 0), q4 = sp_field<UNI && RTX_SH_SPUNI>(rec, 4);
	const f3 p = mk3(q0.x, q0.y, q0.z);
	const uint32_t obj = __float_as_uint(q4.x) & ~RTX_SP_FAR, far = __float_as_uint(q4.x) & RTX_SP_FAR;
	const DEmitter *emitters = unip(ks.emitters);
	const auto *EM = cptr(emitters);
	const uint32_t num_emitters = uni(ks.num_emitters);
	/* the sample's emitter: one pass over the emitter table, read through the scalar cache */
	uint32_t j = idx, e = RTX_NONE;
	for (uint32_t k = 0; k < num_emitters; k++) {
		const uint32_t eo = EM[k].obj, enl = EM[k].num_lights;
		if (eo == obj || e != RTX_NONE)
			continue;
		if (j < enl)
			e = k;
		else
			j -= enl;
	}
	if (e == RTX_NONE)
		e = 0;
	/* every live lane's emitter the same (a packet inside one emitter's samples: the usual case):
	 * its record through the scalar cache too, else per lane */
	const u64 am = ballot(act);
	const uint32_t lead = readlane(e, am ? (uint32_t)__ffsll((long long)am) - 1 : 0u);
	f3 ldir, li;
	float ldist, dsq;
	uint32_t eobj;
	bool clear = false; /* UNI: the packet's cone meets no top-level box of the tree (cone_clear) */
	if (!ballot(act && e != lead)) {
		const DEmitter Eu = emitter_uni(emitters + lead);
		emitter_sample(ks, Eu, lead, j, __float_as_uint(q4.y), __float_as_uint(q4.z), p, ldir, ldist, dsq, li);
		eobj = Eu.obj;
		/* the point's cone_mask, kept in the wave's LDS table (a 64-bit mask in SGPRs across the walk
		 * cost the walk a spilled register) */
		clear = UNI && WALK == WALK_W8 && ((uni(cmask[lead >> 5]) >> (lead & 31u)) & 1u);
	} else {
		const DEmitter &E = emitters[e];
		emitter_sample(ks, E, e, j, __float_as_uint(q4.y), __float_as_uint(q4.z), p, ldir, ldist, dsq, li);
		eobj = E.obj;
	}
	/* the lane-slot path: every live lane's point clear for its emitter (cone_mask_lane) */
	if (!UNI && SC) {
		const bool lc = e < 8u && ((lclr >> (e & 7u)) & 1u);
		clear = ballot(act) && !ballot(act && !lc);
	}
	const float attf = sample_att(ks, ldist, dsq);
	const QBvh Q = make_qbvh<WALK>(ks, top_q, top_e, stk, t8, wv);
	const bool have_tree = uni(ks.have_tree) != 0 && !RTX_DEBUG_NOWALK && !clear;
	if (COUNT && clear)
		sc.clear += (u64)popc64(ballot(act));
	const bool blocked = shadow_query<COUNT, WALK, LA>(Q, unip(ks.recs), unip(ks.mats), unip(ks.planes), uni(ks.num_planes),
						 unip(ks.lin), uni(ks.num_lin), have_tree, ks.tf, act, far != 0, p, ldir, ldist, eobj, li,
							 sc);
	reread_barrier();
	if (!UNI && RTX_SH_RECAFTER) {
		asm volatile("" : "+v"(sidv));
		rec = unip(ks.sp) + (size_t)sidv * SPREC;
	}
	f3 contribution = mk3(0.f, 0.f, 0.f);
	if (act && !blocked)
		contribution = shade_light<UNI && RTX_SH_SPUNI>(ks, rec, ldir, li, attf);
	return contribution;
}

/* ------------------------------------------------------------------------ */
/* the kernel                                                               */
/* ------------------------------------------------------------------------ */
/* Persistent workgroups of RTX_SH_NW waves.  A workgroup copies the threaded BVH's top levels
 * to LDS once; then each wave takes per_wave shade points at a time from a global queue
 * (RTX_C_SPQUEUE), in processing (Morton) order, until the points run out. */
/* PATH: 0 both packet layouts (a runtime branch on slot_b: the counting instances), 1 only the
 * wave-uniform packets (slot_b = 64), 2 only the lane slots (slot_b < 64), 3 the lane slots with
 * their cone cull (RTX_OPT_SHADOW_CULL 2).  The product launches a
 * kernel of one layout, so each gets a register allocation of its own: with both in one kernel a
 * change to the slot loop moved the uniform loop's spills into its walk */
template <bool COUNT, int OCC, int WALK, int PATH>
__global__ __launch_bounds__(WAVE *RTX_SH_NW, OCC) void k_shadow(KShadow ka)
{
	constexpr bool TOP = WALK == WALK_BVH2;
	__shared__ uint4 top_q[TOP ? RTX_TOP_MAX : 1];    /* the top records (rtx_device.h RTX_QTOP_CUT) */
	__shared__ uint32_t top_e[TOP ? RTX_TOP_MAX : 1]; /* cut records: the DQNode index after the subtree */
	/* the wide walks' lane stacks (16-byte aligned: the slot fold below reuses a wave's stack area as
	 * float4 records, RTX_SH_SLOTFOLD) */
	__shared__ __attribute__((aligned(16))) uint32_t wstk[RTX_SH_NW][WALK == WALK_W8 ? RTX_W8_STACK + RTX_W8_TQ : 1][WAVE];
	static_assert(WALK != WALK_W8 || (RTX_W8_STACK + RTX_W8_TQ) * WAVE * sizeof(uint32_t) >= WAVE * sizeof(float4),
		      "a wave's lane-stack area must hold one float4 per lane for the slot fold");
	__shared__ KShadow ks_s; /* the arguments, one copy for the workgroup */
	/* WALK_W8: the 8-wide tree's top levels (RTX_W8_TOP_LEVELS), read by divergent steps from LDS */
	__shared__ uint4 t8[WALK == WALK_W8 && RTX_W8_TOP ? RTX_W8_TOP_MAX * 4 : 1];
	/* one wave's tables in one struct, so every lane addresses them from one base register */
	struct WaveTables {
		uint32_t off[WAVE + 1]; /* first lane slot of each shade point, total */
		uint32_t nls[WAVE];     /* shadow rays of each shade point */
		uint32_t sid[WAVE];     /* each shade point's index in the record array */
		float Ls[3][WAVE];      /* per shade point light sum, in packet order */
		uint32_t cm[2];         /* the current point's cone_mask (wave-uniform path) */
		uint8_t clr[WAVE];      /* each shade point's cone_mask_lane, emitters 0..7 (lane-slot path; a byte:
		                         * the LDS of two workgroups must still fit a CU) */
	};
	__shared__ WaveTables wt_w[RTX_SH_NW];
	const uint32_t ntop = TOP ? ka.ntop : 0u;
	for (uint32_t i = threadIdx.x; i < ntop; i += WAVE * RTX_SH_NW) {
		top_q[i] = ldg4u(ka.top + 4 * i);
		top_e[i] = gptr(ka.top)[4 * ntop + i];
	}
	const uint32_t nt8 = (WALK == WALK_W8 && RTX_W8_TOP) ? min(ka.w8top, (uint32_t)RTX_W8_TOP_MAX) : 0u;
	for (uint32_t i = threadIdx.x; i < 4 * nt8; i += WAVE * RTX_SH_NW)
		t8[i] = ldg4u((const uint32_t *)ka.w8 + 4 * i);
	const uint32_t wv = uni(threadIdx.x / WAVE);
	if (threadIdx.x == 0)
		ks_s = ka;
	__syncthreads();
	KShadow &ks = ks_s;
	uint32_t *off = wt_w[wv].off, *nls = wt_w[wv].nls, *sid = wt_w[wv].sid;
	uint8_t *clr = wt_w[wv].clr;
	float(*Ls)[WAVE] = wt_w[wv].Ls;
	/* the lane-stack addresses: per lane, or formed from lane_id() at each access (RTX_W8_LANEADDR; 2:
	 * the lane-slot kernel only, whose allocation spilled the per-lane address and reloaded it at
	 * every push and pop) */
	constexpr bool LA = RTX_W8_LANEADDR == 2 ? PATH >= 2 : RTX_W8_LANEADDR != 0;
	/* the lane-slot path's cone cull (RTX_OPT_SHADOW_CULL 2) lives in its own instance, PATH 3, so
	 * the default lane-slot kernel keeps its register allocation (with the code present but off,
	 * scene6's k_shadow took 1083.4 against 1074.8 ms) */
	constexpr bool SC = RTX_SH_SLOTCULL && WALK == WALK_W8 && (PATH == 3 || PATH == 0);
	lds_u32 *stk = (lds_u32 *)&wstk[wv][0][LA ? 0u : lane_id()];
	ShadowCount sc = { 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0 };
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
		if (PATH == 1 || (PATH == 0 && uni(ks.slot_b) == WAVE)) {
			/* >= 64 lights: every packet is 64 samples of ONE shade point.  The point is wave-uniform
			 * (its record is read once per packet through one address, no owner search), each lane
			 * sums its samples over the point's packets, and one butterfly per point reduces them. */
			for (uint32_t k = 0; k < cnt; k++) {
				reread_barrier();
				const uint32_t nl = uni(nls[k]);
				const float4 *rec = unip(ks.sp) + (size_t)uni(sid[k]) * SPREC;
				if (WALK == WALK_W8) {
					/* the point through vector loads made uniform, not the scalar loads light_sample
					 * makes: shared with them, the point was live from here and the compiler hoisted
					 * the far path's double-precision copies of it out of the packet loop and
					 * spilled them, three stores per point */
					const float4 q0 = ldg4(rec, 0), q4 = ldg4(rec, 64);
					const f3 pu = mk3(__uint_as_float(uni(__float_as_uint(q0.x))), __uint_as_float(uni(__float_as_uint(q0.y))),
							  __uint_as_float(uni(__float_as_uint(q0.z))));
					const u64 m = cone_mask(ks, pu, (uni(__float_as_uint(q4.x)) & RTX_SP_FAR) != 0);
					if (lane_id() == 0) {
						wt_w[wv].cm[0] = (uint32_t)m;
						wt_w[wv].cm[1] = (uint32_t)(m >> 32);
					}
					lds_sync();
				}
				f3 acc = mk3(0.f, 0.f, 0.f);
				for (uint32_t base = 0; base < nl; base += WAVE) {
					const uint32_t idx = base + lane_id();
					acc = add3(acc, light_sample<COUNT, WALK, true, LA>(ks, rec, 0u, idx, idx < nl, sc, top_q, top_e, stk, t8, wv,
											    wt_w[wv].cm));
				}
				const float sx = wave_sum(acc.x), sy = wave_sum(acc.y), sz = wave_sum(acc.z);
				if (lane_id() == 0) {
					Ls[0][k] = sx;
					Ls[1][k] = sy;
					Ls[2][k] = sz;
				}
			}
			lds_sync();
		} else {
			/* several points share a packet: each point's samples fill consecutive slots of B
			 * (power of two) lanes, B = slot_b; a point may straddle packets */
			if (SC) { /* each lane its own point's cone_mask_lane */
				uint32_t m = 0u;
				if (uni(ks.num_cull) && uni(ks.cull_slots)) {
					const float4 *my = unip(ks.sp) + (size_t)my_sid * SPREC;
					const float4 q0 = ldg4(my, 0), q4 = ldg4(my, 64);
					const bool far = (__float_as_uint(q4.x) & RTX_SP_FAR) != 0;
					m = cone_mask_lane(ks, mk3(q0.x, q0.y, q0.z), own && !far);
				}
				clr[lane_id()] = (uint8_t)m;
				lds_sync();
			}
			uint32_t kp = 0; /* this lane's point in the previous packet (its slots only move forward) */
			for (uint32_t base = 0;;) {
				reread_barrier();
				const uint32_t tot = uni(off[WAVE]), slot_b = uni(ks.slot_b), slot_lg = uni(ks.slot_lg);
				if (base >= tot)
					break;
				const uint32_t slot = base + (lane_id() >> slot_lg);
				uint32_t k = 0;
				if (slot < tot) {
					if (RTX_SH_OWNINC) { /* owner_of from the previous packet's owner: a step or two, not six */
						k = kp;
						while (off[k + 1] <= slot)
							k++;
						kp = k;
					} else {
						k = owner_of(off, slot);
					}
				}
				const uint32_t idx = ((slot - off[k]) << slot_lg) + (lane_id() & (slot_b - 1));
				const bool act = slot < tot && idx < nls[k];
				const f3 contribution = light_sample<COUNT, WALK, false, LA, SC>(ks, nullptr, sid[k], idx, act, sc, top_q, top_e, stk,
											 t8, wv, nullptr,
											 SC ? (uint32_t)clr[k] : 0u);
				/* per-shade-point sums.  Each slot's B lanes reduce in a fixed butterfly (masks B/2 .. 1),
				 * then the slot sums are added to their point's total one slot at a time in slot order, so a
				 * point whose slots straddle packets gets the same sum whatever its neighbours (with one slot
				 * per point this is the 64-lane butterfly over zeros and one slot it replaced, bit for bit) */
				const uint32_t t2 = uni(off[WAVE]), sb = uni(ks.slot_b), lg = uni(ks.slot_lg), spp = WAVE >> lg;
				f3 v = act ? contribution : mk3(0.f, 0.f, 0.f);
				if (sb > 16) {
					v.x += lane_xor_f<16>(v.x);
					v.y += lane_xor_f<16>(v.y);
					v.z += lane_xor_f<16>(v.z);
				}
				if (sb > 8) {
					v.x += lane_xor_f<8>(v.x);
					v.y += lane_xor_f<8>(v.y);
					v.z += lane_xor_f<8>(v.z);
				}
				if (sb > 4) {
					v.x += lane_xor_f<4>(v.x);
					v.y += lane_xor_f<4>(v.y);
					v.z += lane_xor_f<4>(v.z);
				}
				if (sb > 2) {
					v.x += lane_xor_f<2>(v.x);
					v.y += lane_xor_f<2>(v.y);
					v.z += lane_xor_f<2>(v.z);
				}
				if (sb > 1) {
					v.x += lane_xor_f<1>(v.x);
					v.y += lane_xor_f<1>(v.y);
					v.z += lane_xor_f<1>(v.z);
				}
				const uint32_t ns = min(t2 - base, spp);
				if (WALK == WALK_W8 && RTX_SH_SLOTFOLD) {
					/* the same fold with the slot sums handed over in LDS instead of v_readlane (four
					 * single-issue reads and three adds on SGPR operands per slot): each slot's first
					 * lane stores (sum, point) in the wave's lane-stack area, empty between walks, and
					 * lane 0 folds them in slot order (an LDS read, a compare and three adds per slot) */
					float4 *sl = (float4 *)&wstk[wv][0][0];
					if (!(lane_id() & (sb - 1)) && (lane_id() >> lg) < ns)
						sl[lane_id() >> lg] = make_float4(v.x, v.y, v.z, __uint_as_float(k));
					lds_sync();
					if (lane_id() == 0) {
						uint32_t kc = __float_as_uint(sl[0].w);
						float rx = Ls[0][kc], ry = Ls[1][kc], rz = Ls[2][kc];
						for (uint32_t j = 0; j < ns; j++) {
							const float4 q = sl[j];
							const uint32_t kj = __float_as_uint(q.w);
							if (kj != kc) {
								Ls[0][kc] = rx;
								Ls[1][kc] = ry;
								Ls[2][kc] = rz;
								kc = kj;
								rx = Ls[0][kc];
								ry = Ls[1][kc];
								rz = Ls[2][kc];
							}
							rx += q.x;
							ry += q.y;
							rz += q.z;
						}
						Ls[0][kc] = rx;
						Ls[1][kc] = ry;
						Ls[2][kc] = rz;
					}
					lds_sync();
					base += spp;
					continue;
				}
				uint32_t kc = readlane(k, 0);
				float rx = Ls[0][kc], ry = Ls[1][kc], rz = Ls[2][kc];
				for (uint32_t j = 0; j < ns; j++) {
					const uint32_t kj = readlane(k, j * sb);
					if (kj != kc) {
						if (lane_id() == 0) {
							Ls[0][kc] = rx;
							Ls[1][kc] = ry;
							Ls[2][kc] = rz;
						}
						kc = kj;
						rx = Ls[0][kc];
						ry = Ls[1][kc];
						rz = Ls[2][kc];
					}
					rx += readlanef(v.x, j * sb);
					ry += readlanef(v.y, j * sb);
					rz += readlanef(v.z, j * sb);
				}
				if (lane_id() == 0) {
					Ls[0][kc] = rx;
					Ls[1][kc] = ry;
					Ls[2][kc] = rz;
				}
				lds_sync();
				base += spp;
			}
		}
		reread_barrier();
		if (lane_id() < cnt) {
			const uint32_t me = sid[lane_id()]; /* re-read: my_sid need not stay live across the walks */
			const float4 *my = unip(ks.sp) + (size_t)me * SPREC;
			const float4 q0 = my[0], q1 = my[1], q2 = my[2], q5 = my[5];
			const f3 w = mk3(q0.w, q1.w, q2.w);
			const f3 c = mul3v(w, mk3(Ls[0][lane_id()], Ls[1][lane_id()], Ls[2][lane_id()]));
			unip(ks.contrib)[me] = make_float4(c.x, c.y, c.z, q5.x);
		}
		rays_total += uni(wave_sum_u(lane_id() < cnt ? nls[lane_id()] : 0u));
	}
	if (lane_id() == 0) {
		unsigned long long *ctr = unip(ks.ctr);
		atomicAdd(&ctr[RTX_C_SHADOW], rays_total);
		if (COUNT) {
			atomicAdd(&ctr[RTX_C_SBOXES], sc.boxes);
			atomicAdd(&ctr[RTX_C_SGBOXES], sc.gboxes);
			atomicAdd(&ctr[RTX_C_STRIS], sc.tris);
			atomicAdd(&ctr[RTX_C_SSPHERES], sc.sph);
			atomicAdd(&ctr[RTX_C_SPLANES], sc.pln);
			atomicAdd(&ctr[RTX_C_SSTEPS], sc.steps);
			atomicAdd(&ctr[RTX_C_SWALKS], sc.walks);
			atomicAdd(&ctr[RTX_C_SLEAFR], sc.lrounds);
			atomicAdd(&ctr[RTX_C_SUNIF], sc.unif);
			atomicAdd(&ctr[RTX_C_FARS], sc.far);
			atomicAdd(&ctr[RTX_C_SSPILL], sc.spills);
			atomicAdd(&ctr[RTX_C_SCLEAR], sc.clear);
		}
	}
}

/* ------------------------------------------------------------------------ */
/* known answers of the fast device functions k_shadow runs (rtx_kat.h)     */
/* ------------------------------------------------------------------------ */
__global__ void k_kat_shadow(int kind, uint32_t n, const float *__restrict__ in, float *__restrict__ out)
{
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n)
		return;
	const float *x = in + (size_t)i * rtx_kat_in_width[kind];
	float *y = out + (size_t)i * rtx_kat_out_width[kind];
	switch (kind) {
	case RTX_KAT_ANY_TRI:
		y[0] = any_tri(ld3(x + 6), ld3(x + 9), ld3(x + 12), ld3(x), ld3(x + 3), x[15], x[16]) ? 1.f : 0.f;
		break;
	case RTX_KAT_SPH_LIGHT_SH: {
		DEmitter e;
		e.type = RTX_SPHERE;
		for (int k = 0; k < 3; k++)
			e.p0[k] = x[k];
		e.radius = x[3];
		const f3 l = light_point_sh(e, ld3(x + 4), x[7], x[8]);
		y[0] = l.x;
		y[1] = l.y;
		y[2] = l.z;
	} break;
	case RTX_KAT_SPEC_POW:
		y[0] = fmaxf(0.f, sh_pow(x[0], x[1]));
		break;
	case RTX_KAT_BOX_Q: {
		/* the walk's setup (shadow_query / shadow_walk) and its box test on the quantised box */
		const f3 o = ld3(x), d = ld3(x + 3), qo = ld3(x + 12), qs = ld3(x + 15);
		const uint4 nd = make_uint4(rtx_quantise(x[6], x[9], qo.x, qs.x), rtx_quantise(x[7], x[10], qo.y, qs.y),
					    rtx_quantise(x[8], x[11], qo.z, qs.z), 0u);
		const f3 inv = safe_inv_fast(d);
		const f3 invq = mk3(inv.x * (1.f / qs.x), inv.y * (1.f / qs.y), inv.z * (1.f / qs.z));
		const f3 oq = mk3((o.x - qo.x) * qs.x, (o.y - qo.y) * qs.y, (o.z - qo.z) * qs.z);
		const f3 oi = mul3v(oq, invq);
		const uint32_t oct = ((~__float_as_uint(inv.x)) >> 31) | (((~__float_as_uint(inv.y)) >> 31) << 1) |
				     (((~__float_as_uint(inv.z)) >> 31) << 2);
		bool ho = false;
		switch (oct) {
#define RTX_KATOCT(K)                                      \
	case K:                                                \
		ho = box_hit_q<K>(nd, oi, invq, x[18]);            \
		break;
			RTX_KATOCT(0) RTX_KATOCT(1) RTX_KATOCT(2) RTX_KATOCT(3) RTX_KATOCT(4) RTX_KATOCT(5) RTX_KATOCT(6)
			RTX_KATOCT(7)
#undef RTX_KATOCT
		}
		y[0] = box_hit_q<8>(nd, oi, invq, x[18]) ? 1.f : 0.f;
		y[1] = ho ? 1.f : 0.f;
	} break;
	case RTX_KAT_BOX_Q8: {
		/* the 8-wide walk's setup and child test on the box quantised to 16 bits, then to 8 bits in
		 * the node frame (org, e) given by the record, exactly as rtx_wide8_build does */
		const f3 o = ld3(x), d = ld3(x + 3), qo = ld3(x + 12), qs = ld3(x + 15);
		uint32_t w[16];
		for (int k = 0; k < 16; k++)
			w[k] = 0;
		const uint32_t org[3] = { (uint32_t)x[19], (uint32_t)x[20], (uint32_t)x[21] };
		const uint32_t ex[3] = { (uint32_t)x[22], (uint32_t)x[23], (uint32_t)x[24] };
		w[0] = org[0] | (org[1] << 16);
		w[1] = org[2] | (ex[0] << 16) | (ex[1] << 20) | (ex[2] << 24);
		w[3] = 1u;
		for (int a = 0; a < 3; a++) {
			const uint32_t q8 = rtx_quantise8(rtx_quantise(x[6 + a], x[9 + a], x[12 + a], x[15 + a]), org[a], ex[a]);
			w[4 + 4 * a] = (q8 & 0xFFu) | 0xFFFFFF00u; /* slot 0 the box, slots 1..7 empty */
			w[5 + 4 * a] = 0xFFFFFFFFu;
			w[6 + 4 * a] = q8 >> 8;
			w[7 + 4 * a] = 0u;
		}
		const f3 inv = safe_inv_fast(d);
		const f3 invq = mk3(inv.x * (1.f / qs.x), inv.y * (1.f / qs.y), inv.z * (1.f / qs.z));
		const f3 oq = mk3((o.x - qo.x) * qs.x, (o.y - qo.y) * qs.y, (o.z - qo.z) * qs.z);
		const f3 oi = mul3v(oq, invq);
		const uint32_t oct = ((~__float_as_uint(inv.x)) >> 31) | (((~__float_as_uint(inv.y)) >> 31) << 1) |
				     (((~__float_as_uint(inv.z)) >> 31) << 2);
		f3 sc, bc;
		w8_frame(w, invq, oi, sc, bc);
		uint32_t ho = 0;
		switch (oct) {
#define RTX_KATOCT8(K)                                                        \
	case K:                                                                   \
		ho = w8_hits<K, (~(uint32_t)K & 7u)>(w, sc, bc, x[18]);               \
		ho = ho == (1u << (~(uint32_t)K & 7u)) ? 1u : ho ? 2u : 0u;           \
		break;
			RTX_KATOCT8(0) RTX_KATOCT8(1) RTX_KATOCT8(2) RTX_KATOCT8(3) RTX_KATOCT8(4) RTX_KATOCT8(5) RTX_KATOCT8(6)
			RTX_KATOCT8(7)
#undef RTX_KATOCT8
		}
		const uint32_t hg = w8_hits<8, 0u>(w, sc, bc, x[18]);
		/* 1 = slot 0 hit alone; 2 would flag an empty slot hit (never expected) */
		y[0] = hg == 1u ? 1.f : hg ? 2.f : 0.f;
		y[1] = (float)ho;
	} break;
	}
}

/* the 8-wide BVH's leaf entries: the primitive records they stand for (leafmap[i] = primitive
 * index, RTX_NONE for node entries and holes) */
__global__ void k_w8_fill(const DPrim *__restrict__ prims, const DMaterial *__restrict__ mats, const uint32_t *__restrict__ leafmap,
			  uint32_t n, DW8 *__restrict__ out)
{
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= 4 * n)
		return;
	const uint32_t e = i >> 2, p = leafmap[e];
	if (p == RTX_NONE)
		return;
	float4 v = ldg4((const char *)(prims + p), 16 * (i & 3));
	if ((i & 3) == 3) { /* the walks' copy: the material's kt in place of the normal, the record index */
		const DMaterial &m = mats[__float_as_uint(prims[p].c[3]) & RTX_META_MAT];
		v = make_float4(m.kt[0], m.kt[1], m.kt[2], __uint_as_float(p));
	}
	((float4 *)(out + e))[i & 3] = v;
}

extern "C" hipError_t rtx_launch_w8_fill(const DPrim *prims, const DMaterial *mats, const uint32_t *leafmap, uint32_t n, DW8 *out,
					  hipStream_t stream)
{
	if (!n)
		return hipSuccess;
	hipLaunchKernelGGL(k_w8_fill, dim3((4 * n + 255) / 256), dim3(256), 0, stream, prims, mats, leafmap, n, out);
	return hipGetLastError();
}

extern "C" hipError_t rtx_launch_kat_shadow(int kind, uint32_t n, const float *in, float *out, hipStream_t stream)
{
	if (kind < RTX_KAT_FIRST_SHADOW || kind >= RTX_KAT_NKINDS)
		return hipErrorInvalidValue;
	hipLaunchKernelGGL(k_kat_shadow, dim3((n + 255) / 256), dim3(256), 0, stream, kind, n, in, out);
	return hipGetLastError();
}

/* ------------------------------------------------------------------------ */
/* launcher (called from rtx_api.cpp)                                       */
/* ------------------------------------------------------------------------ */
template <bool C, int O, int W, int P> static hipError_t shadow_slots(uint32_t cus, uint32_t *slots)
{
	int per_cu = 0;
	hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void *>(&k_shadow<C, O, W, P>),
								   WAVE * RTX_SH_NW, 0);
	*slots = per_cu > 0 && cus > 0 ? (uint32_t)per_cu * cus : 1024u;
	return e;
}

/* the persistent grid: as many workgroups as are resident on the device at once (no more than
 * the work needs); the waves then share the shade points through RTX_C_SPQUEUE */
template <bool C, int O, int W, int P> static hipError_t launch_shadow_p(const KShadow &ka, uint32_t nw, uint32_t cus, hipStream_t stream)
{
	uint32_t slots = 0;
	hipError_t e = shadow_slots<C, O, W, P>(cus, &slots);
	if (e != hipSuccess)
		return e;
	const uint32_t need = (nw + RTX_SH_NW - 1) / RTX_SH_NW;
	hipLaunchKernelGGL((k_shadow<C, O, W, P>), dim3(need < slots ? need : slots), dim3(WAVE * RTX_SH_NW), 0, stream, ka);
	return hipGetLastError();
}
/* the counting instances keep both layouts in one kernel; the product picks the layout's own */
template <bool C, int O, int W> static hipError_t launch_shadow(const KShadow &ka, uint32_t nw, uint32_t cus, hipStream_t stream)
{
	if constexpr (C) {
		return launch_shadow_p<C, O, W, 0>(ka, nw, cus, stream);
	} else {
		if (ka.slot_b == WAVE)
			return launch_shadow_p<C, O, W, 1>(ka, nw, cus, stream);
		if (W == WALK_W8 && ka.cull_slots && ka.num_cull)
			return launch_shadow_p<C, O == RTX_SHADOW_OCC_DEFAULT ? RTX_SHADOW_OCC_SLOT : O, W, 3>(ka, nw, cus, stream);
		return launch_shadow_p<C, O == RTX_SHADOW_OCC_DEFAULT ? RTX_SHADOW_OCC_SLOT : O, W, 2>(ka, nw, cus, stream);
	}
}

template <int W> static hipError_t launch_walk(const KShadow &ka, uint32_t nw, uint32_t cus, int count, hipStream_t stream)
{
	if (count)
		return launch_shadow<true, 1, W>(ka, nw, cus, stream);
#if RTX_MEASURE
	/* occupancy variant (measurement builds): RTX_SHADOW_OCC = 1 (the compiler's choice) */
	const char *env = getenv("RTX_SHADOW_OCC");
	if (env && atoi(env) != RTX_SHADOW_OCC_DEFAULT)
		return launch_shadow<false, 1, W>(ka, nw, cus, stream);
#endif
	return launch_shadow<false, RTX_SHADOW_OCC_DEFAULT, W>(ka, nw, cus, stream);
}

/* the walk k_shadow runs for a scene: the 8-wide BVH when built, else the threaded BVH2 */
static int walk_of(const DScene *S) { return S->w8 ? WALK_W8 : WALK_BVH2; }

/* grid lanes of the largest k_shadow launch on `cus` CUs (sizes the 8-wide walk's spill area) */
extern "C" hipError_t rtx_shadow_grid_lanes(uint32_t cus, uint32_t *lanes)
{
	uint32_t a = 0, b = 0, a2 = 0;
	hipError_t e = shadow_slots<false, RTX_SHADOW_OCC_DEFAULT, WALK_W8, 1>(cus, &a);
	if (e == hipSuccess)
		e = shadow_slots<false, RTX_SHADOW_OCC_SLOT, WALK_W8, 2>(cus, &a2);
	if (e == hipSuccess) {
		uint32_t a3 = 0;
		e = shadow_slots<false, RTX_SHADOW_OCC_SLOT, WALK_W8, 3>(cus, &a3);
		a2 = a2 > a3 ? a2 : a3;
	}
	a = a > a2 ? a : a2;
	if (e == hipSuccess)
		e = shadow_slots<true, 1, WALK_W8, 0>(cus, &b);
#if RTX_MEASURE
	uint32_t c = 0, c2 = 0;
	if (e == hipSuccess)
		e = shadow_slots<false, 1, WALK_W8, 1>(cus, &c);
	if (e == hipSuccess)
		e = shadow_slots<false, 1, WALK_W8, 2>(cus, &c2);
	c = c > c2 ? c : c2;
	b = b > c ? b : c;
#endif
	*lanes = (a > b ? a : b) * WAVE * RTX_SH_NW;
	return e;
}

extern "C" hipError_t rtx_launch_shadow(const DScene *S, const DParams *P, const float4 *sp, const uint32_t *perm,
					uint32_t n_sp, uint32_t per_wave, uint32_t slot_b, float4 *contrib,
					unsigned long long *ctr, int count, uint32_t cus, hipStream_t stream)
{
	const uint32_t nw = per_wave ? (n_sp + per_wave - 1) / per_wave : 0u;
	if (!slot_b || (slot_b & (slot_b - 1)) || slot_b > WAVE || !per_wave || per_wave > WAVE)
		return hipErrorInvalidValue;
	if (!nw)
		return hipSuccess;
	if (S->num_top > RTX_TOP_MAX)
		return hipErrorInvalidValue;
	const int walk = walk_of(S);
	if (walk == WALK_W8 && (S->w8lstk < 1 || S->w8lstk > RTX_W8_STACK))
		return hipErrorInvalidValue;
	if (walk == WALK_W8 && S->w8depth > S->w8lstk + 1) {
		/* deep trees spill lane-stack entries to HBM: the area must cover this launch's grid */
		uint32_t lanes = 0;
		hipError_t e = rtx_shadow_grid_lanes(cus, &lanes);
		if (e != hipSuccess)
			return e;
		if (!S->w8spill || S->w8spill_lanes < lanes)
			return hipErrorInvalidValue;
	}
	KShadow ka;
	ka.prims = S->prims;
	ka.recs = (const char *)S->nodes;
	ka.qnodes = S->qnodes;
	ka.top = S->top;
	ka.ntop = S->num_top;
	ka.tf = S->tf;
for (int a = 0; a < 3; a++) {
		ka.qo[a] = S->qo[a];
		ka.qs[a] = S->qs[a];
		ka.qsi[a] = 1.f / S->qs[a];
	}
	ka.mats = S->mats;
	ka.planes = S->planes;
	ka.emitters = S->emitters;
	ka.sp = sp;
	ka.perm = perm;
	ka.contrib = contrib;
	ka.ctr = ctr;
	ka.have_tree = S->root_ref != RTX_EMPTY_REF && !S->lin && (S->w8 || S->qnodes); /* the walk of walk_of(S) has its tree */
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
	ka.w8 = S->w8;
	ka.w8s = S->w8s;
	ka.w8spill = S->w8spill;
	ka.w8lstk = S->w8lstk;
	ka.w8top = S->w8top;
	ka.w8sph = S->w8sph;
	ka.lin = S->lin; /* a tiny scene: every bounded object, no walk */
	ka.cull = (const float4 *)S->cull;
	ka.num_cull = (walk == WALK_W8 && S->cull) ? S->num_cull : 0u;
	ka.cull_slots = S->cull_slots;
	ka.num_lin = S->lin ? S->num_lin : 0u;
	if (walk == WALK_W8) { /* the 8-wide tree's own frame; the emitters it leaves out are tested linearly */
		for (int a = 0; a < 3; a++) {
			ka.qo[a] = S->w8qo[a];
			ka.qs[a] = S->w8qs[a];
			ka.qsi[a] = 1.f / S->w8qs[a];
		}
		ka.lin = S->emitters;
		ka.num_lin = S->w8noemit ? S->num_emitters : 0u;
	}
	if (walk == WALK_W8)
		return launch_walk<WALK_W8>(ka, nw, cus, count, stream);
	return launch_walk<WALK_BVH2>(ka, nw, cus, count, stream);
}

/* the code object of this file on the current device, loaded now (rtx_open) rather than at the
 * first launch inside an upload or a render */
extern "C" __attribute__((visibility("hidden"))) hipError_t rtx_load_shadow(void)
{
	hipFuncAttributes a;
	return hipFuncGetAttributes(&a, (const void *)k_w8_fill);
}
