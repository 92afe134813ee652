/*
 * Wavefront helpers and the shade-point record shared by the gfx950 kernels
 * (rtx_trace.hip: k_trace / k_accum / k_kat, rtx_shadow.hip: k_shadow).
 * One wavefront = 64 lanes; every reduction here runs in a fixed lane order,
 * so sums are bit-identical whichever wave or GPU computes them.
 */
#ifndef RTX_WAVE_H
#define RTX_WAVE_H

#include <hip/hip_runtime.h>
#include <float.h>

#include "rtx_math.h"
#include "rtx_rng.h"

#define WAVE 64

/* ------------------------------------------------------------------------ */
/* wave helpers                                                             */
/* ------------------------------------------------------------------------ */
typedef unsigned long long u64;

__device__ __forceinline__ u64 ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }
__device__ __forceinline__ uint32_t popc64(u64 m) { return (uint32_t)__popcll(m); }
/* recomputed at every use (two VALU), never a value kept live across the walks (the register
 * allocator spilled it and reloaded it inside the walk loop) */
__device__ __forceinline__ uint32_t lane_id()
{
	uint32_t l;
	asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
	return l;
}
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

/* The value of lane (lane ^ M), from immediate lane patterns only (no per-lane address registers,
 * which __shfl_xor's ds_bpermute needs and the compiler keeps live across whole kernels):
 * M = 1, 2 DPP quad_perm, M = 4, 8, 16 ds_swizzle (xor mode within 32 lanes). */
template <int M> __device__ __forceinline__ uint32_t lane_xor_u(uint32_t v)
{
	if (M == 1)
		return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false); /* quad_perm [1,0,3,2] */
	if (M == 2)
		return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false); /* quad_perm [2,3,0,1] */
	return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, (M << 10) | 0x1F);
}
template <int M> __device__ __forceinline__ float lane_xor_f(float v) { return __uint_as_float(lane_xor_u<M>(__float_as_uint(v))); }

/* deterministic butterfly sum: every lane gets the same total.  Step M adds lane ^ M's value,
 * M = 32, 16, ..., 1; the cross-half step is v_permlane32_swap (both halves' values in every
 * lane; the two operand orders of lanes i and i ^ 32 give the same IEEE sum). */
__device__ __forceinline__ float wave_sum(float v)
{
	const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
	v = __uint_as_float(r[0]) + __uint_as_float(r[1]);
	v += lane_xor_f<16>(v);
	v += lane_xor_f<8>(v);
	v += lane_xor_f<4>(v);
	v += lane_xor_f<2>(v);
	v += lane_xor_f<1>(v);
	return v;
}

__device__ __forceinline__ uint32_t wave_sum_u(uint32_t v)
{
	const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
	v = r[0] + r[1];
	v += lane_xor_u<16>(v);
	v += lane_xor_u<8>(v);
	v += lane_xor_u<4>(v);
	v += lane_xor_u<2>(v);
	v += lane_xor_u<1>(v);
	return v;
}

/* exclusive prefix sum over the wave, bit by bit: the lanes below with bit b set are
 * mbcnt(ballot(bit b)); *tot = total (uniform).  No shuffles, so no per-lane address registers. */
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v, uint32_t *tot)
{
	uint32_t ex = 0, t = 0;
	for (uint32_t b = 0; b < 32; b++) {
		const u64 m = ballot((v >> b) & 1u);
		if (!ballot((v >> b) != 0u))
			break;
		ex += mbcnt(m) << b;
		t += popc64(m) << b;
	}
	*tot = t;
	return ex;
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
/* shade points: every hit that sees lights becomes one 96-byte record      */
/* (6 x float4), written by k_trace and read by k_shadow:                   */
/*   q0 = P, W.x   q1 = n, W.y   q2 = d, W.z   q3 = tex, mat                */
/*   q4 = obj, key_lo, key_hi, nl   q5 = slot, -, -, -                      */
/* (W: the hit's throughput, nl: its light samples, slot: its pixel lane)   */
/* ------------------------------------------------------------------------ */
#define SPREC 6 /* float4 per shade-point record */

#endif
