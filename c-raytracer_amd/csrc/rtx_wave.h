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
/* shade points: every hit that sees lights becomes one 96-byte record      */
/* (6 x float4), written by k_trace and read by k_shadow:                   */
/*   q0 = P, W.x   q1 = n, W.y   q2 = d, W.z   q3 = tex, mat                */
/*   q4 = obj, key_lo, key_hi, nl   q5 = slot, -, -, -                      */
/* (W: the hit's throughput, nl: its light samples, slot: its pixel lane)   */
/* ------------------------------------------------------------------------ */
#define SPREC 6 /* float4 per shade-point record */

#endif
