/*
 * rtx_rng.h — counter-based replacement for rand_flt() (system.c:93-96).
 *
 * The reference draws every random number from one shared glibc rand() stream
 * seeded with wall-clock seconds, so its images are neither reproducible nor
 * thread-count independent.  The MI355X path keys every draw by
 *     (seed, pixel, ray-tree node, stream, index)
 * so a pixel's value does not depend on which GPU / wave / order rendered it.
 *
 *   node key : primary ray of pixel p       k = rtx_key_pixel(seed, p)
 *              reflection child             rtx_key_child(k, RTX_CHILD_REFLECT)
 *              refraction child             rtx_key_child(k, RTX_CHILD_REFRACT)
 *              path-GI sample i             rtx_key_child(k, RTX_CHILD_GI0 + i)
 *   draws    : light j of emitter e   (u1,u2) = rtx_draw2(k, e, j)       -> (inclination|p, azimuth|q)
 *              GI sample i            (u1,u2) = rtx_draw2(k, RTX_STREAM_GI, i)
 * u in [0,1) with 24-bit resolution.  Shared by the HIP kernels and the CPU
 * oracle (plain C, no dependencies), so both see identical random numbers.
 */
#ifndef RTX_RNG_H
#define RTX_RNG_H

#include <stdint.h>

#if defined(__HIPCC__)
#define RTX_HD __host__ __device__ __forceinline__
#else
#define RTX_HD static inline
#endif

#define RTX_CHILD_REFLECT 1u
#define RTX_CHILD_REFRACT 2u
#define RTX_CHILD_GI0 3u
#define RTX_STREAM_GI 0xFFFFFu

/* splitmix64 finaliser */
RTX_HD uint64_t rtx_mix64(uint64_t z)
{
	z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
	z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
	return z ^ (z >> 31);
}

RTX_HD uint64_t rtx_key_pixel(uint64_t seed, uint32_t pixel)
{
	return rtx_mix64(rtx_mix64(seed ^ 0x5851f42d4c957f2dull) + (uint64_t)pixel);
}

RTX_HD uint64_t rtx_key_child(uint64_t key, uint32_t tag)
{
	return rtx_mix64(key + 0x9e3779b97f4a7c15ull * ((uint64_t)tag + 1u));
}

/* 32-bit integer hash (C. Wellons' "lowbias32": two multiplies, full avalanche) */
RTX_HD uint32_t rtx_hash32(uint32_t x)
{
	x ^= x >> 16;
	x *= 0x21f0aaadu;
	x ^= x >> 15;
	x *= 0x735a2d97u;
	x ^= x >> 15;
	return x;
}

/* two uniform floats in [0,1).  The (key, stream) part is one splitmix64 round, the same for every
 * index, so a wave whose lanes share the key and the stream (the 64 light samples of one shade
 * point) computes it once in scalar registers; each index then costs two 32-bit hashes. */
RTX_HD void rtx_draw2(uint64_t key, uint32_t stream, uint32_t index, float *u1, float *u2)
{
	const uint64_t s = rtx_mix64(key ^ ((uint64_t)stream + 1u) * 0xd1b54a32d192ed03ull);
	const uint32_t a = rtx_hash32((uint32_t)s ^ index);
	const uint32_t b = rtx_hash32((uint32_t)(s >> 32) ^ a);
	*u1 = (float)(a >> 8) * (1.0f / 16777216.0f);
	*u2 = (float)(b >> 8) * (1.0f / 16777216.0f);
}

#endif
