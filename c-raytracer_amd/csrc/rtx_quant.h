/*
 * Quantisation of the threaded BVH's boxes (rtx_device.h DQNode), shared by the uploader
 * (rtx_api.cpp) and the device KAT of the quantised box test (rtx_shadow.hip), so the KAT
 * tests exactly the boxes the walk reads.  Compiled by hipcc only.
 *
 * A plane pair (lo, hi) on one axis of the frame (qo, qs) becomes 16-bit integers
 * ql = floor((lo - qo) * qs) - 1 and qh = ceil((hi - qo) * qs) + 1, clamped to [0, 65535]:
 * rounded outward and widened by one step on each side, so the quantised box contains the
 * float box (and the walk's rounding, far below one step, keeps the test conservative).
 */
#ifndef RTX_QUANT_H
#define RTX_QUANT_H

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

__host__ __device__ static inline uint32_t rtx_quantise(float lo, float hi, float qo, float qs)
{
	const double a = floor(((double)lo - qo) * (double)qs) - 1.0, b = ceil(((double)hi - qo) * (double)qs) + 1.0;
	const uint32_t ql = (uint32_t)fmin(65535.0, fmax(0.0, a)), qh = (uint32_t)fmin(65535.0, fmax(0.0, b));
	return ql | (qh << 16);
}

/* one axis of a child box in an 8-wide node's frame (rtx_device.h DW8): the 16-bit plane pair
 * q16 (rtx_quantise) relative to the node origin org (<= its lo) in steps of 2^e, rounded
 * outward, so [org + lo8 * 2^e, org + hi8 * 2^e] contains [lo16, hi16]; lo8 | hi8 << 8.  The
 * caller picks e so that hi8 <= 255. */
__host__ __device__ static inline uint32_t rtx_quantise8(uint32_t q16, uint32_t org, uint32_t e)
{
	const uint32_t lo = ((q16 & 0xFFFFu) - org) >> e, hi = ((q16 >> 16) - org + (1u << e) - 1u) >> e;
	return lo | (hi << 8);
}

#endif
