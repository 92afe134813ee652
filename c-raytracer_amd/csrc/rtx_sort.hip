/*
 * Shade-point ordering for k_shadow: shade points are sorted by the Morton code of their
 * position before the shadow pass, so the waves resident on one XCD at any moment cast
 * their shadow packets from one small region of the scene and walk one small part of the
 * BVH.  k_shadow maps blocks to XCDs so that each XCD's L2 serves a contiguous range of the
 * sorted order (the per-XCD L2s are 4 MB each; the benchmark BVH is 33 MB).
 *
 * Order only changes which wave computes a shade point, never what it computes: every
 * point's light sum comes from its own lane slots and lands in contrib[original index], so
 * the image is bit-identical with and without the sort.
 *
 * The sort itself is rocPRIM's radix sort (through hipCUB) on 30-bit keys; the key kernel
 * is ours.
 */
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>

#define SPREC 6 /* float4 per shade-point record (rtx_kernels.hip) */

__device__ __forceinline__ uint32_t spread10(uint32_t v)
{
	v &= 0x3FFu;
	v = (v | (v << 16)) & 0x030000FFu;
	v = (v | (v << 8)) & 0x0300F00Fu;
	v = (v | (v << 4)) & 0x030C30C3u;
	v = (v | (v << 2)) & 0x09249249u;
	return v;
}

__global__ __launch_bounds__(256) void k_spkey(const float4 *__restrict__ sp, uint32_t n, float lox, float loy,
						float loz, float sx, float sy, float sz, uint32_t *__restrict__ keys,
						uint32_t *__restrict__ vals)
{
	const uint32_t j = blockIdx.x * 256u + threadIdx.x;
	if (j >= n)
		return;
	const float4 q = sp[(size_t)j * SPREC];
	const float x = fminf(fmaxf((q.x - lox) * sx, 0.f), 1023.f);
	const float y = fminf(fmaxf((q.y - loy) * sy, 0.f), 1023.f);
	const float z = fminf(fmaxf((q.z - loz) * sz, 0.f), 1023.f);
	/* NaN coordinates (never produced for a hit) would land in cell 0 */
	keys[j] = spread10((uint32_t)x) | (spread10((uint32_t)y) << 1) | (spread10((uint32_t)z) << 2);
	vals[j] = j;
}

/* temp-storage bytes the sort of n pairs needs */
extern "C" hipError_t rtx_spsort_temp_bytes(uint32_t n, size_t *bytes)
{
	hipcub::DoubleBuffer<uint32_t> k(nullptr, nullptr), v(nullptr, nullptr);
	return hipcub::DeviceRadixSort::SortPairs(nullptr, *bytes, k, v, (int)n, 0, 30);
}

/* keys/vals: two buffers of n each (ping-pong); *perm <- the sorted shade-point indices */
extern "C" hipError_t rtx_launch_spsort(const float4 *sp, uint32_t n, const float lo[3], const float hi[3],
					uint32_t *keys0, uint32_t *keys1, uint32_t *vals0, uint32_t *vals1, void *temp,
					size_t temp_bytes, const uint32_t **perm, hipStream_t stream)
{
	*perm = vals0;
	if (!n)
		return hipSuccess;
	float s[3];
	for (int a = 0; a < 3; a++) {
		const float ext = hi[a] - lo[a];
		s[a] = ext > 0.f ? 1024.f / ext : 0.f;
	}
	hipLaunchKernelGGL(k_spkey, dim3((n + 255) / 256), dim3(256), 0, stream, sp, n, lo[0], lo[1], lo[2], s[0], s[1],
			   s[2], keys0, vals0);
	hipError_t e = hipGetLastError();
	if (e != hipSuccess)
		return e;
	hipcub::DoubleBuffer<uint32_t> k(keys0, keys1), v(vals0, vals1);
	e = hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, k, v, (int)n, 0, 30, stream);
	*perm = v.Current();
	return e;
}

/* the code object of this file on the current device, loaded now (rtx_open) rather than at the
 * first launch inside an upload or a render */
extern "C" __attribute__((visibility("hidden"))) hipError_t rtx_load_sort(void)
{
	hipFuncAttributes a;
	return hipFuncGetAttributes(&a, (const void *)k_spkey);
}
