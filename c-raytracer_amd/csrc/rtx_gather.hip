/*
 * Tile packing for the multi-device frame gather (rtx_group_render, rtx_group.cpp): each
 * device packs the tiles of its shard from its rgb/z framebuffer into 16-byte records
 * (rtx_tiles.h), RCCL carries them to device 0, which unpacks them into the full frame.
 * Pure HBM streaming: 28 B read + 16 B written per pixel.
 */
#include <hip/hip_runtime.h>

#include "rtx_tiles.h"

__global__ void k_tile_pack(const float *__restrict__ rgb, const float *__restrict__ z, uint32_t w, uint32_t h,
			    uint32_t off, uint32_t stride, uint32_t nrec, float4 *__restrict__ out)
{
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= nrec)
		return;
	uint32_t x, y;
	rtx_shard_pixel(i, rtx_tiles_x(w), off, stride, &x, &y);
	float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
	if (x < w && y < h) {
		const size_t p = (size_t)y * w + x;
		v = make_float4(rgb[3 * p], rgb[3 * p + 1], rgb[3 * p + 2], z[p]);
	}
	out[i] = v;
}

__global__ void k_tile_unpack(const float4 *__restrict__ in, uint32_t w, uint32_t h, uint32_t off, uint32_t stride,
			      uint32_t nrec, float *__restrict__ rgb, float *__restrict__ z)
{
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= nrec)
		return;
	uint32_t x, y;
	rtx_shard_pixel(i, rtx_tiles_x(w), off, stride, &x, &y);
	if (x >= w || y >= h)
		return;
	const size_t p = (size_t)y * w + x;
	const float4 v = in[i];
	rgb[3 * p] = v.x;
	rgb[3 * p + 1] = v.y;
	rgb[3 * p + 2] = v.z;
	z[p] = v.w;
}

extern "C" hipError_t rtx_launch_tile_pack(const float *rgb, const float *z, uint32_t w, uint32_t h, uint32_t off,
					   uint32_t stride, float4 *out, hipStream_t stream)
{
	const uint32_t nrec = rtx_shard_tiles(w, h, off, stride) * RTX_TILE_PX;
	if (!nrec)
		return hipSuccess;
	hipLaunchKernelGGL(k_tile_pack, dim3((nrec + 255) / 256), dim3(256), 0, stream, rgb, z, w, h, off, stride, nrec, out);
	return hipGetLastError();
}

extern "C" hipError_t rtx_launch_tile_unpack(const float4 *in, uint32_t w, uint32_t h, uint32_t off, uint32_t stride,
					     float *rgb, float *z, hipStream_t stream)
{
	const uint32_t nrec = rtx_shard_tiles(w, h, off, stride) * RTX_TILE_PX;
	if (!nrec)
		return hipSuccess;
	hipLaunchKernelGGL(k_tile_unpack, dim3((nrec + 255) / 256), dim3(256), 0, stream, in, w, h, off, stride, nrec, rgb, z);
	return hipGetLastError();
}

/* the code object of this file on the current device, loaded now (rtx_open) rather than at the
 * first launch inside an upload or a render */
extern "C" __attribute__((visibility("hidden"))) hipError_t rtx_load_gather(void)
{
	hipFuncAttributes a;
	return hipFuncGetAttributes(&a, (const void *)k_tile_pack);
}
