/*
 * Postprocess kernels: the reference's postprocessor
 * (src/postprocess/postproc.c) on the device-resident rgb+z framebuffer.
 *
 *   k_post_prep   brighten (postproc.c:93-101, mul3s) and, for depth of field, each source
 *                 pixel's circle of confusion: radius = (int)(|z*scale + bias| * .5),
 *                 alpha = MIN(1/radius^2, 1), pv = rgb * alpha (postproc.c:111-118);
 *                 plus the largest radius (atomicMax) that bounds the gather window
 *   k_post_zrange z_min / z_max over the z-buffer for --dof-camera (postproc.c:56-63),
 *                 strict < / > from FLT_MAX / FLT_MIN like the reference
 *   k_post_dof    the reference scatters every source pixel's pv over a disc
 *                 (x in [-r, r], |y| <= (int)sqrtf(r^2 - x^2)) onto pixels no nearer than the
 *                 source (postproc.c:119-155) and then normalises by the summed alphas
 *                 (postproc.c:160-161).  Each destination pixel receives its contributions
 *                 in increasing source index.  Here one thread per destination pixel walks
 *                 the (2R+1)^2 window of candidate sources in that same row-major order, so
 *                 every float sum is formed in the reference's order: bit-identical output.
 *   k_post_mist   postproc.c:165-188
 * All float arithmetic is IEEE single without contraction (-ffp-contract=off), as the
 * reference's -O3 (no fast-math) build does.
 */
#include <hip/hip_runtime.h>
#include <float.h>
#include <stdint.h>
#include <string.h>

#include "rtx.h"

__global__ __launch_bounds__(256) void k_post_prep(uint32_t n, float *__restrict__ rgb, const float *__restrict__ z,
						   int brighten, float factor, int dof, float scale, float bias,
						   int *__restrict__ rad, float4 *__restrict__ pv, unsigned *__restrict__ rmax)
{
	const uint32_t i = blockIdx.x * 256u + threadIdx.x;
	if (i >= n)
		return;
	float r = rgb[3 * (size_t)i], g = rgb[3 * (size_t)i + 1], b = rgb[3 * (size_t)i + 2];
	if (brighten) {
		r *= factor;
		g *= factor;
		b *= factor;
		rgb[3 * (size_t)i] = r;
		rgb[3 * (size_t)i + 1] = g;
		rgb[3 * (size_t)i + 2] = b;
	}
	if (!dof)
		return;
	const float coc = fabsf(z[i] * scale + bias);
	const int radius = (int)(coc * .5f);
	const int radius_sqr = radius * radius;
	const float inv = 1.f / (float)radius_sqr;
	const float alpha = inv < 1.f ? inv : 1.f; /* MIN(1.f / radius_sqr, 1.f) */
	rad[i] = radius;
	pv[i] = make_float4(r * alpha, g * alpha, b * alpha, alpha);
	atomicMax(rmax, (unsigned)(radius > 0 ? radius : 0));
}

/* order-preserving float <-> uint map for atomic min/max */
__device__ __forceinline__ unsigned fkey(float f)
{
	const unsigned u = __float_as_uint(f);
	return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__global__ __launch_bounds__(256) void k_post_zrange(uint32_t n, const float *__restrict__ z, unsigned *__restrict__ mm)
{
	float lo = FLT_MAX, hi = FLT_MIN;
	for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) {
		const float v = z[i];
		if (v < lo)
			lo = v;
		if (v > hi)
			hi = v;
	}
	for (int o = 32; o > 0; o >>= 1) {
		lo = fminf(lo, __shfl_xor(lo, o, 64));
		hi = fmaxf(hi, __shfl_xor(hi, o, 64));
	}
	if ((threadIdx.x & 63u) == 0) {
		atomicMin(&mm[0], fkey(lo));
		atomicMax(&mm[1], fkey(hi));
	}
}

__global__ __launch_bounds__(256) void k_post_dof(uint32_t w, uint32_t h, int R, const int *__restrict__ rad,
						  const float4 *__restrict__ pv, const float *__restrict__ z,
						  float *__restrict__ rgb)
{
	const int dx = (int)(blockIdx.x * 16u + (threadIdx.x & 15u)), dy = (int)(blockIdx.y * 16u + (threadIdx.x >> 4));
	if (dx >= (int)w || dy >= (int)h)
		return;
	const float zd = z[(size_t)dy * w + dx];
	float ar = 0.f, ag = 0.f, ab = 0.f, aa = 0.f;
	const int y0 = max(0, dy - R), y1 = min((int)h - 1, dy + R);
	const int x0 = max(0, dx - R), x1 = min((int)w - 1, dx + R);
	for (int sy = y0; sy <= y1; sy++) {
		const size_t row = (size_t)sy * w;
		const int y = dy - sy;
		for (int sx = x0; sx <= x1; sx++) {
			const int r = rad[row + sx];
			const int x = dx - sx;
			if (x < -r || x > r || y < -r || y > r)
				continue;
			const int hh = (int)sqrtf((float)(r * r - x * x));
			if (y < -hh || y > hh)
				continue;
			if (!(z[row + sx] <= zd)) /* postproc.c:133,148: depth <= z_buffer[idx] */
				continue;
			const float4 c = pv[row + sx];
			ar = ar + c.x;
			ag = ag + c.y;
			ab = ab + c.z;
			aa = aa + c.w;
		}
	}
	const float inv = 1.f / aa; /* postproc.c:160-161 */
	const size_t d = 3 * ((size_t)dy * w + dx);
	rgb[d] = ar * inv;
	rgb[d + 1] = ag * inv;
	rgb[d + 2] = ab * inv;
}

__global__ __launch_bounds__(256) void k_post_mist(uint32_t n, float *__restrict__ rgb, const float *__restrict__ z,
						   float start, float inv_depth, int falloff, float cr, float cg, float cb)
{
	const uint32_t i = blockIdx.x * 256u + threadIdx.x;
	if (i >= n)
		return;
	float f = (z[i] - start) * inv_depth; /* clamp(num, 0, 1), calc.c:164-168 */
	f = f < 0.f ? 0.f : f;
	f = f > 1.f ? 1.f : f;
	float op = f;
	if (falloff == RTX_FALLOFF_QUAD)
		op = f * f;
	else if (falloff == RTX_FALLOFF_INV_QUAD)
		op = sqrtf(f);
	const float k = 1.f - op;
	float *p = rgb + 3 * (size_t)i;
	p[0] = p[0] * k + cr * op;
	p[1] = p[1] * k + cg * op;
	p[2] = p[2] * k + cb * op;
}

extern "C" hipError_t rtx_launch_post(uint32_t w, uint32_t h, const rtx_post *pp, float *rgb, const float *z,
				      int *rad, float4 *pv, unsigned *scratch, hipStream_t stream)
{
	const uint32_t n = w * h;
	const dim3 g1((n + 255) / 256);
	float scale = pp->dof_scale, bias = pp->dof_bias;
	if (pp->dof == RTX_DOF_CAMERA) {
		const unsigned init[2] = { 0xFFFFFFFFu, 0u };
		hipError_t e = hipMemcpyAsync(scratch, init, sizeof(init), hipMemcpyHostToDevice, stream);
		if (e != hipSuccess)
			return e;
		hipLaunchKernelGGL(k_post_zrange, dim3(min((n + 255) / 256, 4096u)), dim3(256), 0, stream, n, z, scratch);
		unsigned mm[2];
		if ((e = hipMemcpyAsync(mm, scratch, sizeof(mm), hipMemcpyDeviceToHost, stream)) != hipSuccess ||
		    (e = hipStreamSynchronize(stream)) != hipSuccess)
			return e;
		auto unkey = [](unsigned k) {
			const unsigned u = (k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k;
			float f;
			memcpy(&f, &u, 4);
			return f;
		};
		const float z_min = unkey(mm[0]), z_max = unkey(mm[1]);
		const float A = pp->aperture, F = pp->focal_length, P = pp->plane_in_focus;
		/* postproc.c:65-66, same operation order */
		scale = (A * F * P * (z_max - z_min)) / ((P - F) * z_min * z_max);
		bias = (A * F * (z_min - P)) / ((P * F) * z_min);
	}
	if (pp->dof != RTX_DOF_NONE) {
		hipError_t e = hipMemsetAsync(scratch + 2, 0, sizeof(unsigned), stream);
		if (e != hipSuccess)
			return e;
	}
	if (pp->brighten || pp->dof != RTX_DOF_NONE)
		hipLaunchKernelGGL(k_post_prep, g1, dim3(256), 0, stream, n, rgb, z, pp->brighten, pp->brighten_factor,
				   pp->dof != RTX_DOF_NONE, scale, bias, rad, pv, scratch + 2);
	if (pp->dof != RTX_DOF_NONE) {
		unsigned R = 0;
		hipError_t e;
		if ((e = hipMemcpyAsync(&R, scratch + 2, sizeof(R), hipMemcpyDeviceToHost, stream)) != hipSuccess ||
		    (e = hipStreamSynchronize(stream)) != hipSuccess)
			return e;
		/* a radius beyond the frame reaches every pixel anyway */
		const int Rc = (int)min(R, max(w, h));
		hipLaunchKernelGGL(k_post_dof, dim3((w + 15) / 16, (h + 15) / 16), dim3(256), 0, stream, w, h, Rc, rad, pv, z,
				   rgb);
	}
	if (pp->mist)
		hipLaunchKernelGGL(k_post_mist, g1, dim3(256), 0, stream, n, rgb, z, pp->mist_start, 1.f / pp->mist_depth,
				   pp->mist_falloff, pp->mist_color[0], pp->mist_color[1], pp->mist_color[2]);
	return hipGetLastError();
}

/* the code object of this file on the current device, loaded now (rtx_open) rather than at the
 * first launch inside an upload or a render */
extern "C" __attribute__((visibility("hidden"))) hipError_t rtx_load_post(void)
{
	hipFuncAttributes a;
	return hipFuncGetAttributes(&a, (const void *)k_post_prep);
}
