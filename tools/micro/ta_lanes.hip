// Microbenchmark (measurement only, not part of the product): cost of a wave's
// global_load_dwordx4 on gfx950 as a function of the active lanes, of how many distinct
// 128-B lines the lanes touch, and of where the table lives (L1-resident 16 KB, L2-resident 2 MB).
// Every wave issues `iters` independent 16-B loads; reports ns per wave-load per CU.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(256) void k_loads(const uint4 *__restrict__ t, uint32_t mask, int active, int share, int iters, uint4 *out)
{
	const uint32_t lane = threadIdx.x & 63;
	uint32_t h = ((blockIdx.x * 256 + threadIdx.x) / share) * 2654435761u; /* lanes of a share group: one address */
	uint4 acc = make_uint4(0, 0, 0, 0);
	if ((int)lane < active) {
		for (int i = 0; i < iters; i++) {
			h = h * 1664525u + 1013904223u;
			const uint4 v = t[((h >> 8) & mask) & ~7u]; /* 128-B aligned line */
			acc.x ^= v.x;
			acc.y ^= v.y;
			acc.z += v.z;
			acc.w += v.w;
		}
	}
	if (acc.x == 0x12345678u)
		out[0] = acc;
}

int main()
{
	uint4 *t, *o;
	(void)hipMalloc(&t, (1 << 17) * sizeof(uint4));
	(void)hipMalloc(&o, 64);
	(void)hipMemset(t, 1, (1 << 17) * sizeof(uint4));
	hipEvent_t a, b;
	(void)hipEventCreate(&a);
	(void)hipEventCreate(&b);
	const int iters = 256, blocks = 256 * 8 * 4;
	for (uint32_t n : {1u << 10, 1u << 17}) { /* 16 KB, 2 MB */
		for (int share : {1, 4, 16, 64}) {
			for (int active : {64, 16, 8, 1}) {
				if (share > active && share != 64)
					continue;
				float ms = 0;
				for (int rep = 0; rep < 2; rep++) {
					(void)hipEventRecord(a);
					hipLaunchKernelGGL(k_loads, dim3(blocks), dim3(256), 0, 0, t, n - 1, active, share, iters, o);
					(void)hipEventRecord(b);
					(void)hipEventSynchronize(b);
					(void)hipEventElapsedTime(&ms, a, b);
				}
				const double per = ms * 1e6 / ((double)blocks * 4 * iters / 256);
				printf("table %7u B  lanes/line %2d  active %2d: %.3f ms  %.2f ns per wave-load per CU\n", n * 16, share, active, ms, per);
			}
		}
	}
	return 0;
}
