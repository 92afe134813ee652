// Microbenchmark (measurement only): per-instruction floor of a wave's global load on gfx950 by
// width (dword / dwordx2 / dwordx4) with all lanes on one 128-B line (L1-resident), and with 8
// lanes active.  Reports ns per wave-load per CU.
#include <hip/hip_runtime.h>
#include <cstdio>

template <typename T>
__global__ __launch_bounds__(256) void k_w(const T *__restrict__ t, int active, int iters, uint32_t *out)
{
	const uint32_t lane = threadIdx.x & 63;
	uint32_t h = blockIdx.x * 2654435761u, acc = 0;
	if ((int)lane < active) {
		for (int i = 0; i < iters; i++) {
			h = h * 1664525u + 1013904223u;
			const uint32_t per = 128 / sizeof(T); /* elements per 128-B line */
			const T v = t[((h >> 8) & 63) * per + (lane % per)];
			acc ^= *(const uint32_t *)&v;
		}
	}
	if (acc == 0x12345678u)
		out[0] = acc;
}

template <typename T> void run(const char *name, const void *t, uint32_t *o, int active)
{
	hipEvent_t a, b;
	(void)hipEventCreate(&a);
	(void)hipEventCreate(&b);
	const int iters = 256, blocks = 256 * 8 * 4;
	float ms = 0;
	for (int rep = 0; rep < 2; rep++) {
		(void)hipEventRecord(a);
		hipLaunchKernelGGL(k_w<T>, dim3(blocks), dim3(256), 0, 0, (const T *)t, active, iters, o);
		(void)hipEventRecord(b);
		(void)hipEventSynchronize(b);
		(void)hipEventElapsedTime(&ms, a, b);
	}
	printf("%-8s active %2d: %.3f ms  %.2f ns per wave-load per CU\n", name, active, ms, ms * 1e6 / ((double)blocks * 4 * iters / 256));
}

int main()
{
	void *t;
	uint32_t *o;
	(void)hipMalloc(&t, 1 << 16);
	(void)hipMalloc(&o, 64);
	(void)hipMemset(t, 1, 1 << 16);
	for (int active : {64, 8, 1}) {
		run<uint32_t>("dword", t, o, active);
		run<uint2>("dwordx2", t, o, active);
		run<uint4>("dwordx4", t, o, active);
	}
	return 0;
}
