// Microbenchmark: issue rate of single VALU instruction forms on gfx950 (the 8-wide box test's
// building blocks).  Each wave runs 8 independent chains of one instruction, 64 per loop trip;
// the chip is filled with 8 waves per SIMD.  Prints wave-instructions per second and cycles per
// wave-instruction per SIMD.
// build: hipcc --offload-arch=gfx950 -O3 tools/dev/valu_rates.hip -o tools/dev/valu_rates
#include <hip/hip_runtime.h>
#include <cstdio>

#define ITERS 2048
#define R8(X) X(x0) X(x1) X(x2) X(x3) X(x4) X(x5) X(x6) X(x7)
#define R64(X) R8(X) R8(X) R8(X) R8(X) R8(X) R8(X) R8(X) R8(X)

#define KERNEL(NAME, ASM, ...)                                                                         \
	__global__ void __launch_bounds__(256) NAME(float *out, float a, float b, uint32_t sel)         \
	{                                                                                          \
		float x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, \
		      x6 = x0 + 6, x7 = x0 + 7;                                                        \
		for (int i = 0; i < ITERS; i++) {                                                      \
			_Pragma("unroll") for (int u = 0; u < 1; u++) {                                \
				R64(OP_##NAME)                                                         \
			}                                                                          \
		}                                                                                  \
		out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;   \
	}

#define OP_k_fma_vvv(x) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x) : "v"(a), "v"(b));
#define OP_k_fma_vsv(x) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x) : "s"(sel), "v"(b));
#define OP_k_fma_vvc(x) asm volatile("v_fma_f32 %0, %0, %1, 1.0" : "+v"(x) : "v"(a));
#define OP_k_fma_neg(x) asm volatile("v_fma_f32 %0, %0, %1, -%2" : "+v"(x) : "v"(a), "v"(b));
#define OP_k_fmac(x) asm volatile("v_fmac_f32_e32 %0, %1, %2" : "+v"(x) : "v"(a), "v"(b));
#define OP_k_mul(x) asm volatile("v_mul_f32_e32 %0, %1, %0" : "+v"(x) : "v"(a));
#define OP_k_add(x) asm volatile("v_add_f32_e32 %0, %1, %0" : "+v"(x) : "v"(a));
#define OP_k_sub(x) asm volatile("v_sub_f32_e32 %0, %1, %0" : "+v"(x) : "v"(a));
#define OP_k_min(x) asm volatile("v_min_f32_e32 %0, %1, %0" : "+v"(x) : "v"(a));
#define OP_k_max3(x) asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(x) : "v"(a), "v"(b));
#define OP_k_med3(x) asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(x) : "v"(a), "v"(b));
#define OP_k_mix(x) asm volatile("v_fma_mix_f32 %0, %0, %1, %2 op_sel_hi:[1,0,0]" : "+v"(x) : "v"(a), "v"(b));
#define OP_k_cvtub(x) asm volatile("v_cvt_f32_ubyte1 %0, %0" : "+v"(x));
#define OP_k_cvtu(x) asm volatile("v_cvt_f32_u32 %0, %0" : "+v"(x));
#define OP_k_perm(x) asm volatile("v_perm_b32 %0, 0, %0, %1" : "+v"(x) : "s"(sel));
#define OP_k_and(x) asm volatile("v_and_b32_e32 %0, %1, %0" : "+v"(x) : "v"(a));
#define OP_k_or3(x) asm volatile("v_or3_b32 %0, %0, %1, %2" : "+v"(x) : "v"(a), "v"(b));
#define OP_k_addu(x) asm volatile("v_add_u32_e32 %0, %1, %0" : "+v"(x) : "v"(a));
#define OP_k_bfe(x) asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(x));
#define OP_k_lshr(x) asm volatile("v_lshrrev_b32_e32 %0, 8, %0" : "+v"(x));
#define OP_k_mov(x) asm volatile("v_mov_b32_e32 %0, %1" : "=v"(x) : "v"(a));
#define OP_k_cndmask(x) asm volatile("v_cndmask_b32_e64 %0, %0, %1, s[0:1]" : "+v"(x) : "v"(a) : "s0", "s1");
#define OP_k_cmp(x) asm volatile("v_cmp_le_f32_e64 s[0:1], %0, %1" : : "v"(x), "v"(a) : "s0", "s1");
#define OP_k_pkfma(x) asm volatile("v_pk_fma_f32 v[0:1], v[0:1], v[2:3], v[4:5]" ::: "v0", "v1", "v2", "v3", "v4", "v5");
#define OP_k_pkmul(x) asm volatile("v_pk_mul_f32 v[0:1], v[0:1], v[2:3]" ::: "v0", "v1", "v2", "v3");
#define OP_k_pkadd(x) asm volatile("v_pk_add_f32 v[0:1], v[0:1], v[2:3]" ::: "v0", "v1", "v2", "v3");
#define OP_k_ldexp(x) asm volatile("v_ldexp_f32 %0, %0, %1" : "+v"(x) : "v"(sel));
#define OP_k_rcp(x) asm volatile("v_rcp_f32_e32 %0, %0" : "+v"(x));
#define OP_k_cvtf16(x) asm volatile("v_cvt_f32_f16_e32 %0, %0" : "+v"(x));
#define OP_k_fmaf16(x) asm volatile("v_fma_f16 %0, %0, %1, %2" : "+v"(x) : "v"(a), "v"(b));
#define OP_k_dot2(x) asm volatile("v_dot2c_f32_f16_e32 %0, %1, %2" : "+v"(x) : "v"(a), "v"(b));

#define OP_k_cmp32(x) asm volatile("v_cmp_le_f32_e32 vcc, %0, %1" : : "v"(x), "v"(a) : "vcc");
#define OP_k_cnd32(x) asm volatile("v_cndmask_b32_e32 %0, 0, %0, vcc" : "+v"(x) : : "vcc");
#define OP_k_or(x) asm volatile("v_or_b32_e32 %0, %1, %0" : "+v"(x) : "v"(a));
#define OP_k_xor(x) asm volatile("v_xor_b32_e32 %0, %1, %0" : "+v"(x) : "v"(a));
#define OP_k_lshl(x) asm volatile("v_lshlrev_b32_e32 %0, 3, %0" : "+v"(x));
#define OP_k_max(x) asm volatile("v_max_f32_e32 %0, %1, %0" : "+v"(x) : "v"(a));
#define OP_k_subu(x) asm volatile("v_sub_u32_e32 %0, %1, %0" : "+v"(x) : "v"(a));
#define OP_k_andlit(x) asm volatile("v_and_b32_e32 %0, 0x80000000, %0" : "+v"(x));
#define OP_k_addsgpr(x) asm volatile("v_add_f32_e32 %0, %1, %0" : "+v"(x) : "s"(sel));
#define OP_k_mullit(x) asm volatile("v_mul_f32_e32 %0, 0x3f800001, %0" : "+v"(x));
#define OP_k_orsdwa(x) asm volatile("v_or_b32_sdwa %0, %1, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "+v"(x) : "v"(a));
#define OP_k_cvtsdwa(x) asm volatile("v_cvt_f32_u32_sdwa %0, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1" : "+v"(x));
#define OP_k_bfi(x) asm volatile("v_bfi_b32 %0, %0, %1, %2" : "+v"(x) : "v"(a), "v"(b));
#define OP_k_lshlor(x) asm volatile("v_lshl_or_b32 %0, %0, 1, %1" : "+v"(x) : "v"(a));
#define OP_k_fmaak(x) asm volatile("v_fmaak_f32 %0, %0, %1, 0x3f800000" : "+v"(x) : "v"(a));
#define OP_k_mulu24(x) asm volatile("v_mul_u32_u24_e32 %0, %1, %0" : "+v"(x) : "v"(a));
#define OP_k_cvtpkbf(x) asm volatile("v_cvt_pk_f32_bf8_e32 v[0:1], %0" : : "v"(x) : "v0", "v1");
#define OP_k_maxu(x) asm volatile("v_max_u32_e32 %0, %1, %0" : "+v"(x) : "v"(a));
#define OP_k_minmix(x) asm volatile("v_min_f32_e32 %0, %1, %0\n v_add_f32_e32 v2, v3, v2" : "+v"(x) : "v"(a) : "v2", "v3");

#define OP_k_mullo(x) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x) : "v"(a));
#define OP_k_mulhi(x) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x) : "v"(a));
#define OP_k_mad64(x) asm volatile("v_mad_u64_u32 v[0:1], s[0:1], %0, %1, v[2:3]" : : "v"(x), "v"(a) : "v0", "v1", "s0", "s1");
#define OP_k_alignbit(x) asm volatile("v_alignbit_b32 %0, %0, %0, 13" : "+v"(x));
#define OP_k_add3(x) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x) : "v"(a), "v"(b));
#define OP_k_xad(x) asm volatile("v_xad_u32 %0, %0, %1, %2" : "+v"(x) : "v"(a), "v"(b));
#define OP_k_sqrt(x) asm volatile("v_sqrt_f32_e32 %0, %0" : "+v"(x));
#define OP_k_sin(x) asm volatile("v_sin_f32_e32 %0, %0" : "+v"(x));
#define OP_k_divfmas(x) asm volatile("v_div_fmas_f32 %0, %0, %1, %2" : "+v"(x) : "v"(a), "v"(b) : "vcc");
#define OP_k_rndne(x) asm volatile("v_rndne_f32_e32 %0, %0" : "+v"(x));
#define OP_k_mbcnt(x) asm volatile("v_mbcnt_lo_u32_b32 %0, -1, %0" : "+v"(x));
#define OP_k_movsgpr(x) asm volatile("v_mov_b32_e32 %0, %1" : "=v"(x) : "s"(sel));
#define OP_k_mul64(x) asm volatile("v_lshrrev_b64 v[0:1], 7, v[0:1]" ::: "v0", "v1");

#define LIST3(X) X(k_mullo) X(k_mulhi) X(k_mad64) X(k_alignbit) X(k_add3) X(k_xad) X(k_sqrt) X(k_sin) X(k_divfmas) X(k_rndne) X(k_mbcnt) X(k_movsgpr) X(k_mul64)

#define LIST2(X) X(k_cmp32) X(k_cnd32) X(k_or) X(k_xor) X(k_lshl) X(k_max) X(k_subu) X(k_andlit) X(k_addsgpr) \
	X(k_mullit) X(k_orsdwa) X(k_cvtsdwa) X(k_bfi) X(k_lshlor) X(k_fmaak) X(k_mulu24) X(k_cvtpkbf) X(k_maxu) X(k_minmix)

#define LIST(X)                                                                                    \
	X(k_fma_vvv) X(k_fma_vsv) X(k_fma_vvc) X(k_fma_neg) X(k_fmac) X(k_mul) X(k_add) X(k_sub)     \
	X(k_min) X(k_max3) X(k_med3) X(k_mix) X(k_cvtub) X(k_cvtu) X(k_perm) X(k_and) X(k_or3)       \
	X(k_addu) X(k_bfe) X(k_lshr) X(k_mov) X(k_cndmask) X(k_cmp) X(k_pkfma) X(k_pkmul) X(k_pkadd) \
	X(k_ldexp) X(k_rcp) X(k_cvtf16) X(k_fmaf16) X(k_dot2)

#define DEF(N) KERNEL(N, 0)
LIST(DEF)
LIST2(DEF)
LIST3(DEF)

typedef void (*kfn)(float *, float, float, uint32_t);
static void run(const char *name, kfn f, float *out, int blocks, double clk_ghz, int cus)
{
	hipEvent_t e0, e1;
	hipEventCreate(&e0);
	hipEventCreate(&e1);
	hipLaunchKernelGGL(f, dim3(blocks), dim3(256), 0, 0, out, 1.0001f, 0.5f, 0x0C010C00u);
	hipEventRecord(e0);
	for (int r = 0; r < 3; r++)
		hipLaunchKernelGGL(f, dim3(blocks), dim3(256), 0, 0, out, 1.0001f, 0.5f, 0x0C010C00u);
	hipEventRecord(e1);
	hipEventSynchronize(e1);
	float ms = 0;
	hipEventElapsedTime(&ms, e0, e1);
	const double winst = 3.0 * blocks * 4.0 * ITERS * 64.0;
	const double rate = winst / (ms * 1e-3);
	printf("%-12s %8.3f ms  %7.1f G wave-instr/s  %5.2f cyc/wave-instr/SIMD\n", name + 2, ms, rate * 1e-9,
	       cus * 4.0 * clk_ghz * 1e9 / rate);
}

int main()
{
	hipDeviceProp_t p;
	hipGetDeviceProperties(&p, 0);
	const int blocks = p.multiProcessorCount * 8;
	float *out;
	hipMalloc(&out, (size_t)blocks * 256 * sizeof(float));
	printf("%s, %d CUs, clock %.2f GHz (cycles computed at 2.4 GHz)\n", p.gcnArchName, p.multiProcessorCount,
	       p.clockRate * 1e-6);
#define RUN(N) run(#N, N, out, blocks, 2.4, p.multiProcessorCount);
	LIST(RUN)
	LIST2(RUN)
	LIST3(RUN)
	hipFree(out);
	return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
