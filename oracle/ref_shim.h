/*
 * ORACLE TEST INFRASTRUCTURE — not part of the product path.
 *
 * Force-included (gcc -include) into every translation unit of the reference
 * when oracle/Makefile builds it from /root/reference/src into oracle/_ref/.
 * It makes the reference bit-reproducible without touching its sources
 * (SURVEY.md Appendix B):
 *
 *  1. malloc -> calloc: the framebuffer is accumulated with += into an
 *     uninitialised malloc'd buffer (image.c:45, render.c:364).
 *  2. RNG: system.c:39 seeds glibc rand() with wall-clock seconds and
 *     rand_flt() (system.c:93-96) draws from one shared stream.
 *       -DREF_CONST_RNG : rand() == RAND_MAX/2, so rand_flt() == 0.5f exactly,
 *                         reproducible at any thread count.
 *       -DREF_KAT_RNG   : rand() returns values queued by oracle/ref_kat.c.
 *       otherwise       : srand(seed) with seed = $RTX_REF_SEED (default 1),
 *                         reproducible with -m 1.
 */
#ifndef RTX_REF_SHIM_H
#define RTX_REF_SHIM_H

#include <stdlib.h>

#define malloc(n) calloc(1, (n))

#if defined(REF_KAT_RNG)
/* oracle/ref_kat.c feeds chosen draws */
int rtx_kat_rand(void);
#define rand() rtx_kat_rand()
#elif defined(REF_CONST_RNG)
static inline int rtx_ref_const_rand(void)
{
	return RAND_MAX / 2;
}
#define rand() rtx_ref_const_rand()
#else
static inline unsigned rtx_ref_seed(void)
{
	const char *s = getenv("RTX_REF_SEED");
	return s ? (unsigned)strtoul(s, NULL, 10) : 1u;
}
#define srand(x) srand(rtx_ref_seed())
#endif

#endif
