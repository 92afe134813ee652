/*
 * ORACLE TEST INFRASTRUCTURE — not part of the product path.
 *
 * Ray counter for the reference build `oracle/_ref/engine_count`.
 * render.c is compiled with -finstrument-functions; gcc then calls
 * __cyg_profile_func_enter on entry to every function of that file, also for
 * copies it inlines.  We count entries of the two queries that define the
 * BASELINE metric:
 *   cast_ray          render.c:136  (closest-hit query: primary, reflection,
 *                                    refraction, GI)
 *   is_light_blocked  render.c:126  (shadow any-hit query)
 * and print them at exit.  The reference sources are not modified.
 */
#include <stdio.h>
#include <stdatomic.h>

/* Addresses only; the real prototypes live in the reference's render.c. */
extern char cast_ray[];
extern char is_light_blocked[];

static atomic_ullong n_closest, n_shadow;

void __cyg_profile_func_enter(void *fn, void *site) __attribute__((no_instrument_function));
void __cyg_profile_func_exit(void *fn, void *site) __attribute__((no_instrument_function));

void __cyg_profile_func_enter(void *fn, void *site)
{
	(void)site;
	if (fn == (void *)cast_ray)
		atomic_fetch_add_explicit(&n_closest, 1, memory_order_relaxed);
	else if (fn == (void *)is_light_blocked)
		atomic_fetch_add_explicit(&n_shadow, 1, memory_order_relaxed);
}

void __cyg_profile_func_exit(void *fn, void *site)
{
	(void)fn;
	(void)site;
}

__attribute__((destructor, no_instrument_function)) static void rtx_ref_count_report(void)
{
	fprintf(stderr, "RTX_REF_COUNT closest=%llu shadow=%llu\n",
		(unsigned long long)atomic_load(&n_closest), (unsigned long long)atomic_load(&n_shadow));
}
