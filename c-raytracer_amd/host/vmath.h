/*
 * Host-side float vector helpers with the same operation order as the
 * reference's src/core/calc.c (e.g. dot3 = (x*x' + y*y') + z*z', norm3 =
 * v * (1/|v|)), so host-computed scene values (edges, normals, epsilons,
 * image plane) round like the reference's generic build.
 */
#ifndef RTX_VMATH_H
#define RTX_VMATH_H

#include <math.h>

static inline float vm_sqr(float v) { return v * v; }
static inline float vm_dot3(const float *a, const float *b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static inline float vm_magsqr3(const float *a) { return vm_sqr(a[0]) + vm_sqr(a[1]) + vm_sqr(a[2]); }
static inline float vm_mag3(const float *a) { return sqrtf(vm_magsqr3(a)); }
static inline void vm_mul3s(const float *a, float s, float *r)
{
	r[0] = a[0] * s;
	r[1] = a[1] * s;
	r[2] = a[2] * s;
}
static inline void vm_add3v(const float *a, const float *b, float *r)
{
	r[0] = a[0] + b[0];
	r[1] = a[1] + b[1];
	r[2] = a[2] + b[2];
}
static inline void vm_sub3v(const float *a, const float *b, float *r)
{
	r[0] = a[0] - b[0];
	r[1] = a[1] - b[1];
	r[2] = a[2] - b[2];
}
static inline void vm_cross(const float *a, const float *b, float *r)
{
	float x = a[1] * b[2] - a[2] * b[1];
	float y = a[2] * b[0] - a[0] * b[2];
	float z = a[0] * b[1] - a[1] * b[0];
	r[0] = x;
	r[1] = y;
	r[2] = z;
}
static inline void vm_norm3(float *a) { vm_mul3s(a, 1.f / vm_mag3(a), a); }
static inline void vm_assign3(float *d, const float *s)
{
	d[0] = s[0];
	d[1] = s[1];
	d[2] = s[2];
}

#endif
