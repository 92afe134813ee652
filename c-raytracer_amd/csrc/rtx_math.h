/*
 * Device math + the hot-path leaf functions, restated for gfx950 from the
 * reference (file:line in /root/reference):
 *   vector ops            src/core/calc.c            (same operation order)
 *   hit_sphere            object.c:306-321  line_intersects_sphere
 *   hit_triangle          object.c:422-441  moller_trumbore
 *   hit_plane             object.c:473-488  plane_get_intersection
 *   slab (reference form) accel.c:112-158   bounding_cuboid_intersects (KAT only;
 *                         traversal uses the branch-free min/max form below)
 *   simplex3              lib/SimplexNoise/SimplexNoise.c:99-194
 *   texture_color         material.c:152-200
 *   light_point           object.c:293-304, 403-419
 *   gi_direction          render.c:240-281
 *   refract_dir           render.c:320-335
 * IEEE single precision throughout (no fast-math); FMA contraction allowed.
 */
#ifndef RTX_MATH_H
#define RTX_MATH_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rtx.h"
#include "rtx_device.h"

#define RTX_PI 3.1415927f /* type.h:32 */

struct f3 {
	float x, y, z;
};

__device__ __forceinline__ f3 mk3(float x, float y, float z)
{
	f3 r;
	r.x = x;
	r.y = y;
	r.z = z;
	return r;
}
__device__ __forceinline__ f3 ld3(const float *p) { return mk3(p[0], p[1], p[2]); }
__device__ __forceinline__ f3 add3(f3 a, f3 b) { return mk3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ f3 sub3(f3 a, f3 b) { return mk3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ f3 mul3s(f3 a, float s) { return mk3(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ f3 mul3v(f3 a, f3 b) { return mk3(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ float dot3(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ float magsqr3(f3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
__device__ __forceinline__ float mag3(f3 a) { return sqrtf(magsqr3(a)); }
__device__ __forceinline__ f3 cross3(f3 a, f3 b)
{
	return mk3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
__device__ __forceinline__ f3 norm3(f3 a) { return mul3s(a, 1.f / mag3(a)); }
__device__ __forceinline__ bool isnan3(f3 a) { return a.x != a.x || a.y != a.y || a.z != a.z; }

/* ---- primitives ---- */
__device__ __forceinline__ bool hit_sphere(f3 c, float r, f3 o, f3 d, float eps, float &t)
{
	f3 rel = sub3(o, c);
	float b = -dot3(d, rel);
	float cc = dot3(rel, rel) - r * r;
	float det = b * b - cc;
	if (det < 0.f)
		return false;
	float sq = sqrtf(det);
	t = b - sq;
	if (t > eps)
		return true;
	t = b + sq;
	return t > eps;
}

__device__ __forceinline__ bool hit_triangle(f3 v0, f3 e1, f3 e2, f3 o, f3 d, float eps, float &t)
{
	f3 h = cross3(d, e2);
	float a = dot3(e1, h);
	if (a < eps && a > -eps)
		return false;
	float f = 1.f / a;
	f3 s = sub3(o, v0);
	float u = f * dot3(s, h);
	if (u < 0.f || u > 1.f)
		return false;
	f3 q = cross3(s, e1);
	float v = f * dot3(d, q);
	if (v < 0.f || u + v > 1.f)
		return false;
	t = f * dot3(e2, q);
	return t > eps;
}

__device__ __forceinline__ bool hit_plane(f3 n, float dd, f3 o, f3 d, float eps, float &t)
{
	float a = dot3(n, d);
	if (fabsf(a) < eps)
		return false;
	t = (dd - dot3(n, o)) / a;
	return t > eps;
}

/* bounding_cuboid_intersects, reference form (accel.c:112-158) */
__device__ __forceinline__ bool slab_ref(f3 lo, f3 hi, float eps, f3 o, f3 d, float &tmin, float &tmax)
{
	float tymin, tymax, tzmin, tzmax;
	float divx = 1.f / d.x;
	if (divx >= 0) {
		tmin = (lo.x - o.x) * divx;
		tmax = (hi.x - o.x) * divx;
	} else {
		tmin = (hi.x - o.x) * divx;
		tmax = (lo.x - o.x) * divx;
	}
	float divy = 1.f / d.y;
	if (divy >= 0) {
		tymin = (lo.y - o.y) * divy;
		tymax = (hi.y - o.y) * divy;
	} else {
		tymin = (hi.y - o.y) * divy;
		tymax = (lo.y - o.y) * divy;
	}
	if ((tmin > tymax) || (tymin > tmax))
		return false;
	if (tymin > tmin)
		tmin = tymin;
	if (tymax < tmax)
		tmax = tymax;
	float divz = 1.f / d.z;
	if (divz >= 0) {
		tzmin = (lo.z - o.z) * divz;
		tzmax = (hi.z - o.z) * divz;
	} else {
		tzmin = (hi.z - o.z) * divz;
		tzmax = (lo.z - o.z) * divz;
	}
	if (tmin > tzmax || tzmin > tmax)
		return false;
	if (tzmin > tmin)
		tmin = tzmin;
	if (tzmax < tmax)
		tmax = tzmax;
	return tmax > eps;
}

/* 1/d with zero components mapped to +-1e30 so (lo-o)*inv never forms 0*inf */
__device__ __forceinline__ f3 safe_inv(f3 d)
{
	return mk3(fabsf(d.x) > 1e-30f ? 1.f / d.x : copysignf(1e30f, d.x),
		   fabsf(d.y) > 1e-30f ? 1.f / d.y : copysignf(1e30f, d.y),
		   fabsf(d.z) > 1e-30f ? 1.f / d.z : copysignf(1e30f, d.z));
}

/* the same with v_rcp_f32 (1 ulp) for the walks' culling-only box tests: 1/d clamped to
 * [-1e30, 1e30] by one v_med3_f32 (1/(+-0) = +-inf lands on +-1e30, the sign of a zero kept as
 * copysign keeps it) instead of a compare, a select and a copysign per component */
__device__ __forceinline__ f3 safe_inv_fast(f3 d)
{
	return mk3(__builtin_amdgcn_fmed3f(__builtin_amdgcn_rcpf(d.x), -1e30f, 1e30f),
		   __builtin_amdgcn_fmed3f(__builtin_amdgcn_rcpf(d.y), -1e30f, 1e30f),
		   __builtin_amdgcn_fmed3f(__builtin_amdgcn_rcpf(d.z), -1e30f, 1e30f));
}

/* a point / direction in the trees' frame (rtx_device.h DTreeFrame): x' = R (x - c), d' = R d.
 * Culling only: the leaf boxes are padded for this rounding (rtx_frame.cpp) */
__device__ __forceinline__ f3 tf_dir(const float (&r)[3][3], f3 d)
{
	return mk3(fmaf(r[0][0], d.x, fmaf(r[0][1], d.y, r[0][2] * d.z)), fmaf(r[1][0], d.x, fmaf(r[1][1], d.y, r[1][2] * d.z)),
		   fmaf(r[2][0], d.x, fmaf(r[2][1], d.y, r[2][2] * d.z)));
}
__device__ __forceinline__ f3 tf_point(const float (&r)[3][3], const float (&c)[3], f3 x)
{
	return tf_dir(r, mk3(x.x - c[0], x.y - c[1], x.z - c[2]));
}

/* Ray origins far from the bounded objects.  The slab test's rounding grows with the origin's
 * distance (the transform's about 3 * 2^-24 (|x - c| + t), the world trees' (lo - o) * inv about
 * 2^-24 |o|), and the leaf boxes are padded for origins within a few radii of the objects
 * (rtx_frame.cpp; the world trees' 2e-6 relative padding).  An origin beyond RTX_FRAME_FAR radii
 * of their centre (the frame's max-norm about cf: DTreeFrame.cf, 0 for a rotated frame) gets a
 * frame origin near the objects computed in double, so the box tests stay conservative for any
 * origin, in every frame; the world ray the primitives are tested with is untouched, so no hit
 * changes. */
#define RTX_FRAME_FAR 4.f
__device__ __forceinline__ bool tf_far(f3 ob, const float (&cf)[3], float rad)
{
	return fmaxf(fabsf(ob.x - cf[0]), fmaxf(fabsf(ob.y - cf[1]), fabsf(ob.z - cf[2]))) > RTX_FRAME_FAR * rad;
}
/* x' = R (x - c) of the world point x + s d, the sum and product formed in double */
__device__ __forceinline__ f3 tf_point_at(const float (&r)[3][3], const float (&c)[3], f3 x, f3 d, float s)
{
	const double v0 = ((double)x.x - c[0]) + (double)s * d.x, v1 = ((double)x.y - c[1]) + (double)s * d.y,
		     v2 = ((double)x.z - c[2]) + (double)s * d.z;
	return mk3((float)(r[0][0] * v0 + r[0][1] * v1 + r[0][2] * v2), (float)(r[1][0] * v0 + r[1][1] * v1 + r[1][2] * v2),
		   (float)(r[2][0] * v0 + r[2][1] * v1 + r[2][2] * v2));
}
/* the same in the world frame (R = I, c = 0): x + s d rounded once */
__device__ __forceinline__ f3 tf_world_at(f3 x, f3 d, float s)
{
	return mk3((float)((double)x.x + (double)s * d.x), (float)((double)x.y + (double)s * d.y),
		   (float)((double)x.z + (double)s * d.z));
}
/* closest-hit rays (k_trace): the frame origin moved along the ray to t0, 2 radii before its
 * closest approach to c (every bounded object lies within sqrt(3) radii of c, so no hit comes
 * before t0); the walk then tests boxes against tbest - t0.  t0 = 0 for a ray leaving the scene. */
__device__ __forceinline__ f3 tf_shift(const float (&r)[3][3], const float (&c)[3], const float (&cf)[3], float rad, f3 o,
				      f3 d, float &t0)
{
	/* the objects' world centre is c + cf (one of the two is 0) */
	const double tca = -(((double)o.x - c[0] - cf[0]) * d.x + ((double)o.y - c[1] - cf[1]) * d.y +
			     ((double)o.z - c[2] - cf[2]) * d.z);
	const double ts = tca - 2.0 * (double)rad;
	t0 = ts > 0.0 ? (float)ts : 0.f;
	return tf_point_at(r, c, o, d, t0);
}

/* slab test on the traversal path: hit iff [max(tnear,0), min(tfar,tlim)] non-empty */
__device__ __forceinline__ bool slab(float lox, float hix, float loy, float hiy, float loz, float hiz, f3 oi, f3 inv,
				     float tlim, float &tnear)
{
	float tx0 = fmaf(lox, inv.x, -oi.x), tx1 = fmaf(hix, inv.x, -oi.x);
	float ty0 = fmaf(loy, inv.y, -oi.y), ty1 = fmaf(hiy, inv.y, -oi.y);
	float tz0 = fmaf(loz, inv.z, -oi.z), tz1 = fmaf(hiz, inv.z, -oi.z);
	float tn = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fmaxf(fminf(tz0, tz1), 0.f));
	float tf = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fminf(fmaxf(tz0, tz1), tlim));
	tnear = tn;
	return tn <= tf;
}

/* A far ray (tf_far) intersects a sphere only when it meets the sphere's world box, tested from
 * its origin shifted near the objects (oiw = ow * iw, ow formed in double).  The reference tests
 * every object's own world box before the object (accel.c:112-158, one object per BVH leaf), and
 * line_intersects_sphere's b*b - c (object.c:306-321) cancels catastrophically from far off
 * (|o - c|^2 >> r^2): a sphere sharing a multi-primitive leaf, or one whose leaf box is taken in a
 * rotated frame, could otherwise be "hit" by a far ray that passes well clear of it. */
/* does the ray x(t) = o + (s + sgn t) d, t in [0, tlim], meet the world box [lo, hi]?  Its origin
 * o + s d is formed in double.  Far rays only: the empty asm keeps the compiler from hoisting this
 * set-up (double-precision FMAs, three v_rcp) out of the branch that needs it, so a near ray
 * pays nothing and the registers of the hot loops around it stay free. */
__device__ __forceinline__ bool world_box_at(float lx, float hx, float ly, float hy, float lz, float hz, f3 o, f3 d,
					     float s, float sgn, float tlim)
{
	f3 dd = d;
	asm volatile("" : "+v"(dd.x), "+v"(dd.y), "+v"(dd.z));
	const f3 iw = safe_inv_fast(mk3(sgn * dd.x, sgn * dd.y, sgn * dd.z));
	float tn;
	return slab(lx, hx, ly, hy, lz, hz, mul3v(tf_world_at(o, dd, s), iw), iw, tlim, tn);
}
__device__ __forceinline__ bool far_sphere_box(f3 c, float r, f3 o, f3 d, float t0, float tlim)
{
	const float px = r + 2e-6f * (fabsf(c.x) + r), py = r + 2e-6f * (fabsf(c.y) + r), pz = r + 2e-6f * (fabsf(c.z) + r);
	return world_box_at(c.x - px, c.x + px, c.y - py, c.y + py, c.z - pz, c.z + pz, o, d, t0, 1.f, tlim);
}

/* ---- float -> uint32_t of material.c:164,173 ---- */
__device__ __forceinline__ uint32_t to_u32(float x, int mode)
{
	if (mode == RTX_U32_WRAP) {
		if (!(x > -9.2233720e18f && x < 9.2233720e18f))
			return 0u;
		return (uint32_t)(uint64_t)(int64_t)x;
	}
	if (!(x > -1.f && x < 4294967296.f))
		return 0xFFFFFFFFu;
	return (uint32_t)x;
}

/* ---- simplex noise ---- */
__constant__ static const uint8_t c_perm[256] = {
	151, 160, 137, 91, 90, 15, 131, 13, 201, 95, 96, 53, 194, 233, 7, 225, 140, 36, 103, 30, 69, 142, 8, 99, 37,
	240, 21, 10, 23, 190, 6, 148, 247, 120, 234, 75, 0, 26, 197, 62, 94, 252, 219, 203, 117, 35, 11, 32, 57, 177,
	33, 88, 237, 149, 56, 87, 174, 20, 125, 136, 171, 168, 68, 175, 74, 165, 71, 134, 139, 48, 27, 166, 77, 146,
	158, 231, 83, 111, 229, 122, 60, 211, 133, 230, 220, 105, 92, 41, 55, 46, 245, 40, 244, 102, 143, 54, 65, 25,
	63, 161, 1, 216, 80, 73, 209, 76, 132, 187, 208, 89, 18, 169, 200, 196, 135, 130, 116, 188, 159, 86, 164, 100,
	109, 198, 173, 186, 3, 64, 52, 217, 226, 250, 124, 123, 5, 202, 38, 147, 118, 126, 255, 82, 85, 212, 207, 206,
	59, 227, 47, 16, 58, 17, 182, 189, 28, 42, 223, 183, 170, 213, 119, 248, 152, 2, 44, 154, 163, 70, 221, 153,
	101, 155, 167, 43, 172, 9, 129, 22, 39, 253, 19, 98, 108, 110, 79, 113, 224, 232, 178, 185, 112, 104, 218, 246,
	97, 228, 251, 34, 242, 193, 238, 210, 144, 12, 191, 179, 162, 241, 81, 51, 145, 235, 249, 14, 239, 107, 49,
	192, 214, 31, 181, 199, 106, 157, 184, 84, 204, 176, 115, 121, 50, 45, 127, 4, 150, 254, 138, 236, 205, 93,
	222, 114, 67, 29, 24, 72, 243, 141, 128, 195, 78, 66, 215, 61, 156, 180
};

__device__ __forceinline__ int ph(int i) { return c_perm[(uint8_t)i]; }

__device__ __forceinline__ float corner_term(float x, float y, float z, int gi)
{
	float t = 0.6f - x * x - y * y - z * z;
	if (t < 0.f)
		return 0.f;
	t *= t;
	int h = gi & 15;
	float u = h < 8 ? x : y;
	float v = h < 4 ? y : (h == 12 || h == 14) ? x : z;
	float g = ((h & 1) ? -u : u) + ((h & 2) ? -v : v);
	return t * t * g;
}

__device__ inline float simplex3(float x, float y, float z)
{
	const float F3 = 1.0f / 3.0f, G3 = 1.0f / 6.0f;
	float s = (x + y + z) * F3;
	int i = (int)floorf(x + s), j = (int)floorf(y + s), k = (int)floorf(z + s);
	float t = (float)(i + j + k) * G3;
	float x0 = x - ((float)i - t), y0 = y - ((float)j - t), z0 = z - ((float)k - t);
	int i1, j1, k1, i2, j2, k2;
	if (x0 >= y0) {
		if (y0 >= z0) {
			i1 = 1; j1 = 0; k1 = 0; i2 = 1; j2 = 1; k2 = 0;
		} else if (x0 >= z0) {
			i1 = 1; j1 = 0; k1 = 0; i2 = 1; j2 = 0; k2 = 1;
		} else {
			i1 = 0; j1 = 0; k1 = 1; i2 = 1; j2 = 0; k2 = 1;
		}
	} else {
		if (y0 < z0) {
			i1 = 0; j1 = 0; k1 = 1; i2 = 0; j2 = 1; k2 = 1;
		} else if (x0 < z0) {
			i1 = 0; j1 = 1; k1 = 0; i2 = 0; j2 = 1; k2 = 1;
		} else {
			i1 = 0; j1 = 1; k1 = 0; i2 = 1; j2 = 1; k2 = 0;
		}
	}
	float x1 = x0 - i1 + G3, y1 = y0 - j1 + G3, z1 = z0 - k1 + G3;
	float x2 = x0 - i2 + 2.0f * G3, y2 = y0 - j2 + 2.0f * G3, z2 = z0 - k2 + 2.0f * G3;
	float x3 = x0 - 1.0f + 3.0f * G3, y3 = y0 - 1.0f + 3.0f * G3, z3 = z0 - 1.0f + 3.0f * G3;
	int g0 = ph(i + ph(j + ph(k)));
	int g1 = ph(i + i1 + ph(j + j1 + ph(k + k1)));
	int g2 = ph(i + i2 + ph(j + j2 + ph(k + k2)));
	int g3 = ph(i + 1 + ph(j + 1 + ph(k + 1)));
	float n0 = corner_term(x0, y0, z0, g0), n1 = corner_term(x1, y1, z1, g1);
	float n2 = corner_term(x2, y2, z2, g2), n3 = corner_term(x3, y3, z3, g3);
	return 32.0f * (n0 + n1 + n2 + n3);
}

/* ---- textures ---- */
__device__ inline f3 texture_color(const DMaterial &m, f3 p, int u32mode)
{
	switch (m.tex) {
	case RTX_TEX_CHECKERBOARD: {
		f3 sp = mul3s(p, m.scale);
		uint32_t parity = (to_u32(sp.x, u32mode) + to_u32(sp.y, u32mode) + to_u32(sp.z, u32mode)) % 2u;
		return ld3(m.color[parity]);
	}
	case RTX_TEX_BRICK: {
		f3 sp = mul3s(p, m.scale);
		uint32_t parity = to_u32(sp.x, u32mode) % 2u;
		sp.y -= parity * .5f;
		uint32_t mortar = (sp.x - floorf(sp.x) < m.mortar) || (sp.y - floorf(sp.y) < m.mortar);
		return ld3(m.color[mortar]);
	}
	case RTX_TEX_NOISY_PERIODIC: {
		f3 sp = mul3s(p, m.nfs);
		float angle = (p.x + simplex3(sp.x, sp.y, sp.z) * m.ns) * m.fs;
		float k;
		switch (m.periodic) {
		case RTX_PERIODIC_SIN: k = (1.f + sinf(angle)) * .5f; break;
		case RTX_PERIODIC_SAW: k = angle - floorf(angle); break;
		case RTX_PERIODIC_TRIANGLE: k = fabsf(2.f * (angle - floorf(angle) - .5f)); break;
		default: k = (float)!signbit(sinf(angle)); break;
		}
		return add3(mul3s(ld3(m.color[1]), k), ld3(m.color[0]));
	}
	default:
		return ld3(m.color[0]);
	}
}

/* ---- light samplers ---- */
__device__ __forceinline__ f3 light_point(const DEmitter &e, f3 p, float u1, float u2)
{
	if (e.type == RTX_SPHERE) {
		f3 c = ld3(e.p0);
		f3 nrm = sub3(c, p);
		float inc = u1 * 2.f * RTX_PI, az = u2 * 2.f * RTX_PI;
		float si = sinf(inc);
		f3 ld = mk3(e.radius * cosf(az) * si, e.radius * sinf(az) * si, e.radius * cosf(inc));
		if (dot3(nrm, ld) != 0.f)
			ld = mul3s(ld, -1.f);
		return add3(c, ld);
	}
	float pp = u1, q = u2;
	if (pp + q > 1.f) {
		pp = 1.f - pp;
		q = 1.f - q;
	}
	f3 v0 = ld3(e.p0), v1 = ld3(e.p1), v2 = ld3(e.p2);
	return mk3(v0.x + (v1.x - v0.x) * pp + (v2.x - v0.x) * q, v0.y + (v1.y - v0.y) * pp + (v2.y - v0.y) * q,
		   v0.z + (v1.z - v0.z) * pp + (v2.z - v0.z) * q);
}

/* ---- path-tracing GI direction (uniform hemisphere about n) ---- */
__device__ inline f3 gi_direction(f3 n, float eps, float u1, float u2)
{
	f3 r0, r1, r2;
	if (n.y - eps < -1.f) {
		r0 = mk3(1.f, 0.f, 0.f);
		r1 = mk3(0.f, -1.f, 0.f);
		r2 = mk3(0.f, 0.f, -1.f);
	} else {
		float mul = 1.f / (1.f + n.y);
		r0 = mk3(1.f - n.x * n.x * mul, n.x, -n.x * n.z * mul);
		r1 = mk3(-n.x, 1.f - (n.x * n.x + n.z * n.z) * mul, -n.z);
		r2 = mk3(-n.x * n.z * mul, n.z, 1.f - n.z * n.z * mul);
	}
	float inc = acosf(u1 * 2.f - 1.f), az = u2 * RTX_PI;
	float si = sinf(inc);
	f3 v = mk3(cosf(az) * si, sinf(az) * si, cosf(inc));
	return mk3(dot3(r0, v), dot3(r1, v), dot3(r2, v));
}

/* ---- refraction ---- */
__device__ inline f3 refract_dir(f3 d, f3 n, float b, bool outside, float ior)
{
	float inc = acosf(fabsf(b));
	float mult = outside ? 1.f / ior : ior;
	float refr = asinf(sinf(inc) * mult);
	float delta = refr - inc;
	f3 c = norm3(cross3(d, n));
	if (!outside)
		c = mul3s(c, -1.f);
	f3 f = cross3(c, d);
	return norm3(add3(mul3s(d, cosf(delta)), mul3s(f, sinf(delta))));
}

#endif
