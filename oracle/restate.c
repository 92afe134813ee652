/*
 * ORACLE TEST INFRASTRUCTURE — CPU restatement of C-Raytracer's hot path.
 *
 * This is the checker for the MI355X path (tests/, __graft_entry__.smoke())
 * and the "port" CPU baseline in bench.py.  It is never linked into, loaded by
 * or called from the product path (librtx.so / engine).
 *
 * It restates, in plain C and single-precision like the reference, the
 * semantics of (file:line in /root/reference):
 *   render()                    src/raytracer/render.c:345-368
 *   cast_ray()                  src/raytracer/render.c:136-343
 *   get_closest_intersection()  src/raytracer/render.c:118-124
 *   is_light_blocked()          src/raytracer/render.c:126-134
 *   unbound_objects_*()         src/raytracer/object.c:168-197
 *   accel_init()                src/raytracer/accel.c:266-315 (Morton LBVH, Karras split)
 *   bvh_get_closest_intersection / bvh_is_light_blocked  accel.c:322-387
 *   bounding_cuboid_intersects  accel.c:112-158
 *   sphere/triangle/plane intersectors and light samplers  object.c:254-498
 *   textures                    src/raytracer/material.c:152-200
 *   simplex_noise               lib/SimplexNoise/SimplexNoise.c:99-194
 * with rand_flt() (system.c:93-96) replaced by rtx_rng.h (counter) or the
 * constant 0.5 of the reference's REF_CONST_RNG build.
 *
 * Parity of this restatement is pinned by tests/test_oracle.py against frames
 * and per-function known answers produced by the compiled reference
 * (oracle/_ref, tools/make_goldens.py).
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <omp.h>

#include "rtx.h"
#include "rtx_kat.h"
#include "rtx_rng.h"

#define PI 3.1415927f /* type.h:32 */

typedef float v3[3];

/* ---- calc.c ---- */
static inline float sqr(float v) { return v * v; }
static inline float dot3(const float *a, const float *b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static inline float magsqr3(const float *a) { return sqr(a[0]) + sqr(a[1]) + sqr(a[2]); }
static inline float mag3(const float *a) { return sqrtf(magsqr3(a)); }
static inline void mul3s(const float *a, float s, float *r) { r[0] = a[0] * s; r[1] = a[1] * s; r[2] = a[2] * s; }
static inline void mul3v(const float *a, const float *b, float *r) { r[0] = a[0] * b[0]; r[1] = a[1] * b[1]; r[2] = a[2] * b[2]; }
static inline void add3v(const float *a, const float *b, float *r) { r[0] = a[0] + b[0]; r[1] = a[1] + b[1]; r[2] = a[2] + b[2]; }
static inline void sub3v(const float *a, const float *b, float *r) { r[0] = a[0] - b[0]; r[1] = a[1] - b[1]; r[2] = a[2] - b[2]; }
static inline void assign3(float *d, const float *s) { d[0] = s[0]; d[1] = s[1]; d[2] = s[2]; }
static inline void cross(const float *a, const float *b, float *r)
{
	float x = a[1] * b[2] - a[2] * b[1], y = a[2] * b[0] - a[0] * b[2], z = a[0] * b[1] - a[1] * b[0];
	r[0] = x; r[1] = y; r[2] = z;
}
static inline void norm3(float *a) { mul3s(a, 1.f / mag3(a), a); }

/* ---- float -> uint32_t of material.c:164,173 ---- */
static inline uint32_t to_u32(float x, int mode)
{
	if (mode == RTX_U32_WRAP) {
		if (!(x > -9.2233720e18f && x < 9.2233720e18f))
			return 0u; /* cvttss2si 64-bit indefinite 0x8000000000000000 -> low 32 bits */
		return (uint32_t)(uint64_t)(int64_t)x;
	}
	if (!(x > -1.f && x < 4294967296.f))
		return 0xFFFFFFFFu; /* vcvttss2usi out of range / NaN */
	return (uint32_t)x;
}

/* ---- SimplexNoise.c (Gustavson/Perlin 3D simplex noise) ---- */
static const uint8_t perm[256] = {
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
#define PH(i) perm[(uint8_t)(i)]

static float corner_grad(int hash, float x, float y, float z)
{
	int h = hash & 15;
	float u = h < 8 ? x : y;
	float v = h < 4 ? y : (h == 12 || h == 14) ? x : z;
	return ((h & 1) ? -u : u) + ((h & 2) ? -v : v);
}

static float corner_term(float x, float y, float z, int gi)
{
	float t = 0.6f - x * x - y * y - z * z;
	if (t < 0)
		return 0.f;
	t *= t;
	return t * t * corner_grad(gi, x, y, z);
}

static float simplex3(float x, float y, float z)
{
	const float F3 = 1.0f / 3.0f, G3 = 1.0f / 6.0f;
	float s = (x + y + z) * F3;
	int i = (int)floorf(x + s), j = (int)floorf(y + s), k = (int)floorf(z + s);
	float t = (float)(i + j + k) * G3;
	float x0 = x - ((float)i - t), y0 = y - ((float)j - t), z0 = z - ((float)k - t);
	int i1, j1, k1, i2, j2, k2;
	if (x0 >= y0) {
		if (y0 >= z0) { i1 = 1; j1 = 0; k1 = 0; i2 = 1; j2 = 1; k2 = 0; }
		else if (x0 >= z0) { i1 = 1; j1 = 0; k1 = 0; i2 = 1; j2 = 0; k2 = 1; }
		else { i1 = 0; j1 = 0; k1 = 1; i2 = 1; j2 = 0; k2 = 1; }
	} else {
		if (y0 < z0) { i1 = 0; j1 = 0; k1 = 1; i2 = 0; j2 = 1; k2 = 1; }
		else if (x0 < z0) { i1 = 0; j1 = 1; k1 = 0; i2 = 0; j2 = 1; k2 = 1; }
		else { i1 = 0; j1 = 1; k1 = 0; i2 = 1; j2 = 1; k2 = 0; }
	}
	float x1 = x0 - i1 + G3, y1 = y0 - j1 + G3, z1 = z0 - k1 + G3;
	float x2 = x0 - i2 + 2.0f * G3, y2 = y0 - j2 + 2.0f * G3, z2 = z0 - k2 + 2.0f * G3;
	float x3 = x0 - 1.0f + 3.0f * G3, y3 = y0 - 1.0f + 3.0f * G3, z3 = z0 - 1.0f + 3.0f * G3;
	int g0 = PH(i + PH(j + PH(k)));
	int g1 = PH(i + i1 + PH(j + j1 + PH(k + k1)));
	int g2 = PH(i + i2 + PH(j + j2 + PH(k + k2)));
	int g3 = PH(i + 1 + PH(j + 1 + PH(k + 1)));
	float n0 = corner_term(x0, y0, z0, g0), n1 = corner_term(x1, y1, z1, g1);
	float n2 = corner_term(x2, y2, z2, g2), n3 = corner_term(x3, y3, z3, g3);
	return 32.0f * (n0 + n1 + n2 + n3);
}

/* ---- textures, material.c:152-200 ---- */
static void texture_color(const rtx_material *m, const float *p, int u32mode, float *out)
{
	float sp[3];
	switch (m->texture) {
	case RTX_TEX_UNIFORM:
		assign3(out, m->color[0]);
		return;
	case RTX_TEX_CHECKERBOARD: {
		mul3s(p, m->scale, sp);
		uint32_t parity = (to_u32(sp[0], u32mode) + to_u32(sp[1], u32mode) + to_u32(sp[2], u32mode)) % 2u;
		assign3(out, m->color[parity]);
		return;
	}
	case RTX_TEX_BRICK: {
		mul3s(p, m->scale, sp);
		uint32_t parity = to_u32(sp[0], u32mode) % 2u;
		sp[1] -= parity * .5f;
		uint32_t mortar = (sp[0] - floorf(sp[0]) < m->mortar_width) || (sp[1] - floorf(sp[1]) < m->mortar_width);
		assign3(out, m->color[mortar]);
		return;
	}
	case RTX_TEX_NOISY_PERIODIC: {
		mul3s(p, m->noise_feature_scale, sp);
		float angle = (p[0] + simplex3(sp[0], sp[1], sp[2]) * m->noise_scale) * m->frequency_scale;
		float k = 0.f;
		switch (m->periodic) {
		case RTX_PERIODIC_SIN: k = (1.f + sinf(angle)) * .5f; break;
		case RTX_PERIODIC_SAW: k = angle - floorf(angle); break;
		case RTX_PERIODIC_TRIANGLE: k = fabsf(2.f * (angle - floorf(angle) - .5f)); break;
		case RTX_PERIODIC_SQUARE: k = (float)!signbit(sinf(angle)); break;
		}
		mul3s(m->color[1], k, out);
		add3v(out, m->color[0], out);
		return;
	}
	}
	out[0] = out[1] = out[2] = 0.f;
}

/* ---- primitives, object.c ---- */
typedef struct {
	v3 dir, point;
} ray_t;

/* line_intersects_sphere object.c:306-321 */
static int hit_sphere(const float *c, float r, const float *o, const float *d, float eps, float *t)
{
	v3 rel;
	sub3v(o, c, rel);
	float b = -dot3(d, rel);
	float cc = dot3(rel, rel) - sqr(r);
	float det = sqr(b) - cc;
	if (det < 0)
		return 0;
	float sq = sqrtf(det);
	*t = b - sq;
	if (*t > eps)
		return 1;
	*t = b + sq;
	return *t > eps;
}

/* moller_trumbore object.c:422-441 */
static int hit_triangle(const float *v0, const float *e1, const float *e2, const float *o, const float *d, float eps,
			float *t)
{
	v3 h, s, q;
	cross(d, e2, h);
	float a = dot3(e1, h);
	if (a < eps && a > -eps)
		return 0;
	float f = 1.f / a;
	sub3v(o, v0, s);
	float u = f * dot3(s, h);
	if (u < 0.f || u > 1.f)
		return 0;
	cross(s, e1, q);
	float v = f * dot3(d, q);
	if (v < 0.f || u + v > 1.f)
		return 0;
	*t = f * dot3(e2, q);
	return *t > eps;
}

/* plane_get_intersection object.c:473-488 (also *_intersects_in_range 490-498) */
static int hit_plane(const float *n, float dd, const float *o, const float *d, float eps, float *t)
{
	float a = dot3(n, d);
	if (fabsf(a) < eps)
		return 0;
	*t = (dd - dot3(n, o)) / dot3(n, d);
	return *t > eps;
}

static int obj_intersect(const rtx_object *ob, const ray_t *r, float *t, float *n)
{
	switch (ob->type) {
	case RTX_SPHERE:
		if (hit_sphere(ob->p0, ob->radius, r->point, r->dir, ob->epsilon, t)) {
			if (n) {
				mul3s(r->dir, *t, n);
				add3v(n, r->point, n);
				sub3v(n, ob->p0, n);
				mul3s(n, 1.f / ob->radius, n);
			}
			return 1;
		}
		return 0;
	case RTX_TRIANGLE:
		if (hit_triangle(ob->p0, ob->e1, ob->e2, r->point, r->dir, ob->epsilon, t)) {
			if (n)
				assign3(n, ob->n);
			return 1;
		}
		return 0;
	default:
		if (hit_plane(ob->n, ob->d, r->point, r->dir, ob->epsilon, t)) {
			if (n) {
				if (signbit(dot3(ob->n, r->dir)))
					assign3(n, ob->n);
				else
					mul3s(ob->n, -1.f, n);
			}
			return 1;
		}
		return 0;
	}
}

/* sphere_get_light_point object.c:293-304; triangle_get_light_point 403-419 */
static void light_point(const rtx_object *e, const float *p, float u1, float u2, float *out)
{
	if (e->type == RTX_SPHERE) {
		v3 nrm;
		sub3v(e->p0, p, nrm);
		float inc = u1 * 2.f * PI, az = u2 * 2.f * PI;
		v3 ld = { e->radius * cosf(az) * sinf(inc), e->radius * sinf(az) * sinf(inc), e->radius * cosf(inc) };
		if (dot3(nrm, ld))
			mul3s(ld, -1.f, ld);
		add3v(e->p0, ld, out);
	} else {
		float pp = u1, q = u2;
		if (pp + q > 1.f) {
			pp = 1.f - pp;
			q = 1.f - q;
		}
		for (int i = 0; i < 3; i++)
			out[i] = e->p0[i] + (e->p1[i] - e->p0[i]) * pp + (e->p2[i] - e->p0[i]) * q;
	}
}

/* ---- BVH, accel.c ---- */
typedef struct {
	float eps;
	v3 lo, hi;
} cuboid;

typedef struct {
	cuboid box;
	int32_t leaf;   /* object index, or -1 */
	int32_t c[2];   /* children */
} bnode;

typedef struct {
	uint32_t code;
	int32_t node;
} leaf_code;

typedef struct {
	const rtx_scene_desc *sc;
	bnode *nodes;
	int32_t n_nodes;
	int32_t root;
	int32_t *planes;
	uint32_t n_planes;
} oscene;

/* accel.c:72-88 */
static uint32_t expand_bits(uint32_t n)
{
	n = (n * 0x00010001u) & 0xFF0000FFu;
	n = (n * 0x00000101u) & 0x0F00F00Fu;
	n = (n * 0x00000011u) & 0xC30C30C3u;
	n = (n * 0x00000005u) & 0x49249249u;
	return n;
}
static uint32_t morton(const float *v)
{
	return expand_bits((uint32_t)(1023.f * v[0])) * 4u + expand_bits((uint32_t)(1023.f * v[1])) * 2u +
	       expand_bits((uint32_t)(1023.f * v[2]));
}

/* bounding_cuboid_intersects accel.c:112-158 */
static int slab(const cuboid *c, const ray_t *r, float *tmax, float *tmin)
{
	float tymin, tymax, tzmin, tzmax;
	float divx = 1 / r->dir[0];
	if (divx >= 0) {
		*tmin = (c->lo[0] - r->point[0]) * divx;
		*tmax = (c->hi[0] - r->point[0]) * divx;
	} else {
		*tmin = (c->hi[0] - r->point[0]) * divx;
		*tmax = (c->lo[0] - r->point[0]) * divx;
	}
	float divy = 1 / r->dir[1];
	if (divy >= 0) {
		tymin = (c->lo[1] - r->point[1]) * divy;
		tymax = (c->hi[1] - r->point[1]) * divy;
	} else {
		tymin = (c->hi[1] - r->point[1]) * divy;
		tymax = (c->lo[1] - r->point[1]) * divy;
	}
	if ((*tmin > tymax) || (tymin > *tmax))
		return 0;
	if (tymin > *tmin)
		*tmin = tymin;
	if (tymax < *tmax)
		*tmax = tymax;
	float divz = 1 / r->dir[2];
	if (divz >= 0) {
		tzmin = (c->lo[2] - r->point[2]) * divz;
		tzmax = (c->hi[2] - r->point[2]) * divz;
	} else {
		tzmin = (c->hi[2] - r->point[2]) * divz;
		tzmax = (c->lo[2] - r->point[2]) * divz;
	}
	if (*tmin > tzmax || tzmin > *tmax)
		return 0;
	if (tzmin > *tmin)
		*tmin = tzmin;
	if (tzmax < *tmax)
		*tmax = tzmax;
	return *tmax > c->eps;
}

static void obj_corners(const rtx_object *o, float *lo, float *hi)
{
	if (o->type == RTX_SPHERE) { /* sphere_get_corners object.c:277-282 */
		for (int j = 0; j < 3; j++) {
			lo[j] = o->p0[j] - o->radius;
			hi[j] = o->p0[j] + o->radius;
		}
	} else { /* triangle_get_corners object.c:375-388 */
		const float *v[3] = { o->p0, o->p1, o->p2 };
		assign3(lo, v[2]);
		assign3(hi, v[2]);
		for (int i = 0; i < 2; i++)
			for (int j = 0; j < 3; j++) {
				if (lo[j] > v[i][j])
					lo[j] = v[i][j];
				else if (hi[j] < v[i][j])
					hi[j] = v[i][j];
			}
	}
}

/* stable merge sort by Morton code (glibc 2.35 qsort is a merge sort) */
static void sort_codes(leaf_code *a, leaf_code *tmp, size_t n)
{
	if (n < 2)
		return;
	size_t h = n / 2;
	sort_codes(a, tmp, h);
	sort_codes(a + h, tmp, n - h);
	size_t i = 0, j = h, k = 0;
	while (i < h && j < n) {
		/* bvh_morton_code_compare accel.c:183-186 */
		if ((int)a[j].code - (int)a[i].code < 0)
			tmp[k++] = a[j++];
		else
			tmp[k++] = a[i++];
	}
	while (i < h)
		tmp[k++] = a[i++];
	while (j < n)
		tmp[k++] = a[j++];
	memcpy(a, tmp, n * sizeof(*a));
}

/* bvh_generate_node accel.c:227-264 */
static int32_t gen_node(oscene *s, const leaf_code *lc, size_t first, size_t last)
{
	if (first == last)
		return lc[first].node;
	uint32_t fc = lc[first].code, lcod = lc[last].code;
	size_t split;
	if (fc == lcod) {
		split = (first + last) / 2;
	} else {
		split = first;
		uint32_t common = (uint32_t)__builtin_clz(fc ^ lcod);
		size_t step = last - first;
		do {
			step = (step + 1) >> 1;
			size_t ns = split + step;
			if (ns < last) {
				uint32_t sc = lc[ns].code;
				if (fc ^ sc) {
					uint32_t pre = (uint32_t)__builtin_clz(fc ^ sc);
					if (pre > common)
						split = ns;
				}
			}
		} while (step > 1);
	}
	int32_t l = gen_node(s, lc, first, split);
	int32_t r = gen_node(s, lc, split + 1, last);
	int32_t id = s->n_nodes++;
	bnode *b = &s->nodes[id];
	const cuboid *L = &s->nodes[l].box, *R = &s->nodes[r].box;
	b->box.eps = fmaxf(L->eps, R->eps);
	for (int j = 0; j < 3; j++) {
		b->box.lo[j] = fminf(L->lo[j], R->lo[j]);
		b->box.hi[j] = fmaxf(L->hi[j], R->hi[j]);
	}
	b->leaf = -1;
	b->c[0] = l;
	b->c[1] = r;
	return id;
}

/* accel_init accel.c:266-315 */
static int build_scene(oscene *s, const rtx_scene_desc *sc)
{
	memset(s, 0, sizeof(*s));
	s->sc = sc;
	uint32_t nb = 0;
	for (uint32_t i = 0; i < sc->num_objects; i++)
		if (sc->objects[i].type == RTX_PLANE)
			s->n_planes++;
		else
			nb++;
	s->planes = malloc(sizeof(int32_t) * (s->n_planes + 1));
	s->nodes = malloc(sizeof(bnode) * (2 * (size_t)nb + 1));
	leaf_code *lc = malloc(sizeof(leaf_code) * (nb + 1)), *tmp = malloc(sizeof(leaf_code) * (nb + 1));
	if (!s->planes || !s->nodes || !lc || !tmp)
		return RTX_ERR_NOMEM;
	uint32_t np = 0;
	float mn[3] = { FLT_MAX, FLT_MAX, FLT_MAX }, mx[3] = { FLT_MIN, FLT_MIN, FLT_MIN };
	for (uint32_t i = 0; i < sc->num_objects; i++) {
		const rtx_object *o = &sc->objects[i];
		if (o->type == RTX_PLANE) {
			s->planes[np++] = (int32_t)i;
			continue;
		}
		bnode *b = &s->nodes[s->n_nodes];
		obj_corners(o, b->box.lo, b->box.hi);
		b->box.eps = o->epsilon;
		b->leaf = (int32_t)i;
		lc[s->n_nodes].node = s->n_nodes;
		s->n_nodes++;
		/* get_objects_extents object.c:200-225 */
		for (int j = 0; j < 3; j++) {
			if (b->box.lo[j] < mn[j])
				mn[j] = b->box.lo[j];
			if (b->box.hi[j] > mx[j])
				mx[j] = b->box.hi[j];
		}
	}
	s->root = -1;
	if (nb) {
		v3 mul;
		sub3v(mx, mn, mul);
		mul[0] = 1.f / mul[0];
		mul[1] = 1.f / mul[1];
		mul[2] = 1.f / mul[2];
		mul3s(mul, 0.5f, mul);
		mul3s(mn, 2.f, mn);
		for (uint32_t i = 0; i < nb; i++) {
			const cuboid *c = &s->nodes[i].box;
			v3 np3;
			add3v(c->lo, c->hi, np3);
			mul3v(np3, mul, np3);
			sub3v(np3, mn, np3);
			lc[i].code = morton(np3);
		}
		sort_codes(lc, tmp, nb);
		s->root = gen_node(s, lc, 0, nb - 1);
	}
	free(lc);
	free(tmp);
	return RTX_OK;
}

static void free_scene(oscene *s)
{
	free(s->nodes);
	free(s->planes);
}

typedef struct {
	uint64_t closest, shadow;
} counters;

typedef struct {
	const oscene *s;
	const rtx_params *p;
	counters cnt;
} tctx;

/* bvh_get_closest_intersection accel.c:322-353 */
static void bvh_closest(const oscene *s, int32_t id, const ray_t *r, int32_t *obj, float *n, float *dist)
{
	const bnode *b = &s->nodes[id];
	if (b->leaf >= 0) {
		v3 nn;
		float t;
		if (obj_intersect(&s->sc->objects[b->leaf], r, &t, nn) && t < *dist) {
			*dist = t;
			*obj = b->leaf;
			assign3(n, nn);
		}
		return;
	}
	float tl, tr, tmax;
	int il = slab(&s->nodes[b->c[0]].box, r, &tmax, &tl) && tl < *dist;
	int ir = slab(&s->nodes[b->c[1]].box, r, &tmax, &tr) && tr < *dist;
	if (il && ir) {
		if (tl < tr) {
			bvh_closest(s, b->c[0], r, obj, n, dist);
			bvh_closest(s, b->c[1], r, obj, n, dist);
		} else {
			bvh_closest(s, b->c[1], r, obj, n, dist);
			bvh_closest(s, b->c[0], r, obj, n, dist);
		}
	} else if (il) {
		bvh_closest(s, b->c[0], r, obj, n, dist);
	} else if (ir) {
		bvh_closest(s, b->c[1], r, obj, n, dist);
	}
}

/* bvh_is_light_blocked accel.c:360-387 */
static int bvh_blocked(const oscene *s, int32_t id, const ray_t *r, float dist, float *li, int32_t emitter)
{
	const bnode *b = &s->nodes[id];
	float tmin, tmax;
	if (b->leaf >= 0) {
		if (b->leaf == emitter)
			return 0;
		const rtx_object *o = &s->sc->objects[b->leaf];
		if (obj_intersect(o, r, &tmin, NULL) && tmin < dist) {
			const rtx_material *m = &s->sc->materials[o->material];
			if (m->transparent)
				mul3v(li, m->kt, li);
			else
				return 1;
		}
		return 0;
	}
	for (int i = 0; i < 2; i++)
		if (slab(&s->nodes[b->c[i]].box, r, &tmax, &tmin) && tmin < dist &&
		    bvh_blocked(s, b->c[i], r, dist, li, emitter))
			return 1;
	return 0;
}

/* get_closest_intersection render.c:118-124 + unbound_objects_get_closest_intersection object.c:168-181 */
static void closest(const oscene *s, const ray_t *r, int32_t *obj, float *n, float *dist)
{
	for (uint32_t i = 0; i < s->n_planes; i++) {
		float t;
		v3 nn;
		if (obj_intersect(&s->sc->objects[s->planes[i]], r, &t, nn) && t < *dist) {
			*dist = t;
			*obj = s->planes[i];
			assign3(n, nn);
		}
	}
	if (s->root >= 0)
		bvh_closest(s, s->root, r, obj, n, dist);
}

/* is_light_blocked render.c:126-134 + unbound_objects_is_light_blocked object.c:183-197 */
static int blocked(const oscene *s, const ray_t *r, float dist, float *li, int32_t emitter)
{
	for (uint32_t i = 0; i < s->n_planes; i++) {
		const rtx_object *o = &s->sc->objects[s->planes[i]];
		float t;
		if (hit_plane(o->n, o->d, r->point, r->dir, o->epsilon, &t) && t < dist) {
			const rtx_material *m = &s->sc->materials[o->material];
			if (m->transparent)
				mul3v(li, m->kt, li);
			else
				return 1;
		}
	}
	return s->root >= 0 && bvh_blocked(s, s->root, r, dist, li, emitter);
}

static inline void draw2(const rtx_params *p, uint64_t key, uint32_t stream, uint32_t idx, float *u1, float *u2)
{
	if (p->rng == RTX_RNG_CONST) {
		*u1 = 0.5f;
		*u2 = 0.5f;
	} else {
		rtx_draw2(key, stream, idx, u1, u2);
	}
}

/* GI direction, render.c:240-281 */
static void gi_direction(const float *n, float eps, float u1, float u2, float *dir)
{
	float R[3][3];
	if (n[1] - eps < -1.f) {
		float vx[3][3] = { { 1.f, 0.f, 0.f }, { 0.f, -1.f, 0.f }, { 0.f, 0.f, -1.f } };
		memcpy(R, vx, sizeof(R));
	} else {
		const v3 up = { 0.f, 1.f, 0.f };
		float mul = 1.f / (1.f + dot3(up, n));
		float vx[3][3] = {
			{ 1.f - sqr(n[0]) * mul, n[0], -n[0] * n[2] * mul },
			{ -n[0], 1.f - (sqr(n[0]) + sqr(n[2])) * mul, -n[2] },
			{ -n[0] * n[2] * mul, n[2], 1.f - sqr(n[2]) * mul },
		};
		memcpy(R, vx, sizeof(R));
	}
	float inc = acosf(u1 * 2.f - 1.f), az = u2 * PI;
	v3 v = { 1 * cosf(az) * sinf(inc), 1 * sinf(az) * sinf(inc), 1 * cosf(inc) };
	dir[0] = dot3(R[0], v);
	dir[1] = dot3(R[1], v);
	dir[2] = dot3(R[2], v);
}

/* refraction direction, render.c:320-335 */
static void refract_dir(const float *d, const float *n, float b, int outside, float ior, float *out)
{
	float inc = acosf(fabsf(b));
	float mult = outside ? 1.f / ior : ior;
	float refr = asinf(sinf(inc) * mult);
	float delta = refr - inc;
	v3 c, f, g, h;
	cross(d, n, c);
	norm3(c);
	if (!outside)
		mul3s(c, -1.f, c);
	cross(c, d, f);
	mul3s(d, cosf(delta), g);
	mul3s(f, sinf(delta), h);
	add3v(g, h, out);
	norm3(out);
}

static inline float atten_factor(const rtx_params *p, float dist)
{
	switch (p->attenuation) {
	case RTX_ATT_LIN:
		return 1.f / (p->attenuation_offset + dist);
	case RTX_ATT_SQR:
		return 1.f / sqr(p->attenuation_offset + dist);
	default:
		return 1.f;
	}
}

/* cast_ray render.c:136-343 */
static float cast_ray(tctx *T, const ray_t *ray, const float *kr, float *color, uint32_t rb, int32_t inside, uint64_t key)
{
	const oscene *s = T->s;
	const rtx_params *P = T->p;
	const rtx_scene_desc *sc = s->sc;
	int32_t obj = -1;
	v3 normal;
	float tmin;
	T->cnt.closest++;

	if (inside >= 0 && obj_intersect(&sc->objects[inside], ray, &tmin, normal)) {
		obj = inside;
	} else {
		tmin = FLT_MAX;
		closest(s, ray, &obj, normal, &tmin);
	}
	if (obj < 0)
		return 0.f;

	ray_t out;
	mul3s(ray->dir, tmin, out.point);
	add3v(out.point, ray->point, out.point);

	const rtx_object *ob = &sc->objects[obj];
	const rtx_material *m = &sc->materials[ob->material];
	v3 oc;
	assign3(oc, m->ke);
	float b = dot3(normal, ray->dir);
	int outside = signbit(b) != 0;

	v3 tex;
	int have_tex = 0;
	for (uint32_t i = 0; i < sc->num_emitters; i++) {
		int32_t ei = (int32_t)sc->emitters[i];
		if (ei == obj)
			continue;
		const rtx_object *e = &sc->objects[ei];
		v3 li;
		mul3s(sc->materials[e->material].ke, 1.f / e->num_lights, li);
		for (uint32_t j = 0; j < e->num_lights; j++) {
			v3 lp, inl;
			float u1, u2;
			draw2(P, key, i, j, &u1, &u2);
			if (P->rng == RTX_RNG_STRAT) /* stratified light samples (include/rtx.h RTX_RNG_STRAT) */
				u1 = ((float)j + u1) / (float)e->num_lights;
			light_point(e, out.point, u1, u2, lp);
			assign3(inl, li);
			sub3v(lp, out.point, out.dir);
			float ldist = mag3(out.dir);
			mul3s(out.dir, 1.f / ldist, out.dir);
			float a = dot3(out.dir, normal);
			if (!outside)
				continue;
			T->cnt.shadow++;
			if (blocked(s, &out, ldist, inl, ei))
				continue;
			v3 dv;
			sub3v(lp, out.point, dv);
			if (P->attenuation == RTX_ATT_LIN)
				mul3s(inl, 1.f / (P->attenuation_offset + mag3(dv)), inl);
			else if (P->attenuation == RTX_ATT_SQR)
				mul3s(inl, 1.f / (P->attenuation_offset + magsqr3(dv)), inl);
			if (!have_tex) {
				texture_color(m, out.point, P->u32conv, tex);
				have_tex = 1;
			}
			v3 diff, refl, spec;
			mul3v(tex, inl, diff);
			mul3s(diff, fmaxf(0.f, a), diff);
			float sm;
			if (P->reflection == RTX_BLINN) {
				mul3s(out.dir, -1.f, refl);
				add3v(refl, ray->dir, refl);
				norm3(refl);
				sm = -dot3(normal, refl);
			} else {
				mul3s(normal, 2 * a, refl);
				sub3v(refl, out.dir, refl);
				sm = -dot3(refl, ray->dir);
			}
			mul3v(m->ks, inl, spec);
			mul3s(spec, fmaxf(0.f, powf(sm, m->shininess)), spec);
			for (int k = 0; k < 3; k++)
				oc[k] = oc[k] + diff[k] + spec[k];
		}
	}

	if (P->gi == RTX_GI_AMBIENT) {
		v3 amb;
		mul3v(m->ka, sc->ambient, amb);
		add3v(oc, amb, oc);
	} else if (rb && outside) {
		v3 delta = { 1.f, 1.f, 1.f };
		uint32_t ns;
		if (rb == P->max_bounces) {
			ns = P->samples;
			mul3s(delta, 1.f / (float)ns, delta);
		} else {
			ns = 1;
		}
		for (uint32_t i = 0; i < ns; i++) {
			float u1, u2;
			draw2(P, key, RTX_STREAM_GI, i, &u1, &u2);
			gi_direction(normal, ob->epsilon, u1, u2, out.dir);
			v3 lm;
			mul3s(delta, dot3(normal, out.dir), lm);
			cast_ray(T, &out, lm, oc, 0, -1, rtx_key_child(key, RTX_CHILD_GI0 + i));
		}
	}

	mul3v(oc, kr, oc);
	if (P->attenuation != RTX_ATT_NONE)
		mul3s(oc, atten_factor(P, tmin), oc);
	add3v(color, oc, color);

	if (!rb)
		return 0.f;

	if (inside != obj && m->reflective) {
		v3 rkr;
		mul3v(kr, m->kr, rkr);
		if (P->min_intensity_sqr < magsqr3(rkr)) {
			mul3s(normal, 2 * b, out.dir);
			sub3v(ray->dir, out.dir, out.dir);
			cast_ray(T, &out, rkr, color, rb - 1, -1, rtx_key_child(key, RTX_CHILD_REFLECT));
		}
	}
	if (m->transparent) {
		v3 rkt;
		mul3v(kr, m->kt, rkt);
		if (P->min_intensity_sqr < magsqr3(rkt)) {
			refract_dir(ray->dir, normal, b, outside, m->refractive_index, out.dir);
			cast_ray(T, &out, rkt, color, rb - 1, obj, rtx_key_child(key, RTX_CHILD_REFRACT));
		}
	}
	return tmin;
}

void rtx_oracle_params_default(rtx_params *p)
{
	memset(p, 0, sizeof(*p));
	p->max_bounces = 10;
	p->min_intensity_sqr = .01f * .01f;
	p->reflection = RTX_PHONG;
	p->gi = RTX_GI_AMBIENT;
	p->samples = 1;
	p->attenuation = RTX_ATT_SQR;
	p->attenuation_offset = 1.f;
	p->rng = RTX_RNG_COUNTER;
	p->seed = 1;
	p->u32conv = RTX_U32_SAT;
	p->tile_offset = 0;
	p->tile_stride = 1;
}

/*
 * render() render.c:345-368 over the tiles t (8x8 px, row-major) with
 * t % tile_stride == tile_offset.  rgb/z are written for those pixels only
 * (rgb overwritten, not accumulated).  counts[0] = cast_ray calls,
 * counts[1] = is_light_blocked calls.  threads <= 0: OpenMP default.
 */
int rtx_oracle_render(const rtx_scene_desc *sc, const rtx_frame *fr, const rtx_params *p, float *rgb, float *z,
		      uint64_t counts[2], int threads)
{
	if (!sc || !fr || !p || !fr->width || !fr->height || !p->tile_stride)
		return RTX_ERR_ARG;
	oscene s;
	int rc = build_scene(&s, sc);
	if (rc) {
		free_scene(&s);
		return rc;
	}
	const uint32_t W = fr->width, H = fr->height;
	const uint32_t tiles_x = (W + 7) / 8, tiles_y = (H + 7) / 8;
	const int64_t ntiles = (int64_t)tiles_x * tiles_y;
	uint64_t c0 = 0, c1 = 0;
	const int nt = threads > 0 ? threads : omp_get_max_threads();
#pragma omp parallel num_threads(nt) reduction(+ : c0, c1)
	{
		tctx T = { &s, p, { 0, 0 } };
#pragma omp for schedule(dynamic, 1)
		for (int64_t t = 0; t < ntiles; t++) {
			if ((uint64_t)t % p->tile_stride != p->tile_offset)
				continue;
			uint32_t tx = (uint32_t)(t % tiles_x), ty = (uint32_t)(t / tiles_x);
			for (uint32_t row = ty * 8; row < ty * 8 + 8 && row < H; row++) {
				/* render.c:353-363: P = corner + row*vy, then += vx before each column */
				v3 pp;
				mul3s(fr->step_y, (float)row, pp);
				add3v(pp, fr->corner, pp);
				for (uint32_t col = 0; col < tx * 8; col++)
					add3v(pp, fr->step_x, pp);
				for (uint32_t col = tx * 8; col < tx * 8 + 8 && col < W; col++) {
					add3v(pp, fr->step_x, pp);
					ray_t r;
					assign3(r.point, fr->origin);
					sub3v(pp, fr->origin, r.dir);
					norm3(r.dir);
					const v3 kr = { 1.f, 1.f, 1.f };
					v3 color = { 0.f, 0.f, 0.f };
					uint32_t px = row * W + col;
					float zz = cast_ray(&T, &r, kr, color, p->max_bounces, -1, rtx_key_pixel(p->seed, px));
					if (rgb)
						assign3(rgb + (size_t)px * 3, color);
					if (z)
						z[px] = zz;
				}
			}
		}
		c0 += T.cnt.closest;
		c1 += T.cnt.shadow;
	}
	if (counts) {
		counts[0] = c0;
		counts[1] = c1;
	}
	free_scene(&s);
	return RTX_OK;
}

/*
 * The primary hits alone (render.c:353-363's rays, get_closest_intersection render.c:118-124): the
 * z-buffer render() writes for a frame with -b >= 1 (cast_ray returns the primary hit distance,
 * render.c:342; 0 on a miss), and the hit object's index (-1 on a miss).  Independent of the
 * light-sample stream, so a whole BASELINE frame's depth and hit mask can be checked at any spp.
 */
int rtx_oracle_primary(const rtx_scene_desc *sc, const rtx_frame *fr, float *z, int32_t *obj, int threads)
{
	if (!sc || !fr || !fr->width || !fr->height || !z)
		return RTX_ERR_ARG;
	oscene s;
	int rc = build_scene(&s, sc);
	if (rc) {
		free_scene(&s);
		return rc;
	}
	const uint32_t W = fr->width, H = fr->height;
	const int nt = threads > 0 ? threads : omp_get_max_threads();
#pragma omp parallel for num_threads(nt) schedule(dynamic, 4)
	for (int64_t row = 0; row < (int64_t)H; row++) {
		v3 pp;
		mul3s(fr->step_y, (float)row, pp);
		add3v(pp, fr->corner, pp);
		for (uint32_t col = 0; col < W; col++) {
			add3v(pp, fr->step_x, pp);
			ray_t r;
			assign3(r.point, fr->origin);
			sub3v(pp, fr->origin, r.dir);
			norm3(r.dir);
			int32_t o = -1;
			v3 n;
			float t = FLT_MAX;
			closest(&s, &r, &o, n, &t);
			const size_t px = (size_t)row * W + col;
			z[px] = o >= 0 ? t : 0.f;
			if (obj)
				obj[px] = o;
		}
	}
	free_scene(&s);
	return RTX_OK;
}

/* Per-function known answers (record layouts in rtx_kat.h). */
int rtx_oracle_kat(int kind, uint32_t n, const float *in, float *out, const rtx_params *p)
{
	if (kind < 0 || kind >= RTX_KAT_NKINDS || (n && (!in || !out)))
		return RTX_ERR_ARG;
	const int wi = rtx_kat_in_width[kind], wo = rtx_kat_out_width[kind];
	int u32mode = p ? p->u32conv : RTX_U32_SAT;
	for (uint32_t i = 0; i < n; i++) {
		const float *x = in + (size_t)i * wi;
		float *y = out + (size_t)i * wo;
		memset(y, 0, sizeof(float) * wo);
		switch (kind) {
		case RTX_KAT_MOLLER: {
			float t = 0.f;
			y[0] = (float)hit_triangle(x + 6, x + 9, x + 12, x, x + 3, x[15], &t);
			y[1] = y[0] ? t : 0.f;
		} break;
		case RTX_KAT_SPHERE: {
			rtx_object o;
			memset(&o, 0, sizeof(o));
			o.type = RTX_SPHERE;
			assign3(o.p0, x + 6);
			o.radius = x[9];
			o.epsilon = x[10];
			ray_t r;
			assign3(r.point, x);
			assign3(r.dir, x + 3);
			float t = 0.f;
			y[0] = (float)obj_intersect(&o, &r, &t, y + 2);
			y[1] = y[0] ? t : 0.f;
			if (!y[0])
				y[2] = y[3] = y[4] = 0.f;
		} break;
		case RTX_KAT_PLANE: {
			rtx_object o;
			memset(&o, 0, sizeof(o));
			o.type = RTX_PLANE;
			assign3(o.n, x + 6);
			o.d = x[9];
			o.epsilon = x[10];
			ray_t r;
			assign3(r.point, x);
			assign3(r.dir, x + 3);
			float t = 0.f;
			y[0] = (float)obj_intersect(&o, &r, &t, y + 2);
			y[1] = y[0] ? t : 0.f;
			if (!y[0])
				y[2] = y[3] = y[4] = 0.f;
		} break;
		case RTX_KAT_SLAB: {
			cuboid c;
			assign3(c.lo, x + 6);
			assign3(c.hi, x + 9);
			c.eps = x[12];
			ray_t r;
			assign3(r.point, x);
			assign3(r.dir, x + 3);
			float tmin = 0.f, tmax = 0.f;
			y[0] = (float)slab(&c, &r, &tmax, &tmin);
			y[1] = y[0] ? tmin : 0.f;
			y[2] = y[0] ? tmax : 0.f;
		} break;
		case RTX_KAT_NOISE:
			y[0] = simplex3(x[0], x[1], x[2]);
			break;
		case RTX_KAT_TEXTURE: {
			rtx_material m;
			memset(&m, 0, sizeof(m));
			m.texture = (int32_t)x[0];
			m.periodic = (int32_t)x[1];
			assign3(m.color[0], x + 2);
			assign3(m.color[1], x + 5);
			m.scale = x[8];
			m.mortar_width = x[9];
			m.noise_feature_scale = x[10];
			m.noise_scale = x[11];
			m.frequency_scale = x[12];
			texture_color(&m, x + 13, u32mode, y);
		} break;
		case RTX_KAT_SPH_LIGHT: {
			rtx_object o;
			memset(&o, 0, sizeof(o));
			o.type = RTX_SPHERE;
			assign3(o.p0, x);
			o.radius = x[3];
			light_point(&o, x + 4, x[7], x[8], y);
		} break;
		case RTX_KAT_TRI_LIGHT: {
			rtx_object o;
			memset(&o, 0, sizeof(o));
			o.type = RTX_TRIANGLE;
			assign3(o.p0, x);
			assign3(o.p1, x + 3);
			assign3(o.p2, x + 6);
			light_point(&o, NULL, x[9], x[10], y);
		} break;
		case RTX_KAT_MORTON: {
			uint32_t c = morton(x);
			memcpy(y, &c, 4);
		} break;
		case RTX_KAT_U32: {
			uint32_t a = to_u32(x[0], RTX_U32_SAT), b = to_u32(x[0], RTX_U32_WRAP);
			memcpy(y, &a, 4);
			memcpy(y + 1, &b, 4);
		} break;
		case RTX_KAT_GI_DIR:
			gi_direction(x, x[3], x[4], x[5], y);
			break;
		case RTX_KAT_REFRACT: {
			float b = dot3(x + 3, x);
			refract_dir(x, x + 3, b, signbit(b) != 0, x[6], y);
		} break;
		case RTX_KAT_ANY_TRI: { /* the exact any-hit decision: moller_trumbore hit with t < tlim */
			float t = 0.f;
			int h = hit_triangle(x + 6, x + 9, x + 12, x, x + 3, x[15], &t);
			y[0] = (float)(h && t < x[16]);
		} break;
		case RTX_KAT_SPH_LIGHT_SH: { /* exact light_point; the device runs the fast-trig form */
			rtx_object o;
			memset(&o, 0, sizeof(o));
			o.type = RTX_SPHERE;
			assign3(o.p0, x);
			o.radius = x[3];
			light_point(&o, x + 4, x[7], x[8], y);
		} break;
		case RTX_KAT_SPEC_POW: /* render.c:224 fmaxf(0., powf(specular_mul, shininess)) */
			y[0] = fmaxf(0.f, powf(x[0], x[1]));
			break;
		case RTX_KAT_BOX_Q:
		case RTX_KAT_BOX_Q8: { /* the exact answer in double: does the segment (0, tlim) of the ray meet
				       * the (unquantised) box?  A conservative quantised test must say hit
				       * wherever this does (the frame fields are unused here). */
			double tn = 0.0, tf = x[18];
			for (int a = 0; a < 3 && tn <= tf; a++) {
				const double o = x[a], d = x[3 + a], lo = x[6 + a], hi = x[9 + a];
				if (d == 0.0) {
					if (o < lo || o > hi)
						tn = 1.0, tf = 0.0;
					continue;
				}
				double t0 = (lo - o) / d, t1 = (hi - o) / d;
				if (t0 > t1) {
					const double s = t0;
					t0 = t1;
					t1 = s;
				}
				tn = t0 > tn ? t0 : tn;
				tf = t1 < tf ? t1 : tf;
			}
			y[0] = y[1] = (float)(tn <= tf);
		} break;
		}
	}
	return RTX_OK;
}
