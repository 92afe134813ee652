/*
 * ORACLE TEST INFRASTRUCTURE — not part of the product path.
 *
 * Known-answer generator: links the reference's own translation units
 * (everything under /root/reference/src/{core,raytracer} and lib except main.c,
 * built by oracle/Makefile with the Makefile.rt flags) and evaluates its hot-path
 * functions on seeded random records.  Output: for each kind, a header
 * (kind, n, in_width, out_width as int32) followed by n input records and n
 * output records (float32), in the layouts of include/rtx_kat.h.
 * tools/make_goldens.py turns this into tests/golden/kat.npz.
 *
 * The reference keeps its primitive structs private to object.c / accel.c; the
 * layout-compatible declarations below let us build instances directly.
 * rand() is fed from a queue (REF_KAT_RNG in ref_shim.h) so the light samplers
 * see chosen draws.
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "SimplexNoise.h"
#include "material.h"
#include "object.h"
#include "type.h"

/* object.c:25-44 layouts */
struct KSphere {
	struct Object object;
	v3 position;
	float radius;
};
struct KTriangle {
	struct Object object;
	v3 vertices[3];
	v3 edges[2];
	v3 normal;
};
struct KPlane {
	struct Object object;
	v3 normal;
	float d;
};
/* accel.c:25-28 */
struct KCuboid {
	float epsilon;
	v3 corners[2];
};

/* non-static reference functions not declared in its headers */
bool moller_trumbore(const v3 vertex, v3 edges[2], const v3 line_position, const v3 line_vector, const float epsilon,
		     float *distance);
bool sphere_get_intersection(const struct Object *object, const struct Ray *ray, float *distance, v3 normal);
bool plane_get_intersection(const struct Object *object, const struct Ray *ray, float *distance, v3 normal);
bool bounding_cuboid_intersects(const struct KCuboid *cuboid, const struct Ray *ray, float *tmax, float *tmin);
void sphere_get_light_point(const struct Object *object, const v3 point, v3 light_point);
void triangle_get_light_point(const struct Object *object, const v3 point, v3 light_point);
uint32_t morton_code(const v3 vec);

/* rand() queue for REF_KAT_RNG */
static int rq[2], rq_pos;
int rtx_kat_rand(void)
{
	return rq[rq_pos++ & 1];
}

static unsigned long long lcg = 0x243F6A8885A308D3ull;
static double urand(void)
{
	lcg = lcg * 6364136223846793005ull + 1442695040888963407ull;
	return (double)(lcg >> 11) * (1.0 / 9007199254740992.0);
}
static float frand(float lo, float hi)
{
	return (float)(lo + (hi - lo) * urand());
}
static void rdir(float *d)
{
	float n;
	do {
		d[0] = frand(-1, 1);
		d[1] = frand(-1, 1);
		d[2] = frand(-1, 1);
		n = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
	} while (n < 1e-4f || n > 1.f);
	n = 1.f / sqrtf(n);
	d[0] *= n;
	d[1] *= n;
	d[2] *= n;
}
static void draw_pair(float *u1, float *u2)
{
	rq[0] = (int)(urand() * RAND_MAX);
	rq[1] = (int)(urand() * RAND_MAX);
	rq_pos = 0;
	*u1 = rq[0] / (float)RAND_MAX;
	*u2 = rq[1] / (float)RAND_MAX;
}

static void emit(FILE *f, int kind, int n, int wi, int wo, const float *in, const float *out)
{
	int h[4] = { kind, n, wi, wo };
	fwrite(h, 4, 4, f);
	fwrite(in, 4, (size_t)n * wi, f);
	fwrite(out, 4, (size_t)n * wo, f);
}

int main(int argc, char **argv)
{
	const char *path = argc > 1 ? argv[1] : "kat.bin";
	const int N = argc > 2 ? atoi(argv[2]) : 4096;
	FILE *f = fopen(path, "wb");
	if (!f)
		return 1;
	float *in = calloc((size_t)N * 16, 4), *out = calloc((size_t)N * 5, 4);
	struct Material mat;
	memset(&mat, 0, sizeof(mat));

	/* 0 moller_trumbore: rays aimed near the triangle so hits and misses mix */
	for (int i = 0; i < N; i++) {
		float *x = in + i * 16, *y = out + i * 2;
		float v[3][3];
		for (int k = 0; k < 3; k++)
			for (int j = 0; j < 3; j++)
				v[k][j] = frand(-1, 1);
		v3 e[2];
		for (int j = 0; j < 3; j++) {
			e[0][j] = v[1][j] - v[0][j];
			e[1][j] = v[2][j] - v[0][j];
		}
		float o[3] = { frand(-3, 3), frand(-3, 3), frand(-3, 3) }, tgt[3], d[3];
		float a = frand(-0.2f, 1.1f), b = frand(-0.2f, 1.1f);
		for (int j = 0; j < 3; j++)
			tgt[j] = v[0][j] + e[0][j] * a + e[1][j] * b;
		for (int j = 0; j < 3; j++)
			d[j] = tgt[j] - o[j];
		float nn = 1.f / sqrtf(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
		for (int j = 0; j < 3; j++)
			d[j] *= nn;
		if (i % 7 == 0)
			rdir(d);
		float eps = (i % 3) ? 1e-4f : frand(0, 0.05f);
		memcpy(x, o, 12);
		memcpy(x + 3, d, 12);
		memcpy(x + 6, v[0], 12);
		memcpy(x + 9, e[0], 12);
		memcpy(x + 12, e[1], 12);
		x[15] = eps;
		float t = 0.f;
		y[0] = moller_trumbore(v[0], e, o, d, eps, &t);
		y[1] = y[0] ? t : 0.f;
	}
	emit(f, 0, N, 16, 2, in, out);

	/* 1 sphere_get_intersection */
	for (int i = 0; i < N; i++) {
		float *x = in + i * 11, *y = out + i * 5;
		struct KSphere s;
		memset(&s, 0, sizeof(s));
		for (int j = 0; j < 3; j++)
			s.position[j] = frand(-2, 2);
		s.radius = frand(0.1f, 1.5f);
		object_init(&s.object, &mat, (i % 4) ? s.radius * 0.0003f : frand(0, 0.1f), 0, OBJECT_SPHERE);
		struct Ray r;
		for (int j = 0; j < 3; j++)
			r.point[j] = (i % 5 == 0) ? s.position[j] + frand(-0.5f, 0.5f) * s.radius : frand(-4, 4);
		float tgt[3];
		for (int j = 0; j < 3; j++)
			tgt[j] = s.position[j] + frand(-1.3f, 1.3f) * s.radius;
		for (int j = 0; j < 3; j++)
			r.direction[j] = tgt[j] - r.point[j];
		float nn = 1.f / sqrtf(r.direction[0] * r.direction[0] + r.direction[1] * r.direction[1] +
				       r.direction[2] * r.direction[2]);
		for (int j = 0; j < 3; j++)
			r.direction[j] *= nn;
		memcpy(x, r.point, 12);
		memcpy(x + 3, r.direction, 12);
		memcpy(x + 6, s.position, 12);
		x[9] = s.radius;
		x[10] = s.object.epsilon;
		float t = 0.f;
		v3 n = { 0, 0, 0 };
		y[0] = sphere_get_intersection(&s.object, &r, &t, n);
		y[1] = y[0] ? t : 0.f;
		if (y[0])
			memcpy(y + 2, n, 12);
		else
			y[2] = y[3] = y[4] = 0.f;
	}
	emit(f, 1, N, 11, 5, in, out);

	/* 2 plane_get_intersection */
	for (int i = 0; i < N; i++) {
		float *x = in + i * 11, *y = out + i * 5;
		struct KPlane p;
		memset(&p, 0, sizeof(p));
		rdir(p.normal);
		if (i % 9 == 0) {
			p.normal[0] = 0.f;
			p.normal[1] = 1.f;
			p.normal[2] = 0.f;
		}
		p.d = frand(-3, 3);
		object_init(&p.object, &mat, (i % 3) ? 1e-6f : frand(0, 0.01f), 0, OBJECT_PLANE);
		struct Ray r;
		for (int j = 0; j < 3; j++)
			r.point[j] = frand(-4, 4);
		rdir(r.direction);
		if (i % 11 == 0) /* near-parallel */
			r.direction[1] = 0.f;
		memcpy(x, r.point, 12);
		memcpy(x + 3, r.direction, 12);
		memcpy(x + 6, p.normal, 12);
		x[9] = p.d;
		x[10] = p.object.epsilon;
		float t = 0.f;
		v3 n = { 0, 0, 0 };
		y[0] = plane_get_intersection(&p.object, &r, &t, n);
		y[1] = y[0] ? t : 0.f;
		if (y[0])
			memcpy(y + 2, n, 12);
		else
			y[2] = y[3] = y[4] = 0.f;
	}
	emit(f, 2, N, 11, 5, in, out);

	/* 3 bounding_cuboid_intersects */
	for (int i = 0; i < N; i++) {
		float *x = in + i * 13, *y = out + i * 3;
		struct KCuboid c;
		for (int j = 0; j < 3; j++) {
			float a = frand(-2, 2), b = frand(-2, 2);
			c.corners[0][j] = fminf(a, b);
			c.corners[1][j] = fmaxf(a, b);
		}
		c.epsilon = (i % 3) ? 1e-4f : frand(0, 0.5f);
		struct Ray r;
		for (int j = 0; j < 3; j++)
			r.point[j] = frand(-4, 4);
		rdir(r.direction);
		if (i % 13 == 0)
			r.direction[i % 3] = 0.f; /* axis-parallel: 1/0 = inf */
		memcpy(x, r.point, 12);
		memcpy(x + 3, r.direction, 12);
		memcpy(x + 6, c.corners[0], 12);
		memcpy(x + 9, c.corners[1], 12);
		x[12] = c.epsilon;
		float tmin = 0.f, tmax = 0.f;
		y[0] = bounding_cuboid_intersects(&c, &r, &tmax, &tmin);
		y[1] = y[0] ? tmin : 0.f;
		y[2] = y[0] ? tmax : 0.f;
	}
	emit(f, 3, N, 13, 3, in, out);

	/* 4 simplex_noise */
	for (int i = 0; i < N; i++) {
		float *x = in + i * 3;
		float sc = (i % 4 == 0) ? 100.f : 6.f;
		x[0] = frand(-sc, sc);
		x[1] = frand(-sc, sc);
		x[2] = frand(-sc, sc);
		out[i] = simplex_noise(x[0], x[1], x[2]);
	}
	emit(f, 4, N, 3, 1, in, out);

	/* 5 textures (all kinds, all periodic functions), points incl. negative coordinates */
	for (int i = 0; i < N; i++) {
		float *x = in + i * 16, *y = out + i * 3;
		memset(x, 0, 16 * 4);
		int type = i % 4, per = (i / 4) % 4;
		v3 c0 = { frand(0, 1), frand(0, 1), frand(0, 1) }, c1 = { frand(-0.5f, 1), frand(-0.5f, 1), frand(-0.5f, 1) };
		v3 cs[2];
		memcpy(cs[0], c0, 12);
		memcpy(cs[1], c1, 12);
		float scale = frand(0.5f, 6.f), mortar = frand(0.02f, 0.3f), nfs = frand(0.3f, 3.f), ns = frand(0.f, 1.f),
		      fs = frand(1.f, 20.f);
		v3 P = { frand(-8, 8), frand(-8, 8), frand(-8, 8) };
		struct Texture *t;
		if (type == 0)
			t = texture_uniform_new(c0);
		else if (type == 1)
			t = texture_checkerboard_new(cs, scale);
		else if (type == 2)
			t = texture_brick_new(cs, scale, mortar);
		else
			t = texture_noisy_periodic_new(c0, c1, nfs, ns, fs, (enum PeriodicFunction)per);
		x[0] = (float)type;
		x[1] = (float)per;
		memcpy(x + 2, c0, 12);
		memcpy(x + 5, c1, 12);
		x[8] = scale;
		x[9] = mortar;
		x[10] = nfs;
		x[11] = ns;
		x[12] = fs;
		memcpy(x + 13, P, 12);
		t->get_color(t, P, y);
		free(t);
	}
	emit(f, 5, N, 16, 3, in, out);

	/* 6 sphere_get_light_point */
	for (int i = 0; i < N; i++) {
		float *x = in + i * 9, *y = out + i * 3;
		struct KSphere s;
		memset(&s, 0, sizeof(s));
		for (int j = 0; j < 3; j++)
			s.position[j] = frand(-3, 3);
		s.radius = frand(0.1f, 2.f);
		object_init(&s.object, &mat, 1e-4f, 1, OBJECT_SPHERE);
		v3 P = { frand(-5, 5), frand(-5, 5), frand(-5, 5) };
		float u1, u2;
		draw_pair(&u1, &u2);
		memcpy(x, s.position, 12);
		x[3] = s.radius;
		memcpy(x + 4, P, 12);
		x[7] = u1;
		x[8] = u2;
		sphere_get_light_point(&s.object, P, y);
	}
	emit(f, 6, N, 9, 3, in, out);

	/* 7 triangle_get_light_point */
	for (int i = 0; i < N; i++) {
		float *x = in + i * 11, *y = out + i * 3;
		struct KTriangle t;
		memset(&t, 0, sizeof(t));
		for (int k = 0; k < 3; k++)
			for (int j = 0; j < 3; j++)
				t.vertices[k][j] = frand(-3, 3);
		object_init(&t.object, &mat, 1e-4f, 1, OBJECT_TRIANGLE);
		float u1, u2;
		draw_pair(&u1, &u2);
		memcpy(x, t.vertices, 36);
		x[9] = u1;
		x[10] = u2;
		v3 P = { 0, 0, 0 };
		triangle_get_light_point(&t.object, P, y);
	}
	emit(f, 7, N, 11, 3, in, out);

	/* 8 morton_code */
	for (int i = 0; i < N; i++) {
		float *x = in + i * 3;
		x[0] = frand(0, 1);
		x[1] = frand(0, 1);
		x[2] = frand(0, 1);
		if (i % 17 == 0)
			x[i % 3] = (i % 2) ? 1.f : 0.f;
		uint32_t c = morton_code(x);
		memcpy(out + i, &c, 4);
	}
	emit(f, 8, N, 3, 1, in, out);

	/* 9 float -> uint32_t as this build converts it (material.c:164) */
	for (int i = 0; i < N; i++) {
		volatile float v = (i % 3 == 0) ? frand(-3, 3) : frand(-5e9f, 5e9f);
		if (i < 8) {
			const float sp[8] = { -1.f, -0.5f, -1.5f, 0.f, 4294967040.f, 4294967296.f, -2147483648.f, 2.5f };
			v = sp[i];
		}
		in[i] = v;
		uint32_t a = (uint32_t)v;
		memcpy(out + 2 * i, &a, 4);
		memcpy(out + 2 * i + 1, &a, 4);
	}
	emit(f, 9, N, 1, 2, in, out);

	fclose(f);
	free(in);
	free(out);
	return 0;
}
