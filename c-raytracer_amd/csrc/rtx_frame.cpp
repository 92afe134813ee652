/*
 * The trees' frame (rtx_device.h DTreeFrame) and the leaf boxes taken in it.
 *
 * The reference bounds every object by its world-space box (sphere_get_corners /
 * triangle_get_corners, object.c:277-282, 375-388) and its BVH is built over those boxes
 * (accel.c:266-315).  A mesh loaded with a rotation (scene.c mesh_load -> object.c:548-562) has
 * axis-aligned faces only in its own frame: in world space a face's box is a slab of volume
 * around a tilted square, and the boxes of neighbouring faces overlap, so a ray meets many
 * boxes whose triangles it misses.  The BVHs here may instead be built over the boxes of the
 * objects in a rotated frame x' = R (x - c); a walk then transforms its ray once and tests the
 * same boxes it would test in world space, only tighter.  Which primitives are tested changes
 * (fewer), their tests do not: every primitive whose box a ray meets is still tested with the
 * reference's arithmetic in world space, and a primitive the ray hits always has its box met
 * (the boxes are conservative, below), so closest hits (up to exact ties) and any-hit answers
 * are the world-space trees' (tests/test_gpu_frame.py: bit-identical frames).
 *
 * The frame: among the identity and the frames of the scene's largest triangles (axes: the
 * triangle's shortest edge, the normal, and their cross product), the one of least total
 * surface area of the triangles' boxes over a fixed sample, if it saves at least a quarter of
 * the identity's (a rotated Menger sponge: 0.3; the dragon stand-in keeps the identity).
 *
 * Conservativeness: a walk computes x' and d' in float with fused multiply-adds from the float
 * R and c the device holds, within about 3 * 2^-24 (|x - c| + |t d|) of the exact image of the
 * ray point at parameter t.  Every leaf box is computed exactly (double) from the same float R
 * and c, rounded outward, and padded by RTX_FRAME_PAD times the scene's radius about c on top
 * of the world trees' own relative padding and one 16-bit quantisation step: ample for rays that
 * start within a few scene radii of c (shade points, the camera of any reference scene).  Rays
 * from farther away (a distant camera, a point far out on a plane) get a frame origin near c
 * computed in double (rtx_math.h tf_shift for closest hits, tf_point_at at the segment's other end
 * for shadow rays), so the padding covers them too.
 */
#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <functional>
#include <thread>
#include <vector>

#include "rtx_frame.h"

#define RTX_FRAME_PAD 4e-6     /* leaf-box padding for the ray transform, times the scene radius */
#define RTX_FRAME_SAMPLE 16384 /* objects the cost is sampled over (every k-th bounded object; its triangles) */
#define RTX_FRAME_CANDS 16     /* largest sampled triangles whose frames are tried */
#define RTX_FRAME_GAIN 0.75    /* a rotated frame must cost at most this fraction of the identity's */

/* host threads for the per-object loops: RTX_HOST_THREADS, else OMP_NUM_THREADS, else at most 16
 * (plain threads, not an OpenMP runtime: its first start-up cost ~0.3 s on a GPU box's host) */
static unsigned host_threads()
{
	for (const char *k : { "RTX_HOST_THREADS", "OMP_NUM_THREADS" })
		if (const char *v = getenv(k))
			if (atoi(v) > 0)
				return (unsigned)std::min(atoi(v), 256);
	return std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
}

/* f(begin, end, chunk) over [0, n) in contiguous chunks, one per thread, each of at least `grain`
 * items (serially when n < 2 grain) */
template <class F> static unsigned parallel_chunks(size_t n, F f, size_t grain = 16384)
{
	const unsigned t = n < 2 * grain ? 1u : (unsigned)std::min<size_t>(host_threads(), (n + grain - 1) / grain);
	if (t <= 1) {
		f((size_t)0, n, 0u);
		return 1;
	}
	std::vector<std::thread> th;
	unsigned k = 1;
	try {
		for (; k < t; k++)
			th.emplace_back(f, n * k / t, n * (k + 1) / t, k);
	} catch (...) { /* no more threads: the rest of the chunks on this one */
		for (; k < t; k++)
			f(n * k / t, n * (k + 1) / t, k);
	}
	f((size_t)0, n / t, 0u);
	for (auto &x : th)
		x.join();
	return t;
}

unsigned rtx_host_parallel(size_t n, const std::function<void(size_t, size_t, unsigned)> &f, size_t grain)
{
	return parallel_chunks(n, f, grain);
}

/* per-object boxes lo / hi (3 floats each) by box(k, l, h) and their union blo / bhi */
template <class B> static void boxes_and_union(size_t nb, float *lo, float *hi, float blo[3], float bhi[3], B box)
{
	std::vector<float> part(6 * 256);
	const unsigned t = parallel_chunks(nb, [&](size_t b, size_t e, unsigned c) {
		float P[6] = { FLT_MAX, FLT_MAX, FLT_MAX, -FLT_MAX, -FLT_MAX, -FLT_MAX }; /* the chunk's union, written once */
		for (size_t k = b; k < e; k++) {
			float *l = lo + 3 * k, *h = hi + 3 * k;
			box(k, l, h);
			for (int a = 0; a < 3; a++) {
				P[a] = std::min(P[a], l[a]);
				P[3 + a] = std::max(P[3 + a], h[a]);
			}
		}
		std::copy(P, P + 6, &part[6 * (size_t)c]);
	});
	for (int a = 0; a < 3; a++) {
		blo[a] = FLT_MAX;
		bhi[a] = -FLT_MAX;
	}
	for (unsigned c = 0; c < t; c++)
		for (int a = 0; a < 3; a++) {
			blo[a] = std::min(blo[a], part[6 * (size_t)c + a]);
			bhi[a] = std::max(bhi[a], part[6 * (size_t)c + 3 + a]);
		}
}

static double half_area(const double lo[3], const double hi[3])
{
	const double x = hi[0] - lo[0], y = hi[1] - lo[1], z = hi[2] - lo[2];
	return x * y + y * z + z * x;
}

/* sum of the sampled triangles' box half-areas in the frame with rows r; v: the sample's
 * vertices, 9 floats per triangle (gathered once, so the candidates do not chase the objects) */
static double frame_cost(const std::vector<float> &v, const double (*r)[3])
{
	double cost = 0;
	for (size_t t = 0; t < v.size(); t += 9) {
		const float *p[3] = { &v[t], &v[t + 3], &v[t + 6] };
		double lo[3] = { DBL_MAX, DBL_MAX, DBL_MAX }, hi[3] = { -DBL_MAX, -DBL_MAX, -DBL_MAX };
		for (int k = 0; k < 3; k++)
			for (int i = 0; i < 3; i++) {
				const double y = r[i][0] * p[k][0] + r[i][1] * p[k][1] + r[i][2] * p[k][2];
				lo[i] = std::min(lo[i], y);
				hi[i] = std::max(hi[i], y);
			}
		cost += half_area(lo, hi);
	}
	return cost;
}

static bool unit(double v[3])
{
	const double l = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
	if (!(l > 0) || !std::isfinite(l))
		return false;
	for (int i = 0; i < 3; i++)
		v[i] /= l;
	return true;
}

/* the frame of triangle o: rows u (its shortest edge), v = n x u, n (its normal) */
static bool tri_frame(const rtx_object &o, double r[3][3])
{
	double e[3][3];
	for (int i = 0; i < 3; i++) {
		e[0][i] = (double)o.p1[i] - o.p0[i];
		e[1][i] = (double)o.p2[i] - o.p0[i];
		e[2][i] = (double)o.p2[i] - o.p1[i];
	}
	double n[3] = { e[0][1] * e[1][2] - e[0][2] * e[1][1], e[0][2] * e[1][0] - e[0][0] * e[1][2],
			e[0][0] * e[1][1] - e[0][1] * e[1][0] };
	if (!unit(n))
		return false;
	int s = 0;
	double best = DBL_MAX;
	for (int k = 0; k < 3; k++) {
		const double l = e[k][0] * e[k][0] + e[k][1] * e[k][1] + e[k][2] * e[k][2];
		if (l < best) {
			best = l;
			s = k;
		}
	}
	double u[3];
	const double un = e[s][0] * n[0] + e[s][1] * n[1] + e[s][2] * n[2];
	for (int i = 0; i < 3; i++)
		u[i] = e[s][i] - un * n[i];
	if (!unit(u))
		return false;
	const double v[3] = { n[1] * u[2] - n[2] * u[1], n[2] * u[0] - n[0] * u[2], n[0] * u[1] - n[1] * u[0] };
	for (int i = 0; i < 3; i++) {
		r[0][i] = u[i];
		r[1][i] = v[i];
		r[2][i] = n[i];
	}
	return true;
}

double rtx_frame_choose(const rtx_scene_desc *sc, const std::vector<uint32_t> &bounded, const float world_lo[3],
			const float world_hi[3], DTreeFrame &F)
{
	memset(&F, 0, sizeof(F));
	for (int i = 0; i < 3; i++)
		F.r[i][i] = 1.f;
	/* the triangles among every stride-th bounded object (one pass over the sample, not the scene) */
	const size_t stride = (bounded.size() + RTX_FRAME_SAMPLE - 1) / RTX_FRAME_SAMPLE;
	std::vector<uint32_t> sample;
	for (size_t k = 0; k < bounded.size(); k += std::max<size_t>(stride, 1))
		if (sc->objects[bounded[k]].type == RTX_TRIANGLE)
			sample.push_back(bounded[k]);
	if (sample.size() < 16)
		return 1.0;
	/* candidates: the frames of the largest sampled triangles (ties: lower object index) */
	std::vector<std::pair<double, uint32_t>> by_area;
	std::vector<float> sv;
	sv.reserve(9 * sample.size());
	for (uint32_t oi : sample) {
		const rtx_object &o = sc->objects[oi];
		sv.insert(sv.end(), o.p0, o.p0 + 3);
		sv.insert(sv.end(), o.p1, o.p1 + 3);
		sv.insert(sv.end(), o.p2, o.p2 + 3);
		const double c[3] = { (double)o.e1[1] * o.e2[2] - (double)o.e1[2] * o.e2[1],
				      (double)o.e1[2] * o.e2[0] - (double)o.e1[0] * o.e2[2],
				      (double)o.e1[0] * o.e2[1] - (double)o.e1[1] * o.e2[0] };
		by_area.push_back({ -(c[0] * c[0] + c[1] * c[1] + c[2] * c[2]), oi });
	}
	std::sort(by_area.begin(), by_area.end());
	/* frame 0 the identity, frame k the k-th largest sampled triangle's (as the device holds it:
	 * float rows); each frame's cost summed by one thread in sample order (deterministic) */
	const size_t nc = std::min<size_t>(by_area.size(), RTX_FRAME_CANDS) + 1;
	std::vector<double> rs(9 * nc, 0.0), cost(nc, -1.0);
	for (int i = 0; i < 3; i++)
		rs[4 * i] = 1.0;
	for (size_t k = 1; k < nc; k++) {
		double r[3][3];
		if (!tri_frame(sc->objects[by_area[k - 1].second], r))
			continue;
		for (int i = 0; i < 3; i++)
			for (int j = 0; j < 3; j++)
				rs[9 * k + 3 * i + j] = (double)(float)r[i][j];
		cost[k] = 0.0;
	}
	cost[0] = 0.0;
	rtx_host_parallel(nc, [&](size_t b, size_t e, unsigned) {
		for (size_t k = b; k < e; k++)
			if (cost[k] == 0.0)
				cost[k] = frame_cost(sv, (const double(*)[3]) & rs[9 * k]);
	}, 1);
	const double c_id = cost[0];
	double c_best = c_id;
	size_t best = 0;
	for (size_t k = 1; k < nc; k++)
		if (cost[k] >= 0.0 && cost[k] < c_best) {
			c_best = cost[k];
			best = k;
		}
	double r_best[3][3];
	memcpy(r_best, &rs[9 * best], sizeof(r_best));
	if (!(c_id > 0) || !(c_best <= RTX_FRAME_GAIN * c_id))
		return 1.0;
	for (int i = 0; i < 3; i++) {
		F.c[i] = 0.5f * world_lo[i] + 0.5f * world_hi[i];
		for (int j = 0; j < 3; j++)
			F.r[i][j] = (float)r_best[i][j];
	}
	F.rotated = 1;
	return c_best / c_id;
}

/* the float next to f towards -inf / +inf (nextafterf by its bits; f not a NaN) */
static float next_down(float f)
{
	if (f == 0.f)
		return -FLT_TRUE_MIN;
	uint32_t b;
	memcpy(&b, &f, 4);
	if (b == 0xFF800000u) /* -inf */
		return f;
	b = f > 0.f ? b - 1 : b + 1;
	memcpy(&f, &b, 4);
	return f;
}
static float next_up(float f) { return -next_down(-f); }
/* the largest float <= x / least float >= x */
static float down(double x)
{
	const float f = (float)x;
	return (double)f > x ? next_down(f) : f;
}
static float up(double x)
{
	const float f = (float)x;
	return (double)f < x ? next_up(f) : f;
}

double rtx_frame_radius(const float world_lo[3], const float world_hi[3], const DTreeFrame &F)
{
	/* the largest |x - centre| component over the bounded objects' world box (centre c + cf): it
	 * holds every vertex and every sphere with its radius */
	double rad = 0;
	for (int i = 0; i < 3; i++) {
		const double ce = (double)F.c[i] + F.cf[i];
		rad = std::max(rad, std::max(fabs((double)world_lo[i] - ce), fabs((double)world_hi[i] - ce)));
	}
	return rad;
}

void rtx_frame_far(const float world_lo[3], const float world_hi[3], DTreeFrame &F)
{
	/* a rotated frame is centred on the objects (c); the world frame keeps c = 0 (its boxes are the
	 * world boxes) and names their centre in cf */
	for (int i = 0; i < 3; i++)
		F.cf[i] = F.rotated ? 0.f : 0.5f * world_lo[i] + 0.5f * world_hi[i];
	/* rounded up; a scene without bounded objects (an empty box, lo > hi) keeps rad 0 */
	const double rad = rtx_frame_radius(world_lo, world_hi, F);
	F.rad = std::isfinite(rad) ? std::nextafter((float)rad, FLT_MAX) : FLT_MAX;
}

void rtx_frame_box(const rtx_object &o, const DTreeFrame &F, double pad, float lo[3], float hi[3])
{
	double l[3], h[3];
	if (o.type == RTX_SPHERE) {
		for (int i = 0; i < 3; i++) {
			double y = 0, rn = 0;
			for (int j = 0; j < 3; j++) {
				y += (double)F.r[i][j] * ((double)o.p0[j] - F.c[j]);
				rn += (double)F.r[i][j] * F.r[i][j];
			}
			l[i] = y - o.radius * sqrt(rn);
			h[i] = y + o.radius * sqrt(rn);
		}
	} else {
		const float *p[3] = { o.p0, o.p1, o.p2 };
		for (int i = 0; i < 3; i++) {
			l[i] = DBL_MAX;
			h[i] = -DBL_MAX;
			for (int k = 0; k < 3; k++) {
				double y = 0;
				for (int j = 0; j < 3; j++)
					y += (double)F.r[i][j] * ((double)p[k][j] - F.c[j]);
				l[i] = std::min(l[i], y);
				h[i] = std::max(h[i], y);
			}
		}
	}
	/* the world trees' relative padding (rtx_world_box) and the transform's */
	for (int i = 0; i < 3; i++) {
		const double ext = std::max(h[0] - l[0], std::max(h[1] - l[1], h[2] - l[2]));
		lo[i] = down(l[i] - (fabs(l[i]) + ext) * 2e-6 - pad);
		hi[i] = up(h[i] + (fabs(h[i]) + ext) * 2e-6 + pad);
	}
}

double rtx_frame_pad(double radius) { return RTX_FRAME_PAD * radius; }

void rtx_frame_boxes(const rtx_scene_desc *sc, const std::vector<uint32_t> &bounded, const DTreeFrame &F, double pad,
		     float *lo, float *hi, float blo[3], float bhi[3])
{
	boxes_and_union(bounded.size(), lo, hi, blo, bhi,
			[&](size_t k, float *l, float *h) { rtx_frame_box(sc->objects[bounded[k]], F, pad, l, h); });
}

void rtx_world_box(const rtx_object &o, float lo[3], float hi[3])
{
	float l[3], h[3];
	for (int a = 0; a < 3; a++) {
		if (o.type == RTX_SPHERE) {
			l[a] = o.p0[a] - o.radius;
			h[a] = o.p0[a] + o.radius;
		} else {
			l[a] = std::min(o.p0[a], std::min(o.p1[a], o.p2[a]));
			h[a] = std::max(o.p0[a], std::max(o.p1[a], o.p2[a]));
		}
	}
	/* padded so the traversal's FMA slab test is conservative */
	const float ext = std::max(h[0] - l[0], std::max(h[1] - l[1], h[2] - l[2]));
	for (int a = 0; a < 3; a++) {
		lo[a] = l[a] - (std::fabs(l[a]) + ext) * 2e-6f - 1e-30f;
		hi[a] = h[a] + (std::fabs(h[a]) + ext) * 2e-6f + 1e-30f;
	}
}

void rtx_world_boxes(const rtx_scene_desc *sc, const std::vector<uint32_t> &bounded, float *lo, float *hi, float blo[3],
		     float bhi[3])
{
	boxes_and_union(bounded.size(), lo, hi, blo, bhi, [&](size_t k, float *l, float *h) { rtx_world_box(sc->objects[bounded[k]], l, h); });
}

extern "C" int rtx_tree_frame(const rtx_scene_desc *sc, int *rotated, float rot[9], float center[3], double *cost_ratio)
{
	if (!sc || !rotated || !rot || !center)
		return rtx_fail(RTX_ERR_ARG, "null argument");
	if (sc->num_objects && !sc->objects)
		return rtx_fail(RTX_ERR_ARG, "objects pointer is null");
	std::vector<uint32_t> bounded;
	for (uint32_t i = 0; i < sc->num_objects; i++)
		if (sc->objects[i].type == RTX_SPHERE || sc->objects[i].type == RTX_TRIANGLE)
			bounded.push_back(i);
	std::vector<float> bl(3 * bounded.size()), bh(3 * bounded.size());
	float lo[3], hi[3];
	rtx_world_boxes(sc, bounded, bl.data(), bh.data(), lo, hi);
	DTreeFrame F;
	const double ratio = rtx_frame_choose(sc, bounded, lo, hi, F);
	memcpy(rot, F.r, 36);
	memcpy(center, F.c, 12);
	if (cost_ratio)
		*cost_ratio = ratio;
	*rotated = F.rotated ? 1 : 0;
	return RTX_OK;
}
