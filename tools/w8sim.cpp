/*
 * Development tool (not product, not a test): builds a scene's BVH2 and 8-wide shadow BVH exactly
 * as rtx_build_scene does, then simulates k_shadow's 8-wide walk (rtx_shadow.hip shadow_walk8)
 * on the CPU for sampled shadow rays to report tree shape and per-ray / per-wave work:
 * node visits, box tests, primitive tests, and, for packets of 64 light samples of one shade
 * point walking in lockstep, wave steps and leaf rounds.  Shade points are the primary hits of
 * sampled 1080p pixels and their -n 64 GI hits; light samples are i.i.d. like the library's
 * default RTX_RNG_COUNTER (W8SIM_STRAT=1: stratified like RTX_RNG_STRAT).  W8SIM_OCC=1 adds the
 * occluder-first tests (a cached opaque blocker tested before the walk).
 *   build: tools/w8sim.sh       run: tools/w8sim <scene.json> [base_dir] [points]
 */
#include <chrono>
#include <float.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <array>
#include <tuple>
#include <random>
#include <vector>

#include "bvh_build.h"
#include "rtx_frame.h"
#include "rtx_internal.h"
#include "rtx_quant.h"
#include "rtx_scene.h"

int rtx_fail(int code, const char *, ...) { return code; }

static float area3(const float *a, const float *b, const float *c)
{
	const float e1[3] = { b[0] - a[0], b[1] - a[1], b[2] - a[2] }, e2[3] = { c[0] - a[0], c[1] - a[1], c[2] - a[2] };
	const float x = e1[1] * e2[2] - e1[2] * e2[1], y = e1[2] * e2[0] - e1[0] * e2[2], z = e1[0] * e2[1] - e1[1] * e2[0];
	return 0.5f * sqrtf(x * x + y * y + z * z);
}

/* closest hit over planes and the BVH2 (float boxes), for camera-visible shade points */
struct Scene2 {
	const rtx_scene_desc *sc;
	const std::vector<DNode> *inner;
	const std::vector<DPrim> *prims;
	uint32_t nnodes, root;
};

static bool tri_hit(const DPrim &p, const double o[3], const double d[3], double &t)
{
	const double e1[3] = { p.b[0], p.b[1], p.b[2] }, e2[3] = { p.c[0], p.c[1], p.c[2] };
	const double h[3] = { d[1] * e2[2] - d[2] * e2[1], d[2] * e2[0] - d[0] * e2[2], d[0] * e2[1] - d[1] * e2[0] };
	const double aa = e1[0] * h[0] + e1[1] * h[1] + e1[2] * h[2];
	if (fabs(aa) < p.a[3])
		return false;
	const double f = 1 / aa, s[3] = { o[0] - p.a[0], o[1] - p.a[1], o[2] - p.a[2] };
	const double uu = f * (s[0] * h[0] + s[1] * h[1] + s[2] * h[2]);
	const double q[3] = { s[1] * e1[2] - s[2] * e1[1], s[2] * e1[0] - s[0] * e1[2], s[0] * e1[1] - s[1] * e1[0] };
	const double vv = f * (d[0] * q[0] + d[1] * q[1] + d[2] * q[2]);
	t = f * (e2[0] * q[0] + e2[1] * q[1] + e2[2] * q[2]);
	return uu >= 0 && vv >= 0 && uu + vv <= 1 && t > p.a[3];
}

static bool box_hit(const float lo[3], const float hi[3], const double o[3], const double inv[3], double tmax)
{
	double tn = 0, tf = tmax;
	for (int a = 0; a < 3; a++) {
		const double t0 = (lo[a] - o[a]) * inv[a], t1 = (hi[a] - o[a]) * inv[a];
		tn = std::max(tn, std::min(t0, t1));
		tf = std::min(tf, std::max(t0, t1));
	}
	return tn <= tf;
}

/* closest hit: t, the normal (unnormalised for triangles) */
static bool closest(const Scene2 &S, const double o[3], const double d[3], double &tbest, double n[3])
{
	tbest = 1e30;
	bool hit = false;
	for (uint32_t i = 0; i < S.sc->num_objects; i++) {
		const rtx_object &p = S.sc->objects[i];
		if (p.type != RTX_PLANE)
			continue;
		const double a = p.n[0] * d[0] + p.n[1] * d[1] + p.n[2] * d[2];
		if (fabs(a) < 1e-6)
			continue;
		const double t = (p.d - (p.n[0] * o[0] + p.n[1] * o[1] + p.n[2] * o[2])) / a;
		if (t > 1e-4 && t < tbest) {
			tbest = t;
			hit = true;
			for (int k = 0; k < 3; k++)
				n[k] = p.n[k];
		}
	}
	double inv[3];
	for (int a = 0; a < 3; a++)
		inv[a] = fabs(d[a]) > 1e-30 ? 1.0 / d[a] : copysign(1e30, d[a]);
	std::vector<uint32_t> stk{ S.root };
	while (!stk.empty()) {
		const uint32_t ref = stk.back();
		stk.pop_back();
		if (ref & RTX_REF_LEAF) {
			const uint32_t first = (ref & RTX_REF_OFF) / 64 - S.nnodes, cnt = (ref & RTX_REF_CNT) + 1;
			for (uint32_t k = first; k < first + cnt; k++) {
				const DPrim &p = (*S.prims)[k];
				uint32_t meta;
				memcpy(&meta, &p.c[3], 4);
				if ((meta >> 24) == RTX_SPHERE)
					continue;
				double t;
				if (tri_hit(p, o, d, t) && t < tbest) {
					tbest = t;
					hit = true;
					n[0] = p.b[1] * p.c[2] - p.b[2] * p.c[1];
					n[1] = p.b[2] * p.c[0] - p.b[0] * p.c[2];
					n[2] = p.b[0] * p.c[1] - p.b[1] * p.c[0];
				}
			}
			continue;
		}
		const DNode &nd = (*S.inner)[(ref & RTX_REF_OFF) / 64];
		const float l0[3] = { nd.lo0x, nd.lo0y, nd.lo0z }, h0[3] = { nd.hi0x, nd.hi0y, nd.hi0z };
		const float l1[3] = { nd.lo1x, nd.lo1y, nd.lo1z }, h1[3] = { nd.hi1x, nd.hi1y, nd.hi1z };
		if (box_hit(l0, h0, o, inv, tbest))
			stk.push_back(nd.ref0);
		if (box_hit(l1, h1, o, inv, tbest))
			stk.push_back(nd.ref1);
	}
	return hit;
}

struct Stats {
	double rays = 0, visits = 0, boxes = 0, tris = 0, wave_steps = 0, leaf_rounds = 0, packets = 0, blocked = 0;
	double emit = 0;
	/* divergent wave steps (walking lanes at more than one node): distinct 64-B node entries and
	 * 128-B lines per step, and the line touches of the four per-lane loads vs a transposed fetch
	 * (load k = the 16-B quarters of lanes 16k..16k+15's nodes, four lanes per node) */
	double dsteps = 0, dnodes = 0, dlines = 0, touch_lane = 0, touch_tr = 0, walkers = 0, quad_lane = 0, quad_tr = 0;
	double post_nodes[8] = {}, post_leaves[8] = {}; /* postponed leaf tests, threshold T = 8 * k lanes */
	/* lane visits of divergent steps by the node's level (root 0), and of steps where every walking
	 * lane's node is at level <= L (a top-of-tree LDS copy of levels 0..L would serve them all) */
	double dlevel[16] = {}, dstep_top[16] = {};
	/* lane refill simulation (refill threshold RF_T[k]) */
	double rf_steps[6] = {}, rf_usteps[6] = {}, rf_refills[6] = {};
	/* occluder-first tests (opaque blockers): samples a cached occluder resolves, and the packets'
	 * wave steps / leaf rounds once those lanes skip their walk.  [0] probe ray to the light's
	 * centre, [1] the point's last blocker from an earlier packet, [2] the lane's blocker of the
	 * previous point (Morton neighbour), [3] probe + last blocker */
	double occ_hit[4] = {}, occ_steps[4] = {}, occ_rounds[4] = {}, probe_visits = 0, blocked_samples = 0;
	/* packet cull at uniform steps (every walking lane at one node): the node's children, those
	 * some walking lane hits, and those an interval test of the packet's shared origin and
	 * direction bounds keeps: [0] bounds over the packet's 64 rays, [1] over the walking lanes */
	double u_steps = 0, u_kids = 0, u_union = 0, u_cull[2] = {}, u_mixed = 0;
};
static const int RF_T[6] = { 64, 48, 32, 16, 8, 1 };

/* one point's light samples (their node-visit sequences) over one wave of 64 lanes that takes a
 * new sample into a finished lane whenever at least T lanes are idle (T = 64: packets, today) */
static void refill_sim(const std::vector<std::vector<uint32_t>> &seqs, int T, double &steps, double &usteps, double &refills)
{
	const size_t n = seqs.size();
	size_t q = 0;
	long cur[64];
	size_t pos[64];
	for (int l = 0; l < 64; l++)
		cur[l] = -1;
	for (;;) {
		int walking = 0;
		for (int l = 0; l < 64; l++)
			if (cur[l] >= 0 && pos[l] < seqs[cur[l]].size())
				walking++;
		if (!walking && q >= n)
			break;
		if (q < n && (64 - walking >= T || !walking)) {
			for (int l = 0; l < 64 && q < n; l++)
				if (cur[l] < 0 || pos[l] >= seqs[cur[l]].size()) {
					cur[l] = (long)q++;
					pos[l] = 0;
				}
			refills++;
			continue;
		}
		steps++;
		uint32_t first = ~0u;
		bool uni = true;
		for (int l = 0; l < 64; l++)
			if (cur[l] >= 0 && pos[l] < seqs[cur[l]].size()) {
				const uint32_t nd = seqs[cur[l]][pos[l]];
				if (first == ~0u)
					first = nd;
				uni &= nd == first;
				pos[l]++;
			}
		usteps += uni;
	}
}

/* the opaque triangle `obj` blocks the segment P + t d, eps < t < dist (Moller-Trumbore in double,
 * as the walk's leaf test) */
static bool occ_blocks(const rtx_scene_desc *sc, uint32_t obj, const float P[3], const double d[3], double dist)
{
	if (obj == RTX_NONE)
		return false;
	const rtx_object &o = sc->objects[obj];
	if (o.type != RTX_TRIANGLE || sc->materials[o.material].transparent)
		return false;
	const double e1[3] = { o.e1[0], o.e1[1], o.e1[2] }, e2[3] = { o.e2[0], o.e2[1], o.e2[2] };
	const double h[3] = { d[1] * e2[2] - d[2] * e2[1], d[2] * e2[0] - d[0] * e2[2], d[0] * e2[1] - d[1] * e2[0] };
	const double aa = e1[0] * h[0] + e1[1] * h[1] + e1[2] * h[2];
	if (fabs(aa) < o.epsilon)
		return false;
	const double f = 1 / aa, s[3] = { P[0] - o.p0[0], P[1] - o.p0[1], P[2] - o.p0[2] };
	const double uu = f * (s[0] * h[0] + s[1] * h[1] + s[2] * h[2]);
	const double q[3] = { s[1] * e1[2] - s[2] * e1[1], s[2] * e1[0] - s[0] * e1[2], s[0] * e1[1] - s[1] * e1[0] };
	const double vv = f * (d[0] * q[0] + d[1] * q[1] + d[2] * q[2]);
	const double tt = f * (e2[0] * q[0] + e2[1] * q[1] + e2[2] * q[2]);
	return uu >= 0 && vv >= 0 && uu + vv <= 1 && tt > o.epsilon && tt < dist;
}

int main(int argc, char **argv)
{
	if (argc < 2) {
		fprintf(stderr, "usage: %s scene.json [base_dir] [points]\n", argv[0]);
		return 2;
	}
	rtx_scene *scene = nullptr;
	if (rtx_scene_load(argv[1], nullptr, argc > 2 ? argv[2] : nullptr, &scene)) {
		fprintf(stderr, "load: %s\n", rtx_scene_last_error());
		return 1;
	}
	const int npts = argc > 3 ? atoi(argv[3]) : 4000;
	const bool near = getenv("W8SIM_NEAR") != nullptr; /* visit the nearest hit inner child first */
	const rtx_scene_desc *sc = rtx_scene_desc_of(scene);
	std::vector<uint32_t> bounded;
	for (uint32_t i = 0; i < sc->num_objects; i++)
		if (sc->objects[i].type != RTX_PLANE)
			bounded.push_back(i);
	uint32_t nb = (uint32_t)bounded.size();
	std::vector<float> lo(3 * (size_t)nb), hi(3 * (size_t)nb);
	float blo[3] = { FLT_MAX, FLT_MAX, FLT_MAX }, bhi[3] = { -FLT_MAX, -FLT_MAX, -FLT_MAX };
	for (uint32_t k = 0; k < nb; k++) {
		const rtx_object &o = sc->objects[bounded[k]];
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
		const float ext = std::max(h[0] - l[0], std::max(h[1] - l[1], h[2] - l[2]));
		for (int a = 0; a < 3; a++) {
			lo[3 * k + a] = l[a] - (std::fabs(l[a]) + ext) * 2e-6f - 1e-30f;
			hi[3 * k + a] = h[a] + (std::fabs(h[a]) + ext) * 2e-6f + 1e-30f;
			blo[a] = std::min(blo[a], lo[3 * k + a]);
			bhi[a] = std::max(bhi[a], hi[3 * k + a]);
		}
	}
	/* a BVH2 over boxes bl / bh with its primitive records in leaf order (rtx_build_scene's host path) */
	struct Tree2 {
		BvhOutput bvh;
		std::vector<DPrim> prims;
		std::vector<DNode> inner;
		uint32_t nnodes = 0, root = RTX_EMPTY_REF;
	};
	auto build2 = [&](const float *bl, const float *bh, Tree2 &T) {
		BvhConfig cfg;
		bvh_build(BvhInput{ nb, bl, bh }, cfg, T.bvh);
		T.nnodes = (uint32_t)T.bvh.nodes.size();
		T.prims.assign(nb, DPrim{});
		for (uint32_t k = 0; k < nb; k++) {
			const rtx_object &o = sc->objects[bounded[T.bvh.order[k]]];
			DPrim &p = T.prims[k];
			memset(&p, 0, sizeof(p));
			memcpy(p.a, o.p0, 12);
			p.a[3] = o.epsilon;
			if (o.type == RTX_SPHERE)
				p.b[0] = o.radius;
			else {
				memcpy(p.b, o.e1, 12);
				memcpy(p.c, o.e2, 12);
			}
			uint32_t meta = ((uint32_t)o.type << 24) | (uint32_t)o.material;
			if (sc->materials[o.material].transparent)
				meta |= RTX_META_TRANSPARENT;
			const uint32_t oi = bounded[T.bvh.order[k]];
			memcpy(&p.b[3], &oi, 4);
			memcpy(&p.c[3], &meta, 4);
		}
		const uint32_t nn = T.nnodes;
		auto dref = [nn](uint32_t r) -> uint32_t {
			if (r == RTX_EMPTY_REF)
				return r;
			if (r & RTX_LEAF_BIT) {
				const uint32_t first = (r >> 4) & 0x7FFFFFFu, cnt = (r & 15u) + 1;
				return (nn + first) * (uint32_t)sizeof(DNode) | RTX_REF_LEAF | (cnt - 1);
			}
			return r * (uint32_t)sizeof(DNode);
		};
		T.inner = T.bvh.nodes;
		for (DNode &d : T.inner) {
			d.ref0 = dref(d.ref0);
			d.ref1 = dref(d.ref1);
		}
		T.root = dref(T.bvh.root_ref);
	};
	const auto t0 = std::chrono::steady_clock::now();
	Tree2 W; /* world boxes: the shade points' closest hits */
	build2(lo.data(), hi.data(), W);
	const auto t1 = std::chrono::steady_clock::now();
	const BvhOutput &bvh = W.bvh;
	const uint32_t nnodes = W.nnodes;
	std::vector<DPrim> &prims = W.prims;
	std::vector<DNode> &inner = W.inner;
	/* the trees' frame as the uploader chooses it (rtx_frame.cpp; W8SIM_FRAME=0: the world axes),
	 * the 8-wide tree built over the leaf boxes in it */
	DTreeFrame tf;
	const double fratio = getenv("W8SIM_FRAME") && !atoi(getenv("W8SIM_FRAME")) ? (rtx_frame_choose(sc, {}, blo, bhi, tf), 1.0)
										 : rtx_frame_choose(sc, bounded, blo, bhi, tf);
	double fpad = 0.0;
	float tlo[3], thi[3];
	memcpy(tlo, blo, 12);
	memcpy(thi, bhi, 12);
	Tree2 Fr;
	const Tree2 *WT = &W;
	std::vector<float> flo(3 * (size_t)nb), fhi(3 * (size_t)nb);
	/* W8SIM_PAIRS=1: triangles whose frame boxes are identical (the two halves of an axis-aligned
	 * face), same material, same epsilon, share one leaf slot; partner[k] = the other one */
	std::vector<uint32_t> partner(sc->num_objects, RTX_NONE);
	const bool pairs = getenv("W8SIM_PAIRS") && atoi(getenv("W8SIM_PAIRS"));
	if (tf.rotated) {
		fpad = rtx_frame_pad(rtx_frame_radius(blo, bhi, tf));
		rtx_frame_boxes(sc, bounded, tf, fpad, flo.data(), fhi.data(), tlo, thi);
		if (pairs) {
			std::vector<uint32_t> idx(nb);
			for (uint32_t k = 0; k < nb; k++)
				idx[k] = k;
			const double g = 1e-4 * rtx_frame_radius(blo, bhi, tf); /* boxes equal to a 1e-4 radius grid */
			auto key = [&](uint32_t k) {
				const rtx_object &o = sc->objects[bounded[k]];
				auto r = [&](float v) { return (long long)llround(v / g); };
				return std::make_tuple(o.type, o.material, o.epsilon, r(flo[3 * k]), r(flo[3 * k + 1]), r(flo[3 * k + 2]),
						       r(fhi[3 * k]), r(fhi[3 * k + 1]), r(fhi[3 * k + 2]));
			};
			std::sort(idx.begin(), idx.end(), [&](uint32_t a, uint32_t b) { return key(a) < key(b); });
			std::vector<uint32_t> keep;
			std::vector<uint32_t> blist;
			for (size_t i = 0; i < nb;) {
				size_t j = i + 1;
				while (j < nb && key(idx[j]) == key(idx[i]))
					j++;
				if (j - i == 2 && sc->objects[bounded[idx[i]]].type == RTX_TRIANGLE) {
					partner[bounded[idx[i]]] = bounded[idx[i + 1]];
					keep.push_back(idx[i]);
					for (int a = 0; a < 3; a++) { /* the slot's box: the union */
						flo[3 * idx[i] + a] = std::min(flo[3 * idx[i] + a], flo[3 * idx[i + 1] + a]);
						fhi[3 * idx[i] + a] = std::max(fhi[3 * idx[i] + a], fhi[3 * idx[i + 1] + a]);
					}
				} else
					for (size_t q = i; q < j; q++)
						keep.push_back(idx[q]);
				i = j;
			}
			std::sort(keep.begin(), keep.end());
			std::vector<float> plo, phi;
			for (uint32_t k : keep) {
				blist.push_back(bounded[k]);
				plo.insert(plo.end(), &flo[3 * k], &flo[3 * k] + 3);
				phi.insert(phi.end(), &fhi[3 * k], &fhi[3 * k] + 3);
			}
			printf("pairs: %zu units for %u primitives\n", keep.size(), nb);
			bounded.swap(blist); /* build2 reads `bounded` and `nb` */
			nb = (uint32_t)bounded.size();
			build2(plo.data(), phi.data(), Fr);
		} else {
			build2(flo.data(), fhi.data(), Fr);
		}
		WT = &Fr;
	}
	printf("tree frame: %s (leaf-box cost x%.3f)\n", tf.rotated ? "rotated" : "world", fratio);
	QFrame F;
	float ext_max = 0.f;
	for (int a = 0; a < 3; a++)
		ext_max = std::max(ext_max, thi[a] - tlo[a]);
	for (int a = 0; a < 3; a++) {
		F.qo[a] = tlo[a];
		F.qs[a] = 65533.f / std::max(thi[a] - tlo[a], std::max(ext_max, 1.f) * 1e-6f);
	}
	std::vector<DW8> w8;
	std::vector<uint32_t> leafmap;
	std::vector<uint32_t> emit_objs(sc->emitters, sc->emitters + sc->num_emitters);
	bool skipped = false;
	const uint32_t depth = rtx_wide8_build(WT->inner, WT->nnodes, WT->prims.data(), WT->root, tlo, thi, emit_objs, tf, fpad, F,
					       skipped, w8, leafmap);
	const auto t2 = std::chrono::steady_clock::now();
	printf("host SAH build %.1f ms, 8-wide collapse %.1f ms\n", std::chrono::duration<double, std::milli>(t1 - t0).count(),
	       std::chrono::duration<double, std::milli>(t2 - t1).count());
	uint32_t nodes = 0, kids = 0, inner_kids = 0;
	std::vector<uint32_t> hist(9, 0);
	for (const DW8 &e : w8)
		if (e.w[3]) {
			nodes++;
			kids += __builtin_popcount(e.w[3] & 0xFFu);
			inner_kids += __builtin_popcount(e.w[2] & 0xFF);
			hist[__builtin_popcount(e.w[3] & 0xFFu)]++;
		}
	printf("prims %u  bvh2 nodes %u depth %u  w8 entries %zu nodes %u depth %u  children/node %.2f (inner %.2f)  hist",
	       nb, nnodes, bvh.depth, w8.size(), nodes, depth, (double)kids / nodes, (double)inner_kids / nodes);
	for (int i = 1; i <= 8; i++)
		printf(" %u", hist[i]);
	printf("\n");
	/* every node entry's level (root 0) and the node count per level */
	std::vector<uint32_t> level(w8.size(), ~0u), per_level(16, 0);
	{
		std::vector<uint32_t> q{ 0u };
		level[0] = 0;
		for (size_t h = 0; h < q.size(); h++) {
			const DW8 &e = w8[q[h]];
			per_level[std::min<uint32_t>(level[q[h]], 15)]++;
			for (int c = 0; c < 8; c++)
				if ((e.w[2] >> c) & 1) {
					const uint32_t ch = (e.w[2] >> 8) + c;
					level[ch] = level[q[h]] + 1;
					q.push_back(ch);
				}
		}
	}
	printf("nodes per level:");
	for (int i = 0; i < 16 && per_level[i]; i++)
		printf(" %u", per_level[i]);
	printf("\n");
	for (size_t i = 0; i < w8.size(); i++) /* leaf entries hold the primitive records */
		if (leafmap[i] != RTX_NONE)
			memcpy(&w8[i], &WT->prims[leafmap[i]], 64);

	/* shade points on bounded surfaces (area-weighted) and planes, light samples on emitter 0 */
	std::mt19937_64 rng(12345);
	std::uniform_real_distribution<float> U(0.f, 1.f);
	std::vector<double> cdf;
	double acc = 0;
	for (uint32_t k = 0; k < nb; k++) {
		const rtx_object &o = sc->objects[bounded[k]];
		acc += o.type == RTX_SPHERE ? 0.0 : area3(o.p0, o.p1, o.p2);
		cdf.push_back(acc);
	}
	if (!sc->num_emitters) {
		printf("no emitters\n");
		return 0;
	}
	const rtx_object &E = sc->objects[sc->emitters[0]];
	const uint32_t nl = E.num_lights ? E.num_lights : 1;
	Stats S;
	const float qsi[3] = { 1.f / F.qs[0], 1.f / F.qs[1], 1.f / F.qs[2] };
	/* shade points as the bench frame makes them: primary hits of sampled pixels, then -n GI
	 * hits from each (uniform hemisphere about the normal, render.c:231-289) */
	Scene2 S2{ sc, &inner, &prims, nnodes, W.root };
	rtx_frame fr;
	rtx_frame_setup(&sc->camera, 1920, 1080, &fr);
	std::vector<std::array<float, 3>> pts;
	const int gi = 64;
	while ((int)pts.size() < npts) {
		const uint32_t x = (uint32_t)(U(rng) * 1920) % 1920, y = (uint32_t)(U(rng) * 1080) % 1080;
		double o[3], d[3], dn = 0;
		for (int a = 0; a < 3; a++) {
			o[a] = fr.origin[a];
			d[a] = fr.corner[a] + (x + 1) * fr.step_x[a] + y * fr.step_y[a] - o[a];
			dn += d[a] * d[a];
		}
		for (int a = 0; a < 3; a++)
			d[a] /= sqrt(dn);
		double t, n[3];
		if (!closest(S2, o, d, t, n))
			continue;
		double P0[3], nn = sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
		for (int a = 0; a < 3; a++) {
			P0[a] = o[a] + t * d[a];
			n[a] /= nn;
		}
		if (n[0] * d[0] + n[1] * d[1] + n[2] * d[2] > 0)
			for (int a = 0; a < 3; a++)
				n[a] = -n[a];
		pts.push_back({ (float)P0[0], (float)P0[1], (float)P0[2] });
		for (int g = 0; g < gi && (int)pts.size() < npts; g++) {
			double r[3], rn;
			do {
				for (int a = 0; a < 3; a++)
					r[a] = 2 * U(rng) - 1;
				rn = r[0] * r[0] + r[1] * r[1] + r[2] * r[2];
			} while (rn > 1 || rn < 1e-6);
			double dd = 0;
			for (int a = 0; a < 3; a++) {
				r[a] /= sqrt(rn);
				dd += r[a] * n[a];
			}
			if (dd < 0)
				for (int a = 0; a < 3; a++)
					r[a] = -r[a];
			double t2, n2[3];
			if (closest(S2, P0, r, t2, n2))
				pts.push_back({ (float)(P0[0] + t2 * r[0]), (float)(P0[1] + t2 * r[1]), (float)(P0[2] + t2 * r[2]) });
		}
	}
	/* the first opaque blocker of the segment P + t d (t < dist) in the walk's slot order (the
	 * occluder-first probe), and the node visits it took */
	auto probe_blocker = [&](const float P[3], const double d[3], double dist, double &visits) -> uint32_t {
		double ob[3], db[3], invq[3], oi[3];
		for (int a = 0; a < 3; a++) {
			ob[a] = tf.rotated ? tf.r[a][0] * (P[0] - tf.c[0]) + tf.r[a][1] * (P[1] - tf.c[1]) + tf.r[a][2] * (P[2] - tf.c[2]) : P[a];
			db[a] = tf.rotated ? tf.r[a][0] * d[0] + tf.r[a][1] * d[1] + tf.r[a][2] * d[2] : d[a];
		}
		for (int a = 0; a < 3; a++) {
			const double inv = fabs(db[a]) > 1e-30 ? 1.0 / db[a] : copysign(1e30, db[a]);
			invq[a] = inv * qsi[a];
			oi[a] = (ob[a] - F.qo[a]) * F.qs[a] * invq[a];
		}
		std::vector<uint32_t> stk{ 0u };
		while (!stk.empty()) {
			const uint32_t node = stk.back();
			stk.pop_back();
			const DW8 &N = w8[node];
			visits++;
			const double org[3] = { (double)(N.w[0] & 0xFFFF), (double)(N.w[0] >> 16), (double)(N.w[1] & 0xFFFF) };
			const int ex[3] = { (int)((N.w[1] >> 16) & 15), (int)((N.w[1] >> 20) & 15), (int)((N.w[1] >> 24) & 15) };
			const uint32_t base = N.w[2] >> 8;
			for (int c = 7; c >= 0; c--) { /* pushed in reverse: popped in slot order */
				if (!((N.w[3] >> c) & 1))
					continue;
				double tn = 0, tfar = dist;
				for (int a = 0; a < 3; a++) {
					const uint8_t *l8 = (const uint8_t *)&N.w[4 + 4 * a], *h8 = (const uint8_t *)&N.w[6 + 4 * a];
					const double t0 = (org[a] + ldexp(l8[c], ex[a])) * invq[a] - oi[a];
					const double t1 = (org[a] + ldexp(h8[c], ex[a])) * invq[a] - oi[a];
					tn = std::max(tn, std::min(t0, t1));
					tfar = std::min(tfar, std::max(t0, t1));
				}
				if (tn > tfar)
					continue;
				if ((N.w[2] >> c) & 1) {
					stk.push_back(base + c);
					continue;
				}
				const DPrim &p = *(const DPrim *)&w8[base + c];
				uint32_t obj;
				memcpy(&obj, &p.b[3], 4);
				if (occ_blocks(sc, obj, P, d, dist))
					return obj;
			}
		}
		return RTX_NONE;
	};
	const bool occ_sim = getenv("W8SIM_OCC") && atoi(getenv("W8SIM_OCC"));
	/* W8SIM_CONE=1: a per-point cone walk before the packets: the tree's boxes (as bounding spheres)
	 * against the cone from the shade point around the light's bounding sphere; a point whose cone
	 * meets no leaf entry needs no walk for any of its samples */
	const bool cone_sim = getenv("W8SIM_CONE") && atoi(getenv("W8SIM_CONE"));
	double cone_pts_empty = 0, cone_visits = 0, cone_leaves = 0, ws_empty = 0, lr_empty = 0, pk_empty = 0;
	double nohit_pts = 0, ws_nohit = 0; /* points none of whose sample rays reached a leaf box (any cull's bound) */
	/* walking points: steps as packed (index order) against their lanes packed by walk length */
	double wk_steps = 0, wk_sorted = 0, wk_part = 0, wk_lanes = 0, wk_walkers = 0;
	std::vector<double> cone_leaf_hist(8, 0.0), cone_depth_hist(16, 0.0), ws_depth(16, 0.0);
	const int order = getenv("W8SIM_ORDER") ? atoi(getenv("W8SIM_ORDER")) : 0;
	const bool sort_samples = getenv("W8SIM_SORT") && atoi(getenv("W8SIM_SORT"));
	const bool strat = getenv("W8SIM_STRAT") && atoi(getenv("W8SIM_STRAT")); /* RTX_RNG_STRAT light samples */
	uint32_t prev_lane_blk[64];
	for (int l = 0; l < 64; l++)
		prev_lane_blk[l] = RTX_NONE;
	for (int pi = 0; pi < npts; pi++) {
		const float P[3] = { pts[pi][0], pts[pi][1], pts[pi][2] };
		uint32_t probe_occ = RTX_NONE, last_blk = RTX_NONE;
		bool cone_empty = false, point_leafhit = false;
		uint32_t cone_maxd = 0;
		const double ws0 = S.wave_steps, lr0 = S.leaf_rounds, pk0 = S.packets;
		if (cone_sim) {
			double Lc[3], lr;
			if (E.type == RTX_SPHERE) {
				for (int a = 0; a < 3; a++)
					Lc[a] = E.p0[a];
				lr = E.radius;
			} else {
				for (int a = 0; a < 3; a++)
					Lc[a] = E.p0[a] + (E.e1[a] + E.e2[a]) / 3.0;
				lr = 0;
				for (int k = 0; k < 3; k++) {
					double v[3], q = 0;
					for (int a = 0; a < 3; a++)
						v[a] = E.p0[a] + (k == 1 ? E.e1[a] : k == 2 ? E.e2[a] : 0.0) - Lc[a];
					for (int a = 0; a < 3; a++)
						q += v[a] * v[a];
					lr = std::max(lr, sqrt(q));
				}
			}
			lr = lr * (1 + 1e-5) + 1e-6;
			double Pf[3], Cf[3];
			for (int a = 0; a < 3; a++) {
				Pf[a] = tf.rotated ? tf.r[a][0] * (P[0] - tf.c[0]) + tf.r[a][1] * (P[1] - tf.c[1]) + tf.r[a][2] * (P[2] - tf.c[2]) : P[a];
				Cf[a] = tf.rotated ? tf.r[a][0] * (Lc[0] - tf.c[0]) + tf.r[a][1] * (Lc[1] - tf.c[1]) + tf.r[a][2] * (Lc[2] - tf.c[2]) : Lc[a];
			}
			double ax[3], L = 0;
			for (int a = 0; a < 3; a++) {
				ax[a] = Cf[a] - Pf[a];
				L += ax[a] * ax[a];
			}
			L = sqrt(L);
			for (int a = 0; a < 3; a++)
				ax[a] /= L;
			const double sn = std::min(1.0, lr / L), cs = sqrt(std::max(0.0, 1 - sn * sn));
			uint32_t nleaves = 0, maxd = 0;
			std::vector<std::pair<uint32_t, uint32_t>> cst{ { 0u, 1u } };
			while (!cst.empty()) {
				const uint32_t node = cst.back().first, dep = cst.back().second;
				cst.pop_back();
				maxd = std::max(maxd, dep);
				const DW8 &N = w8[node];
				cone_visits++;
				const double org[3] = { (double)(N.w[0] & 0xFFFF), (double)(N.w[0] >> 16), (double)(N.w[1] & 0xFFFF) };
				const int ex[3] = { (int)((N.w[1] >> 16) & 15), (int)((N.w[1] >> 20) & 15), (int)((N.w[1] >> 24) & 15) };
				const uint32_t base = N.w[2] >> 8;
				for (int c = 0; c < 8; c++) {
					if (!((N.w[3] >> c) & 1))
						continue;
					double bc[3], br = 0;
					for (int a = 0; a < 3; a++) {
						const uint8_t *l8 = (const uint8_t *)&N.w[4 + 4 * a], *h8 = (const uint8_t *)&N.w[6 + 4 * a];
						const double lo = (org[a] + ldexp(l8[c], ex[a])) / F.qs[a] + F.qo[a];
						const double hi = (org[a] + ldexp(h8[c], ex[a])) / F.qs[a] + F.qo[a];
						bc[a] = 0.5 * (lo + hi);
						br += 0.25 * (hi - lo) * (hi - lo);
					}
					br = sqrt(br) * (1 + 1e-6) + 1e-6;
					double v[3], t = 0, vv = 0;
					for (int a = 0; a < 3; a++) {
						v[a] = bc[a] - Pf[a];
						t += v[a] * ax[a];
						vv += v[a] * v[a];
					}
					const double e = sqrt(std::max(0.0, vv - t * t));
					const bool hit = vv <= br * br || (t >= -br && t <= L + lr + br && e * cs - t * sn <= br);
					if (!hit)
						continue;
					if ((N.w[2] >> c) & 1) {
						cst.push_back({ base + c, dep + 1 });
					} else {
						const DPrim &pp = *(const DPrim *)&w8[base + c];
						uint32_t obj;
						memcpy(&obj, &pp.b[3], 4);
						if (obj != sc->emitters[0])
							nleaves++;
					}
				}
			}
			cone_leaves += nleaves;
			cone_empty = nleaves == 0;
			cone_pts_empty += cone_empty;
			cone_maxd = maxd;
			if (cone_empty)
				cone_depth_hist[std::min<uint32_t>(maxd, 15)]++;
			int b = 0;
			for (uint32_t x = nleaves; x && b < 7; x >>= 3)
				b++;
			cone_leaf_hist[b]++;
		}
		if (occ_sim) {
			float Lc[3];
			for (int a = 0; a < 3; a++)
				Lc[a] = E.type == RTX_SPHERE ? E.p0[a] : E.p0[a] + (E.e1[a] + E.e2[a]) / 3.f;
			double d[3] = { Lc[0] - P[0], Lc[1] - P[1], Lc[2] - P[2] };
			const double dist = sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
			for (int a = 0; a < 3; a++)
				d[a] /= dist;
			probe_occ = probe_blocker(P, d, dist, S.probe_visits);
		}
		/* packets of 64 light samples */
		std::vector<std::vector<uint32_t>> allseq; /* every sample's node visits (immediate-test walk) */
		/* the point's light samples: i.i.d. (or stratified) draws, walked in index order or, with
		 * W8SIM_SORT=1, in the order of their first draw's bucket among ceil(nl / 64) (k_shadow's
		 * sample_order) */
		std::vector<float> su1(nl), su2(nl);
		for (uint32_t j = 0; j < nl; j++) {
			su1[j] = strat ? ((float)j + U(rng)) / (float)nl : U(rng);
			su2[j] = U(rng);
		}
		std::vector<uint32_t> sord(nl);
		for (uint32_t j = 0; j < nl; j++)
			sord[j] = j;
		if (sort_samples && nl > 64) {
			const uint32_t G = (nl + 63) / 64;
			std::stable_sort(sord.begin(), sord.end(), [&](uint32_t a, uint32_t b) {
				return (uint32_t)(su1[a] * G) < (uint32_t)(su1[b] * G);
			});
		}
		std::vector<uint32_t> pt_len; /* every sample's walk length (visits) of this point */
		for (uint32_t b0 = 0; b0 < nl; b0 += 64) {
			std::vector<uint32_t> visits_lane, leaf_at; /* per-lane per-visit leaf hits */
			std::vector<std::vector<uint32_t>> leaves(64), seq(64);
			uint32_t block_at[64]; /* ordinal (in discovery order) of the lane's blocking leaf test, or ~0 */
			uint32_t blk_obj[64]; /* the lane's blocking primitive (object index), or RTX_NONE */
			double lane_invq[64][3], lane_oq[64][3], lane_tl[64];
			float lane_d[64][3], lane_dist[64];
			uint32_t maxv = 0, imm_len[64] = {};
			for (uint32_t l = 0; l < 64 && b0 + l < nl; l++) {
				const uint32_t j = b0 + l;
				float u1 = su1[sord[j]], u2 = su2[sord[j]];
				float Lp[3];
				if (E.type == RTX_SPHERE) {
					const float inc = u1 * 2.f * 3.1415927f, az = u2 * 2.f * 3.1415927f;
					float ld[3] = { E.radius * cosf(az) * sinf(inc), E.radius * sinf(az) * sinf(inc), E.radius * cosf(inc) };
					const float nr[3] = { E.p0[0] - P[0], E.p0[1] - P[1], E.p0[2] - P[2] };
					if (nr[0] * ld[0] + nr[1] * ld[1] + nr[2] * ld[2] != 0.f)
						for (int a = 0; a < 3; a++)
							ld[a] = -ld[a];
					for (int a = 0; a < 3; a++)
						Lp[a] = E.p0[a] + ld[a];
				} else {
					if (u1 + u2 > 1) {
						u1 = 1 - u1;
						u2 = 1 - u2;
					}
					for (int a = 0; a < 3; a++)
						Lp[a] = E.p0[a] + u1 * E.e1[a] + u2 * E.e2[a];
				}
				double d[3] = { Lp[0] - P[0], Lp[1] - P[1], Lp[2] - P[2] };
				const double dist = sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
				for (int a = 0; a < 3; a++)
					d[a] /= dist;
				for (int a = 0; a < 3; a++)
					lane_d[l][a] = (float)d[a];
				lane_dist[l] = (float)dist;
				blk_obj[l] = RTX_NONE;
				double invq[3], oi[3], ob[3], db[3];
				for (int a = 0; a < 3; a++) { /* the ray in the trees' frame (boxes); primitives in world space */
					ob[a] = tf.rotated ? tf.r[a][0] * (P[0] - tf.c[0]) + tf.r[a][1] * (P[1] - tf.c[1]) + tf.r[a][2] * (P[2] - tf.c[2]) : P[a];
					db[a] = tf.rotated ? tf.r[a][0] * d[0] + tf.r[a][1] * d[1] + tf.r[a][2] * d[2] : d[a];
				}
				int oct = 0;
				for (int a = 0; a < 3; a++) {
					const double inv = fabs(db[a]) > 1e-30 ? 1.0 / db[a] : copysign(1e30, db[a]);
					if (inv >= 0)
						oct |= 1 << a;
					invq[a] = inv * qsi[a];
					oi[a] = (ob[a] - F.qo[a]) * F.qs[a] * invq[a];
					lane_invq[l][a] = invq[a];
					lane_oq[l][a] = (ob[a] - F.qo[a]) * F.qs[a];
				}
				lane_tl[l] = dist;
				/* W8SIM_ORDER: 0 front to back from the shade point (octant order), 1 plain slot order
				 * (k_shadow's RTX_W8_SORDER 0), 2 back to front (front to back from the light) */
				const uint32_t K = order == 1 ? 0u : order == 2 ? (uint32_t)oct & 7u : ~(uint32_t)oct & 7u;
				/* the walk: node, group register, stack; leaf hits counted per visit */
				std::vector<uint32_t> stk;
				uint32_t node = 0, grp = 0, nv = 0, nleaf_total = 0;
				block_at[l] = ~0u;
				bool blocked = false;
				uint32_t nv_imm = 0; /* visits of the immediate-test walk (ends at the blocker's visit) */
				while (node != RTX_NONE) {
					if (!blocked) {
						nv_imm++;
						seq[l].push_back(node);
					}
					const DW8 &N = w8[node];
					nv++;
					S.boxes += __builtin_popcount(N.w[3] & 0xFFu);
					const double org[3] = { (double)(N.w[0] & 0xFFFF), (double)(N.w[0] >> 16), (double)(N.w[1] & 0xFFFF) };
					const int ex[3] = { (int)((N.w[1] >> 16) & 15), (int)((N.w[1] >> 20) & 15), (int)((N.w[1] >> 24) & 15) };
					uint32_t hm = 0, near_p = 8;
					double near_t = 1e300;
					for (int c = 0; c < 8; c++) {
						if (!((N.w[3] >> c) & 1))
							continue;
						double tn = 0, tf = dist;
						for (int a = 0; a < 3; a++) {
							const uint8_t *l8 = (const uint8_t *)&N.w[4 + 4 * a], *h8 = (const uint8_t *)&N.w[6 + 4 * a];
							const double t0 = (org[a] + ldexp(l8[c], ex[a])) * invq[a] - oi[a];
							const double t1 = (org[a] + ldexp(h8[c], ex[a])) * invq[a] - oi[a];
							tn = std::max(tn, std::min(t0, t1));
							tf = std::min(tf, std::max(t0, t1));
						}
						if (tn <= tf) {
							hm |= 1u << (c ^ K);
							if (((N.w[2] >> c) & 1) && tn < near_t) {
								near_t = tn;
								near_p = c ^ K;
							}
						}
					}
					uint32_t io = 0;
					for (int c = 0; c < 8; c++)
						if ((N.w[2] >> c) & 1)
							io |= 1u << (c ^ K);
					const uint32_t base = N.w[2] >> 8;
					uint32_t lm = hm & ~io, im = hm & io;
					uint32_t nleaf = 0;
					for (; lm; lm &= lm - 1) {
						S.tris++;
						const DPrim &p = *(const DPrim *)&w8[base + (__builtin_ctz(lm) ^ K)];
						uint32_t meta;
						memcpy(&meta, &p.c[3], 4);
						uint32_t obj;
						memcpy(&obj, &p.b[3], 4);
						if (obj == sc->emitters[0]) {
							S.emit++;
							continue;
						}
						nleaf++;
						nleaf_total++;
						if ((meta & RTX_META_TRANSPARENT) || (meta >> 24) == RTX_SPHERE)
							continue;
						for (int half = 0; half < (partner[obj] != RTX_NONE ? 2 : 1); half++) {
						DPrim pp = p;
						if (half) { /* the pair's other triangle, in the same leaf round */
							S.tris++;
							const rtx_object &o2 = sc->objects[partner[obj]];
							memcpy(pp.a, o2.p0, 12);
							pp.a[3] = o2.epsilon;
							memcpy(pp.b, o2.e1, 12);
							memcpy(pp.c, o2.e2, 12);
						}
						const DPrim &p = pp;
						/* opaque triangle: Moller-Trumbore in double */
						const double e1[3] = { p.b[0], p.b[1], p.b[2] }, e2[3] = { p.c[0], p.c[1], p.c[2] };
						const double h[3] = { d[1] * e2[2] - d[2] * e2[1], d[2] * e2[0] - d[0] * e2[2], d[0] * e2[1] - d[1] * e2[0] };
						const double aa = e1[0] * h[0] + e1[1] * h[1] + e1[2] * h[2];
						if (fabs(aa) < p.a[3])
							continue;
						const double f = 1 / aa, s[3] = { P[0] - p.a[0], P[1] - p.a[1], P[2] - p.a[2] };
						const double uu = f * (s[0] * h[0] + s[1] * h[1] + s[2] * h[2]);
						const double q[3] = { s[1] * e1[2] - s[2] * e1[1], s[2] * e1[0] - s[0] * e1[2], s[0] * e1[1] - s[1] * e1[0] };
						const double vv = f * (d[0] * q[0] + d[1] * q[1] + d[2] * q[2]);
						const double tt = f * (e2[0] * q[0] + e2[1] * q[1] + e2[2] * q[2]);
						if (!blocked && uu >= 0 && vv >= 0 && uu + vv <= 1 && tt > p.a[3] && tt < dist) {
							blocked = true;
							block_at[l] = nleaf_total - 1;
							blk_obj[l] = half ? partner[obj] : obj;
							/* postponed tests would have kept walking: record the rest of the walk
							 * (the leaf hits of later visits) without stopping at the blocker */
						}
						}
					}
					leaves[l].push_back(nleaf);
				point_leafhit |= nleaf > 0;
					if (im) {
						const uint32_t p0 = near ? near_p : (uint32_t)__builtin_ctz(im);
						node = base + (p0 ^ K);
						im &= ~(1u << p0);
						if (im) {
							if (grp)
								stk.push_back(grp);
							grp = (base << 8) | im;
						}
					} else if (grp) {
						node = (grp >> 8) + (__builtin_ctz(grp) ^ K);
						grp &= grp - 1;
						if (!(grp & 0xFF)) {
							grp = 0;
							if (!stk.empty()) {
								grp = stk.back();
								stk.pop_back();
							}
						}
					} else {
						node = RTX_NONE;
					}
				}
				S.rays++;
				S.visits += nv_imm;
				S.blocked += blocked;
				maxv = std::max(maxv, nv_imm);
				imm_len[l] = nv_imm;
			}
			for (uint32_t l = 0; l < 64 && b0 + l < nl; l++)
				allseq.emplace_back(seq[l].begin(), seq[l].begin() + std::min<size_t>(seq[l].size(), imm_len[l]));
			S.packets++;
			if (occ_sim) {
				const uint32_t nlanes = std::min<uint32_t>(64, nl - b0);
				for (uint32_t l = 0; l < nlanes; l++)
					S.blocked_samples += blk_obj[l] != RTX_NONE;
				for (int v = 0; v < 4; v++) {
					bool res[64] = {};
					for (uint32_t l = 0; l < nlanes; l++) {
						const double dd[3] = { lane_d[l][0], lane_d[l][1], lane_d[l][2] };
						const uint32_t o1 = v == 0 || v == 3 ? probe_occ : v == 1 ? last_blk : prev_lane_blk[l];
						res[l] = occ_blocks(sc, o1, P, dd, lane_dist[l]) ||
							 (v == 3 && occ_blocks(sc, last_blk, P, dd, lane_dist[l]));
						S.occ_hit[v] += res[l];
					}
					uint32_t mv = 0;
					for (uint32_t l = 0; l < nlanes; l++)
						if (!res[l])
							mv = std::max(mv, imm_len[l]);
					S.occ_steps[v] += mv;
					for (uint32_t i = 0; i < mv; i++) {
						uint32_t m = 0;
						for (uint32_t l = 0; l < nlanes; l++)
							if (!res[l] && i < imm_len[l])
								m = std::max(m, leaves[l][i]);
						S.occ_rounds[v] += m;
					}
				}
				for (uint32_t l = 0; l < nlanes; l++)
					if (blk_obj[l] != RTX_NONE) {
						if (last_blk == RTX_NONE || true)
							last_blk = blk_obj[l]; /* the packet's last blocked lane: the cache of the next packet */
						prev_lane_blk[l] = blk_obj[l];
					}
			}
			/* postponed leaf tests: a leaf round only when >= T lanes hold pending leaves or no lane
			 * has node work left (emitter leaves excluded, as a tree without emitters) */
			for (int k = 0; k < 8; k++) {
				const uint32_t T = k ? 8 * k : 1;
				uint32_t v[64] = {}, pend[64] = {}, tested[64] = {};
				bool done[64] = {};
				for (;;) {
					uint32_t L = 0, W = 0;
					for (int l = 0; l < 64; l++) {
						if (done[l])
							continue;
						L += pend[l] > 0;
						W += v[l] < leaves[l].size();
					}
					if (!L && !W)
						break;
					if (!W || L >= T) {
						S.post_leaves[k]++;
						for (int l = 0; l < 64; l++)
							if (!done[l] && pend[l]) {
								pend[l]--;
								if (tested[l]++ == block_at[l])
									done[l] = true;
							}
					} else {
						S.post_nodes[k]++;
						for (int l = 0; l < 64; l++)
							if (!done[l] && v[l] < leaves[l].size())
								pend[l] += leaves[l][v[l]++];
					}
				}
			}
			S.wave_steps += maxv;
			for (uint32_t l = 0; l < 64 && b0 + l < nl; l++)
				pt_len.push_back(imm_len[l]);
			for (uint32_t i = 0; i < maxv; i++) {
				std::vector<uint32_t> at(64, ~0u);
				uint32_t first = ~0u;
				bool div = false;
				for (int l = 0; l < 64; l++)
					if (i < seq[l].size()) {
						at[l] = seq[l][i];
						if (first == ~0u)
							first = at[l];
						div |= at[l] != first;
					}
				if (!div) {
					if (first == ~0u)
						continue;
					/* a uniform step at node `first` */
					const DW8 &N = w8[first];
					const double org[3] = { (double)(N.w[0] & 0xFFFF), (double)(N.w[0] >> 16), (double)(N.w[1] & 0xFFFF) };
					const int ex[3] = { (int)((N.w[1] >> 16) & 15), (int)((N.w[1] >> 20) & 15), (int)((N.w[1] >> 24) & 15) };
					const uint32_t nl2 = std::min<uint32_t>(64, nl - b0);
					S.u_steps++;
					S.u_kids += __builtin_popcount(N.w[3] & 0xFFu);
					double imn[2][3], imx[2][3], tlx[2] = { 0, 0 };
					for (int v = 0; v < 2; v++)
						for (int a = 0; a < 3; a++) {
							imn[v][a] = 1e300;
							imx[v][a] = -1e300;
						}
					for (uint32_t l = 0; l < nl2; l++)
						for (int v = 0; v < 2; v++) {
							if (v == 1 && at[l] == ~0u)
								continue;
							for (int a = 0; a < 3; a++) {
								imn[v][a] = std::min(imn[v][a], lane_invq[l][a]);
								imx[v][a] = std::max(imx[v][a], lane_invq[l][a]);
							}
							tlx[v] = std::max(tlx[v], lane_tl[l]);
						}
					bool mixed = false;
					for (int a = 0; a < 3; a++)
						mixed |= imn[0][a] < 0 && imx[0][a] > 0;
					S.u_mixed += mixed;
					const double *oq = lane_oq[0]; /* one origin per packet (one shade point) */
					for (int c = 0; c < 8; c++) {
						if (!((N.w[3] >> c) & 1))
							continue;
						double lo[3], hi[3];
						for (int a = 0; a < 3; a++) {
							const uint8_t *l8 = (const uint8_t *)&N.w[4 + 4 * a], *h8 = (const uint8_t *)&N.w[6 + 4 * a];
							lo[a] = org[a] + ldexp(l8[c], ex[a]);
							hi[a] = org[a] + ldexp(h8[c], ex[a]);
						}
						bool any = false; /* some walking lane hits the child */
						for (uint32_t l = 0; l < nl2 && !any; l++) {
							if (at[l] == ~0u)
								continue;
							double tn = 0, tf = lane_tl[l];
							for (int a = 0; a < 3; a++) {
								const double t0 = (lo[a] - oq[a]) * lane_invq[l][a], t1 = (hi[a] - oq[a]) * lane_invq[l][a];
								tn = std::max(tn, std::min(t0, t1));
								tf = std::min(tf, std::max(t0, t1));
							}
							any = tn <= tf;
						}
						S.u_union += any;
						for (int v = 0; v < 2; v++) {
							double tn = 0, tf = tlx[v];
							for (int a = 0; a < 3; a++) {
								if (imn[v][a] < 0 && imx[v][a] > 0)
									continue; /* the packet's directions straddle the axis: no bound */
								const double e[4] = { (lo[a] - oq[a]) * imn[v][a], (lo[a] - oq[a]) * imx[v][a],
										      (hi[a] - oq[a]) * imn[v][a], (hi[a] - oq[a]) * imx[v][a] };
								/* near: the lesser plane's least t; far: the greater plane's largest t */
								const double nlo = std::min(std::min(e[0], e[1]), std::min(e[2], e[3]));
								const double fhi = std::max(std::max(e[0], e[1]), std::max(e[2], e[3]));
								/* per ray the near plane is min(t_lo, t_hi) and the far max: bound each
								 * over the interval by the planes' own ranges */
								const double near_max_lo = std::min(std::max(e[0], e[1]) , std::max(e[2], e[3]));
								(void)near_max_lo;
								tn = std::max(tn, nlo);
								tf = std::min(tf, fhi);
							}
							if (tn <= tf)
								S.u_cull[v]++;
						}
					}
					continue;
				}
				S.dsteps++;
				uint32_t maxlev = 0;
				for (int l = 0; l < 64; l++)
					if (at[l] != ~0u) {
						S.dlevel[std::min<uint32_t>(level[at[l]], 15)]++;
						maxlev = std::max(maxlev, level[at[l]]);
					}
				for (uint32_t L = maxlev; L < 16; L++)
					S.dstep_top[L]++;
				std::vector<uint32_t> nodes, lines;
				for (int l = 0; l < 64; l++)
					if (at[l] != ~0u) {
						S.walkers++;
						nodes.push_back(at[l]);
						lines.push_back(at[l] >> 1);
					}
				auto uniq = [](std::vector<uint32_t> v) {
					std::sort(v.begin(), v.end());
					return (double)(std::unique(v.begin(), v.end()) - v.begin());
				};
				S.dnodes += uniq(nodes);
				const double dl = uniq(lines);
				S.dlines += dl;
				S.touch_lane += 4 * dl;
				/* address-path cycles if the texture unit takes 4 lanes (64 B) per cycle and one more
				 * cycle per further distinct line in a quad: per-lane loads (x4 instructions) vs
				 * transposed (each quad = one ray's node) */
				for (int q = 0; q < 16; q++) {
					std::vector<uint32_t> g;
					for (int l = 4 * q; l < 4 * q + 4; l++)
						if (at[l] != ~0u)
							g.push_back(at[l] >> 1);
					if (!g.empty())
						S.quad_lane += 4 * uniq(g);
				}
				S.quad_tr += nodes.size();
				for (int k = 0; k < 4; k++) {
					std::vector<uint32_t> g;
					for (int l = 16 * k; l < 16 * k + 16; l++)
						if (at[l] != ~0u)
							g.push_back(at[l] >> 1);
					S.touch_tr += uniq(g);
				}
			}
			for (uint32_t i = 0; i < maxv; i++) {
				uint32_t m = 0;
				for (int l = 0; l < 64; l++)
					if (i < imm_len[l])
						m = std::max(m, leaves[l][i]);
				S.leaf_rounds += m;
			}
		}
		for (int r = 0; r < 6; r++)
			refill_sim(allseq, RF_T[r], S.rf_steps[r], S.rf_usteps[r], S.rf_refills[r]);
		if (cone_sim && !cone_empty && !pt_len.empty()) {
			double st = 0;
			for (size_t b = 0; b < pt_len.size(); b += 64)
				st += *std::max_element(pt_len.begin() + b, pt_len.begin() + std::min(pt_len.size(), b + 64));
			std::vector<uint32_t> srt = pt_len, prt;
			std::sort(srt.begin(), srt.end(), std::greater<uint32_t>());
			for (uint32_t v : pt_len)
				if (v > 1)
					prt.push_back(v);
			const size_t nwalk = prt.size();
			for (uint32_t v : pt_len)
				if (v <= 1)
					prt.push_back(v);
			double ss = 0, sp = 0;
			for (size_t b = 0; b < srt.size(); b += 64) {
				ss += *std::max_element(srt.begin() + b, srt.begin() + std::min(srt.size(), b + 64));
				sp += *std::max_element(prt.begin() + b, prt.begin() + std::min(prt.size(), b + 64));
			}
			wk_steps += st;
			wk_sorted += ss;
			wk_part += sp;
			wk_lanes += pt_len.size();
			wk_walkers += nwalk;
		}
		if (cone_sim && !point_leafhit) {
			nohit_pts++;
			ws_nohit += S.wave_steps - ws0;
		}
		if (cone_sim && cone_empty) {
			ws_depth[std::min<uint32_t>(cone_maxd, 15)] += S.wave_steps - ws0;
			ws_empty += S.wave_steps - ws0;
			lr_empty += S.leaf_rounds - lr0;
			pk_empty += S.packets - pk0;
		}
	}
	if (cone_sim) {
		printf("cone walk: %.3f of points meet no leaf entry; %.2f node visits and %.1f leaf entries per point; those points "
		       "hold %.3f of the packets, %.3f of the wave steps, %.3f of the leaf rounds\n", cone_pts_empty / npts,
		       cone_visits / npts, cone_leaves / npts, pk_empty / S.packets, ws_empty / S.wave_steps, lr_empty / S.leaf_rounds);
		printf("  leaf entries per point: 0 %.3f, 1-7 %.3f, 8-63 %.3f, 64-511 %.3f, 512-4095 %.3f, >=4096 %.3f\n",
		       cone_leaf_hist[0] / npts, cone_leaf_hist[1] / npts, cone_leaf_hist[2] / npts, cone_leaf_hist[3] / npts,
		       cone_leaf_hist[4] / npts, (cone_leaf_hist[5] + cone_leaf_hist[6] + cone_leaf_hist[7]) / npts);
		printf("  bound: %.3f of points had no sample ray reach a leaf box, holding %.3f of the wave steps\n", nohit_pts / npts,
		       ws_nohit / S.wave_steps);
		printf("  points the cone does not clear: %.3f of their samples walk past the root; node steps as packed %.0f, "
		       "packed by walk length %.0f (%.3f), walkers first %.0f (%.3f)\n", wk_walkers / std::max(1.0, wk_lanes),
		       wk_steps, wk_sorted, wk_sorted / std::max(1.0, wk_steps), wk_part, wk_part / std::max(1.0, wk_steps));
		double cp = 0, cw = 0;
		for (int d = 1; d < 8; d++) {
			cp += cone_depth_hist[d];
			cw += ws_depth[d];
			printf("  proved empty within %d levels: %.3f of points, %.3f of the wave steps\n", d, cp / npts, cw / S.wave_steps);
		}
	}
	printf("lane refill (a finished lane takes the point's next light sample when >= T lanes are idle), per point:\n"
	       "   T   wave steps (uniform)   refill rounds   cost (178/divergent + 95/uniform step + 220/refill)\n");
	for (int k = 0; k < 6; k++)
		printf("  %2d   %8.2f (%6.2f)   %8.2f   %9.0f\n", RF_T[k], S.rf_steps[k] / npts, S.rf_usteps[k] / npts,
		       S.rf_refills[k] / npts,
		       (178.0 * (S.rf_steps[k] - S.rf_usteps[k]) + 95.0 * S.rf_usteps[k] + 220.0 * S.rf_refills[k]) / npts);
	printf("uniform steps %.2f per packet: children %.2f, hit by some walking lane %.2f, kept by the packet interval "
	       "test %.2f (bounds over the packet) / %.2f (over the walking lanes); steps with mixed-sign directions %.1f%%\n",
	       S.u_steps / S.packets, S.u_kids / S.u_steps, S.u_union / S.u_steps, S.u_cull[0] / S.u_steps, S.u_cull[1] / S.u_steps,
	       100 * S.u_mixed / std::max(1.0, S.u_steps));
	if (occ_sim) {
		static const char *nm[4] = { "probe to the light centre", "the point's last blocker (earlier packet)",
					     "the lane's blocker of the previous point", "probe + last blocker" };
		printf("occluder-first (opaque blockers; %.3f of samples blocked; probe %.2f node visits per point):\n"
		       "  occluder                                       resolves (of samples / of blocked)  wave steps/packet  leaf rounds/packet\n",
		       S.blocked_samples / S.rays, S.probe_visits / npts);
		printf("  %-46s %8s %8s          %8.2f          %8.2f\n", "none", "-", "-", S.wave_steps / S.packets, S.leaf_rounds / S.packets);
		for (int v = 0; v < 4; v++)
			printf("  %-46s %8.3f %8.3f          %8.2f          %8.2f\n", nm[v], S.occ_hit[v] / S.rays,
			       S.occ_hit[v] / std::max(1.0, S.blocked_samples), S.occ_steps[v] / S.packets, S.occ_rounds[v] / S.packets);
	}
	printf("rays %.0f  visits/ray %.2f  boxes/ray %.2f  tris/ray %.3f  blocked %.3f  wave steps/packet %.2f  leaf "
	       "rounds/packet %.2f  lanes/leaf round %.1f\n",
	       S.rays, S.visits / S.rays, S.boxes / S.rays, S.tris / S.rays, S.blocked / S.rays, S.wave_steps / S.packets,
	       S.leaf_rounds / S.packets, S.tris / S.leaf_rounds);
	printf("emitter leaf hits/ray %.3f\npostponed leaf tests (no emitter leaves), per packet: T  node steps  leaf rounds  "
	       "cost(290/step + 99/round)\n",
	       S.emit / S.rays);
	printf("divergent steps/packet %.2f  walking lanes %.1f  distinct nodes %.2f  lines %.2f  line touches per step: "
	       "per-lane loads %.1f  transposed %.1f  quad cycles: per-lane %.1f  transposed %.1f\n",
	       S.dsteps / S.packets, S.walkers / S.dsteps, S.dnodes / S.dsteps, S.dlines / S.dsteps, S.touch_lane / S.dsteps,
	       S.touch_tr / S.dsteps, S.quad_lane / S.dsteps, S.quad_tr / S.dsteps);
	printf("divergent-step lane visits by level:");
	for (int i = 0; i < 16; i++)
		if (S.dlevel[i])
			printf(" L%d %.1f%%", i, 100 * S.dlevel[i] / S.walkers);
	printf("\ndivergent steps with every walking lane at level <= L:");
	for (int i = 0; i < 8; i++)
		printf(" L%d %.1f%%", i, 100 * S.dstep_top[i] / S.dsteps);
	printf("\n");
	for (int k = 0; k < 8; k++)
		printf("  %2d  %6.2f  %6.2f  %7.0f\n", k ? 8 * k : 1, S.post_nodes[k] / S.packets, S.post_leaves[k] / S.packets,
		       (290 * S.post_nodes[k] + 99 * S.post_leaves[k]) / S.packets);
	rtx_scene_free(scene);
	return 0;
}
