/*
 * Binned-SAH BVH2 build on the host (OpenMP tasks over subtrees), flattened to
 * the 64-byte DNode layout in depth-first order.  See bvh_build.h.
 */
#include "bvh_build.h"

#include <algorithm>
#include <atomic>
#include <cfloat>
#include <cmath>
#include <cstring>

namespace {

struct Box {
	float lo[3], hi[3];
	void reset()
	{
		for (int i = 0; i < 3; i++) {
			lo[i] = FLT_MAX;
			hi[i] = -FLT_MAX;
		}
	}
	void grow(const Box &b)
	{
		for (int i = 0; i < 3; i++) {
			lo[i] = std::min(lo[i], b.lo[i]);
			hi[i] = std::max(hi[i], b.hi[i]);
		}
	}
	void grow_pt(const float *p)
	{
		for (int i = 0; i < 3; i++) {
			lo[i] = std::min(lo[i], p[i]);
			hi[i] = std::max(hi[i], p[i]);
		}
	}
	float area() const
	{
		float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
		if (dx < 0 || dy < 0 || dz < 0)
			return 0.f;
		return 2.f * (dx * dy + dy * dz + dz * dx);
	}
};

struct TNode {
	Box box;
	int32_t child[2]; /* temp node ids */
	uint32_t first, count;
	bool leaf;
};

struct Builder {
	const BvhInput &in;
	const BvhConfig &cfg;
	std::vector<Box> pbox;
	std::vector<float> cent; /* n*3 */
	std::vector<uint32_t> idx;
	std::vector<TNode> tn;
	std::atomic<uint32_t> ntn{ 0 };
	std::atomic<uint32_t> max_depth{ 0 };

	Builder(const BvhInput &i, const BvhConfig &c) : in(i), cfg(c) {}

	uint32_t alloc()
	{
		return ntn.fetch_add(1);
	}

	void make_leaf(uint32_t id, uint32_t b, uint32_t e, const Box &box)
	{
		TNode &t = tn[id];
		t.box = box;
		t.leaf = true;
		t.first = b;
		t.count = e - b;
		t.child[0] = t.child[1] = -1;
	}

	static int ceil_log2(uint32_t x)
	{
		int l = 0;
		while ((1u << l) < x)
			l++;
		return l;
	}

	void build(uint32_t id, uint32_t b, uint32_t e, uint32_t depth)
	{
		const uint32_t n = e - b;
		Box box, cb;
		box.reset();
		cb.reset();
		for (uint32_t i = b; i < e; i++) {
			box.grow(pbox[idx[i]]);
			cb.grow_pt(&cent[3 * (size_t)idx[i]]);
		}
		uint32_t md = max_depth.load();
		while (depth > md && !max_depth.compare_exchange_weak(md, depth)) {
		}
		if (n <= 1) {
			make_leaf(id, b, e, box);
			return;
		}
		/* depth budget: median splits need ceil(log2(n/max_leaf)) more levels */
		const int need = ceil_log2((n + cfg.max_leaf - 1) / cfg.max_leaf);
		const bool force_median = (int)depth + need + 1 >= (int)cfg.max_depth;

		int best_axis = -1;
		uint32_t best_split = 0;
		float best_cost = FLT_MAX;
		const uint32_t NB = cfg.bins;
		if (!force_median) {
			for (int ax = 0; ax < 3; ax++) {
				float ext = cb.hi[ax] - cb.lo[ax];
				if (!(ext > 0.f))
					continue;
				float k = NB * (1.f - 1e-6f) / ext;
				Box bb[64];
				uint32_t bc[64];
				for (uint32_t i = 0; i < NB; i++) {
					bb[i].reset();
					bc[i] = 0;
				}
				for (uint32_t i = b; i < e; i++) {
					uint32_t p = idx[i];
					int bi = (int)((cent[3 * (size_t)p + ax] - cb.lo[ax]) * k);
					bi = std::min(std::max(bi, 0), (int)NB - 1);
					bc[bi]++;
					bb[bi].grow(pbox[p]);
				}
				float ra[64];
				uint32_t rc[64];
				Box acc;
				acc.reset();
				uint32_t cnt = 0;
				for (int i = (int)NB - 1; i > 0; i--) {
					acc.grow(bb[i]);
					cnt += bc[i];
					ra[i] = acc.area();
					rc[i] = cnt;
				}
				acc.reset();
				cnt = 0;
				for (uint32_t i = 0; i + 1 < NB; i++) {
					acc.grow(bb[i]);
					cnt += bc[i];
					if (!cnt || !rc[i + 1])
						continue;
					float cost = acc.area() * cnt + ra[i + 1] * rc[i + 1];
					if (cost < best_cost) {
						best_cost = cost;
						best_axis = ax;
						best_split = i;
					}
				}
			}
		}
		const float parea = box.area();
		float split_cost = best_axis >= 0 && parea > 0 ? cfg.c_trav + cfg.c_isect * best_cost / parea : FLT_MAX;
		float leaf_cost = cfg.c_isect * n;
		if (n <= cfg.max_leaf && (force_median || leaf_cost <= split_cost)) {
			make_leaf(id, b, e, box);
			return;
		}
		uint32_t mid;
		if (best_axis >= 0 && !force_median) {
			float ext = cb.hi[best_axis] - cb.lo[best_axis];
			float k = NB * (1.f - 1e-6f) / ext;
			const int ax = best_axis;
			/* stable, like the device builder's prefix-scan partition (rtx_build.hip): primitives
			 * with equal centroids (a rotated mesh face's two triangles) keep their order, so both
			 * builders put the same primitive in the same leaf */
			uint32_t *pm = std::stable_partition(idx.data() + b, idx.data() + e, [&](uint32_t p) {
				int bi = (int)((cent[3 * (size_t)p + ax] - cb.lo[ax]) * k);
				bi = std::min(std::max(bi, 0), (int)NB - 1);
				return (uint32_t)bi <= best_split;
			});
			mid = (uint32_t)(pm - idx.data());
		} else {
			mid = e;
		}
		if (mid == b || mid == e) {
			/* median split on the widest centroid axis (or by index if degenerate) */
			int ax = 0;
			float w = -1.f;
			for (int a = 0; a < 3; a++)
				if (cb.hi[a] - cb.lo[a] > w) {
					w = cb.hi[a] - cb.lo[a];
					ax = a;
				}
			mid = b + n / 2;
			if (w > 0.f)
				std::nth_element(idx.data() + b, idx.data() + mid, idx.data() + e, [&](uint32_t x, uint32_t y) {
					return cent[3 * (size_t)x + ax] < cent[3 * (size_t)y + ax];
				});
		}
		uint32_t l = alloc(), r = alloc();
		TNode &t = tn[id];
		t.box = box;
		t.leaf = false;
		t.child[0] = (int32_t)l;
		t.child[1] = (int32_t)r;
		t.first = 0;
		t.count = n;
		if (n > 4096) {
#pragma omp task default(shared) firstprivate(l, b, mid, depth)
			build(l, b, mid, depth + 1);
#pragma omp task default(shared) firstprivate(r, mid, e, depth)
			build(r, mid, e, depth + 1);
#pragma omp taskwait
		} else {
			build(l, b, mid, depth + 1);
			build(r, mid, e, depth + 1);
		}
	}
};

struct Flattener {
	const std::vector<TNode> &tn;
	BvhOutput &out;
	uint32_t ref_of(int32_t id)
	{
		const TNode &t = tn[id];
		if (t.leaf)
			return RTX_LEAF_BIT | (t.first << 4) | (t.count - 1);
		uint32_t me = (uint32_t)out.nodes.size();
		out.nodes.push_back(DNode());
		const TNode &L = tn[t.child[0]], &R = tn[t.child[1]];
		uint32_t r0 = ref_of(t.child[0]);
		uint32_t r1 = ref_of(t.child[1]);
		DNode &d = out.nodes[me];
		d.lo0x = L.box.lo[0];
		d.hi0x = L.box.hi[0];
		d.lo0y = L.box.lo[1];
		d.hi0y = L.box.hi[1];
		d.lo0z = L.box.lo[2];
		d.hi0z = L.box.hi[2];
		d.lo1x = R.box.lo[0];
		d.hi1x = R.box.hi[0];
		d.lo1y = R.box.lo[1];
		d.hi1y = R.box.hi[1];
		d.lo1z = R.box.lo[2];
		d.hi1z = R.box.hi[2];
		d.ref0 = r0;
		d.ref1 = r1;
		/* split axis = axis of largest centroid separation, for near-first ordering */
		int ax = 0;
		float best = -FLT_MAX;
		for (int a = 0; a < 3; a++) {
			float s = std::fabs((L.box.lo[a] + L.box.hi[a]) - (R.box.lo[a] + R.box.hi[a]));
			if (s > best) {
				best = s;
				ax = a;
			}
		}
		const bool lcg = (L.box.lo[ax] + L.box.hi[ax]) > (R.box.lo[ax] + R.box.hi[ax]);
		d.order = 0;
		for (uint32_t o = 0; o < 8; o++) /* left first when the ray moves from the left centroid's side */
			d.order |= ((((o >> ax) & 1u) != 0) != lcg) ? 1u << o : 0u;
		d.pad = 0;
		return me;
	}
};

} // namespace

void bvh_build(const BvhInput &in, const BvhConfig &cfg, BvhOutput &out)
{
	out = BvhOutput();
	if (!in.n)
		return;
	Builder B(in, cfg);
	B.pbox.resize(in.n);
	B.cent.resize(3 * (size_t)in.n);
	B.idx.resize(in.n);
	for (uint32_t i = 0; i < in.n; i++) {
		for (int a = 0; a < 3; a++) {
			B.pbox[i].lo[a] = in.lo[3 * (size_t)i + a];
			B.pbox[i].hi[a] = in.hi[3 * (size_t)i + a];
			B.cent[3 * (size_t)i + a] = 0.5f * (in.lo[3 * (size_t)i + a] + in.hi[3 * (size_t)i + a]);
		}
		B.idx[i] = i;
	}
	B.tn.resize(2 * (size_t)in.n + 1);
	uint32_t root = B.alloc();
#pragma omp parallel
#pragma omp single
	B.build(root, 0, in.n, 1);

	Flattener F{ B.tn, out };
	out.nodes.reserve(in.n);
	out.root_ref = F.ref_of((int32_t)root);
	out.order = B.idx;
	out.depth = B.max_depth.load();
	uint32_t leaves = 0;
	for (uint32_t i = 0; i < B.ntn.load(); i++)
		if (B.tn[i].leaf)
			leaves++;
	out.leaves = leaves;
}
