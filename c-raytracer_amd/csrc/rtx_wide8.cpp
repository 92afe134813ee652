/*
 * The 8-wide compressed shadow BVH (rtx_device.h DW8), collapsed on the host from the BVH2 that
 * replaces the reference's tree (accel.c:266-315; any BVH answers is_light_blocked the same,
 * accel.c:360-387).
 *
 * Which BVH2 nodes become wide nodes is decided by a surface-area cost optimisation over the
 * BVH2 (the dynamic programme of Ylitie, Karras and Laine's compressed wide BVH): C(n, j) is
 * the least expected cost of the subtree n spread over at most j slots of its wide parent,
 *   C(prim, j)  = A(prim) * c_prim                                  (a leaf slot)
 *   C(n, 1)     = A(n) * c_node + D(n, 8)                           (n becomes a wide node)
 *   C(n, j > 1) = min(C(n, j - 1), D(n, j)),  D(n, j) = min_k C(l, k) + C(r, j - k)
 * with A the box's surface area.  A leaf of several primitives enters the programme as a
 * balanced binary tree of its primitives (boxes from the host records).  Primitives of the
 * objects in skip_objs (the emitters) are left out when the host has the records, and the
 * boxes are refitted bottom-up; the tree gets its own 16-bit frame over what remains.  Child
 * boxes are
 * quantised to 8 bits in the node's own frame on the 16-bit grid of the threaded BVH, rounded
 * outward; slots follow the children's centroid octant about the node centre, so the walk's
 * slot order c ^ (~OCT & 7) is front to back for a ray of direction octant OCT.
 */
#include <float.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <vector>

#include "rtx_internal.h"
#include "rtx_quant.h"

namespace {

/* expected-cost weights of a node visit (one 64-byte fetch, eight box tests) and of a primitive
 * test, per unit of surface area */
#ifndef RTX_W8_C_PRIM
#define RTX_W8_C_PRIM 0.3f
#endif
constexpr float C_NODE = 1.0f;
constexpr float C_PRIM = RTX_W8_C_PRIM;

struct TNode {
	float lo[3], hi[3];
	int32_t kid[2];  /* tree indices, -1 for a primitive */
	uint32_t prim;   /* primitive index (record order) when kid[0] < 0 */
};

struct Slot {
	int32_t t;   /* tree index */
	bool node;   /* becomes a wide node (else a primitive's leaf slot) */
};

struct Builder {
	const std::vector<DNode> &inner;
	uint32_t nnodes;
	const DPrim *prims;
	const std::vector<uint32_t> &skip_objs;
	QFrame F;
	DTreeFrame tf{};   /* the frame the tree's boxes are in (rtx_device.h DTreeFrame) */
	double fpad = 0;   /* its transform padding (rtx_frame.cpp) */
	std::vector<DW8> &out;
	std::vector<uint32_t> &leafmap;
	std::vector<TNode> tree;
	std::vector<float> cost;   /* [t * 9 + j], j = 1..8 */
	std::vector<int8_t> pick;  /* [t * 9 + j]: 0 = C(t, j - 1), k > 0 = split k / j - k, -1 = wide node (j = 1) */
	bool ok = true;

	static float area(const float lo[3], const float hi[3])
	{
		const float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
		return dx * dy + dy * dz + dz * dx;
	}

	/* a primitive's box from its record, in the trees' frame, padded like the leaf boxes of
	 * rtx_build_scene (twice the relative padding: v0 + e1 is v1 only to float rounding) */
	void prim_box(uint32_t i, float lo[3], float hi[3]) const
	{
		const DPrim &p = prims[i];
		uint32_t meta;
		memcpy(&meta, &p.c[3], 4);
		const bool sph = (meta >> 24) == RTX_SPHERE;
		double l[3], h[3];
		for (int a = 0; a < 3; a++) {
			if (!tf.rotated) {
				if (sph) {
					l[a] = (float)(p.a[a] - p.b[0]);
					h[a] = (float)(p.a[a] + p.b[0]);
				} else {
					const float v1 = p.a[a] + p.b[a], v2 = p.a[a] + p.c[a];
					l[a] = std::min(p.a[a], std::min(v1, v2));
					h[a] = std::max(p.a[a], std::max(v1, v2));
				}
				continue;
			}
			/* x' = R (x - c) of the vertices (or the sphere's centre +- its radius along row a) */
			auto rot = [&](const float v[3]) {
				double y = 0;
				for (int j = 0; j < 3; j++)
					y += (double)tf.r[a][j] * ((double)v[j] - tf.c[j]);
				return y;
			};
			if (sph) {
				double rn = 0;
				for (int j = 0; j < 3; j++)
					rn += (double)tf.r[a][j] * tf.r[a][j];
				l[a] = rot(p.a) - p.b[0] * std::sqrt(rn);
				h[a] = rot(p.a) + p.b[0] * std::sqrt(rn);
			} else {
				const float v1[3] = { p.a[0] + p.b[0], p.a[1] + p.b[1], p.a[2] + p.b[2] };
				const float v2[3] = { p.a[0] + p.c[0], p.a[1] + p.c[1], p.a[2] + p.c[2] };
				l[a] = std::min(rot(p.a), std::min(rot(v1), rot(v2)));
				h[a] = std::max(rot(p.a), std::max(rot(v1), rot(v2)));
			}
		}
		const double ext = std::max(h[0] - l[0], std::max(h[1] - l[1], h[2] - l[2]));
		for (int a = 0; a < 3; a++) {
			lo[a] = (float)(l[a] - (std::fabs(l[a]) + ext) * 4e-6 - fpad) - 1e-30f;
			hi[a] = (float)(h[a] + (std::fabs(h[a]) + ext) * 4e-6 + fpad) + 1e-30f;
		}
	}

	bool skipped(uint32_t prim) const
	{
		if (!prims || skip_objs.empty())
			return false;
		uint32_t obj;
		memcpy(&obj, &prims[prim].b[3], 4);
		return std::find(skip_objs.begin(), skip_objs.end(), obj) != skip_objs.end();
	}

	/* an inner tree node over children a and b (either may be -1: nothing left), box = union */
	int32_t join(int32_t a, int32_t b)
	{
		if (a < 0 || b < 0)
			return a < 0 ? b : a;
		TNode t;
		for (int k = 0; k < 3; k++) {
			t.lo[k] = std::min(tree[a].lo[k], tree[b].lo[k]);
			t.hi[k] = std::max(tree[a].hi[k], tree[b].hi[k]);
		}
		t.kid[0] = a;
		t.kid[1] = b;
		t.prim = RTX_NONE;
		tree.push_back(t);
		return (int32_t)tree.size() - 1;
	}

	int32_t leaf(uint32_t prim, const float lo[3], const float hi[3])
	{
		if (skipped(prim))
			return -1;
		TNode t;
		memcpy(t.lo, lo, 12);
		memcpy(t.hi, hi, 12);
		t.kid[0] = t.kid[1] = -1;
		t.prim = prim;
		tree.push_back(t);
		return (int32_t)tree.size() - 1;
	}

	/* primitives [first, first + cnt) of a BVH2 leaf as a balanced subtree of single primitives */
	int32_t add_prims(uint32_t first, uint32_t cnt)
	{
		if (cnt == 1) {
			float lo[3], hi[3];
			prim_box(first, lo, hi);
			return leaf(first, lo, hi);
		}
		const uint32_t h = cnt / 2;
		const int32_t a = add_prims(first, h);
		return join(a, add_prims(first + h, cnt - h));
	}

	/* the BVH2 subtree at device ref `ref` (box lo/hi in its parent) into `tree`, children
	 * before their parent; -1 when nothing of it is left */
	int32_t add(uint32_t ref, const float lo[3], const float hi[3])
	{
		if (ref & RTX_REF_LEAF) {
			const uint32_t first = (ref & RTX_REF_OFF) / (uint32_t)sizeof(DNode) - nnodes, cnt = (ref & RTX_REF_CNT) + 1;
			if (cnt == 1)
				return leaf(first, lo, hi);
			if (!prims) {
				ok = false;
				return -1;
			}
			return add_prims(first, cnt);
		}
		const DNode &d = inner[(ref & RTX_REF_OFF) / (uint32_t)sizeof(DNode)];
		const float l0[3] = { d.lo0x, d.lo0y, d.lo0z }, h0[3] = { d.hi0x, d.hi0y, d.hi0z };
		const float l1[3] = { d.lo1x, d.lo1y, d.lo1z }, h1[3] = { d.hi1x, d.hi1y, d.hi1z };
		const int32_t a = add(d.ref0, l0, h0);
		return join(a, add(d.ref1, l1, h1));
	}

	/* the cost programme over all tree nodes; children always precede their parent */
	void solve()
	{
		const size_t n = tree.size();
		cost.assign(n * 9, FLT_MAX);
		pick.assign(n * 9, 0);
		for (size_t t = 0; t < n; t++) {
			const TNode &x = tree[t];
			const float A = area(x.lo, x.hi);
			float *C = &cost[t * 9];
			int8_t *P = &pick[t * 9];
			if (x.kid[0] < 0) {
				for (int j = 1; j <= 8; j++)
					C[j] = A * C_PRIM;
				continue;
			}
			const float *L = &cost[(size_t)x.kid[0] * 9], *R = &cost[(size_t)x.kid[1] * 9];
			float D[9];
			int8_t K[9];
			for (int j = 2; j <= 8; j++) {
				D[j] = FLT_MAX;
				K[j] = 1;
				for (int k = 1; k < j; k++) {
					const float v = L[k] + R[j - k];
					if (v < D[j]) {
						D[j] = v;
						K[j] = (int8_t)k;
					}
				}
			}
			C[1] = A * C_NODE + D[8];
			P[1] = -1;
			for (int j = 2; j <= 8; j++) {
				if (D[j] < C[j - 1]) {
					C[j] = D[j];
					P[j] = K[j];
				} else {
					C[j] = C[j - 1];
					P[j] = 0;
				}
			}
		}
	}

	/* the slots subtree t fills when given j of them */
	void slots(int32_t t, int j, std::vector<Slot> &s) const
	{
		const TNode &x = tree[t];
		if (x.kid[0] < 0) {
			s.push_back(Slot{ t, false });
			return;
		}
		for (;;) {
			const int8_t p = pick[(size_t)t * 9 + j];
			if (p < 0) {
				s.push_back(Slot{ t, true });
				return;
			}
			if (p == 0) {
				j--;
				continue;
			}
			slots(x.kid[0], p, s);
			slots(x.kid[1], j - p, s);
			return;
		}
	}

	/* the children of the wide node made from tree node t: its eight slots distributed */
	void children(int32_t t, std::vector<Slot> &s) const
	{
		s.clear();
		const TNode &x = tree[t];
		if (x.kid[0] < 0) { /* a single primitive as the root */
			s.push_back(Slot{ t, false });
			return;
		}
		/* D(t, 8): the best split of eight slots over its two subtrees */
		const float *L = &cost[(size_t)x.kid[0] * 9], *R = &cost[(size_t)x.kid[1] * 9];
		int best = 1;
		for (int k = 2; k < 8; k++)
			if (L[k] + R[8 - k] < L[best] + R[8 - best])
				best = k;
		slots(x.kid[0], best, s);
		slots(x.kid[1], 8 - best, s);
	}

	/* slot of each child: greedy assignment of the best (child, slot) pairs, where slot s's score
	 * is how far the child's centroid lies towards octant s of the node centre (extent-normalised) */
	void assign_slots(const std::vector<Slot> &kids, int slot_of[8]) const
	{
		const uint32_t n = (uint32_t)kids.size();
		float lo[3] = { FLT_MAX, FLT_MAX, FLT_MAX }, hi[3] = { -FLT_MAX, -FLT_MAX, -FLT_MAX };
		for (uint32_t i = 0; i < n; i++)
			for (int a = 0; a < 3; a++) {
				lo[a] = std::min(lo[a], tree[kids[i].t].lo[a]);
				hi[a] = std::max(hi[a], tree[kids[i].t].hi[a]);
			}
		float score[8][8];
		for (uint32_t i = 0; i < n; i++) {
			const TNode &k = tree[kids[i].t];
			float off[3];
			for (int a = 0; a < 3; a++) {
				const float ext = std::max(hi[a] - lo[a], 1e-30f);
				off[a] = (0.5f * (k.lo[a] + k.hi[a]) - 0.5f * (lo[a] + hi[a])) / ext;
			}
			for (int s = 0; s < 8; s++)
				score[i][s] = ((s & 1) ? off[0] : -off[0]) + ((s & 2) ? off[1] : -off[1]) + ((s & 4) ? off[2] : -off[2]);
		}
		bool kid_done[8] = {}, slot_used[8] = {};
		for (uint32_t r = 0; r < n; r++) {
			int bi = -1, bs = -1;
			float bv = -FLT_MAX;
			for (uint32_t i = 0; i < n; i++) {
				if (kid_done[i])
					continue;
				for (int s = 0; s < 8; s++)
					if (!slot_used[s] && (bi < 0 || score[i][s] > bv)) {
						bv = score[i][s];
						bi = (int)i;
						bs = s;
					}
			}
			kid_done[bi] = true;
			slot_used[bs] = true;
			slot_of[bi] = bs;
		}
	}

	/* node entry `me` for tree node t; returns the depth of its subtree (1 = leaf slots only) */
	uint32_t emit(uint32_t me, int32_t t)
	{
		if (out.size() + 8 > RTX_W8_MAX_ENTRIES) {
			ok = false;
			return 0;
		}
		std::vector<Slot> kids;
		children(t, kids);
		const uint32_t n = (uint32_t)kids.size();
		const uint32_t base = (uint32_t)out.size();
		out.resize(base + 8);
		leafmap.resize(base + 8, RTX_NONE);
		memset(&out[base], 0, 8 * sizeof(DW8));
		int slot_of[8];
		assign_slots(kids, slot_of);
		/* 16-bit grid boxes of the children, the node origin and per-axis steps */
		uint32_t q16[8][3], org[3], ex[3];
		for (int a = 0; a < 3; a++) {
			uint32_t mn = 0xFFFFu, mx = 0;
			for (uint32_t i = 0; i < n; i++) {
				const TNode &k = tree[kids[i].t];
				q16[i][a] = rtx_quantise(k.lo[a], k.hi[a], F.qo[a], F.qs[a]);
				mn = std::min(mn, q16[i][a] & 0xFFFFu);
				mx = std::max(mx, q16[i][a] >> 16);
			}
			org[a] = mn;
			uint32_t e = 0;
			while (((mx - mn) + (1u << e) - 1) >> e > 255u)
				e++;
			ex[a] = e;
		}
		uint8_t lo8[3][8], hi8[3][8];
		memset(lo8, 255, sizeof(lo8));
		memset(hi8, 0, sizeof(hi8));
		uint32_t imask = 0, vmask = 0, tmask = 0;
		for (uint32_t i = 0; i < n; i++) {
			const int s = slot_of[i];
			for (int a = 0; a < 3; a++) {
				const uint32_t q8 = rtx_quantise8(q16[i][a], org[a], ex[a]);
				lo8[a][s] = (uint8_t)(q8 & 0xFFu);
				hi8[a][s] = (uint8_t)(q8 >> 8);
			}
			vmask |= 1u << s;
			if (kids[i].node) {
				imask |= 1u << s;
			} else {
				const uint32_t pr = tree[kids[i].t].prim;
				leafmap[base + s] = pr;
				uint32_t meta = 0; /* without host records no slot is marked (its test is not deferred) */
				if (prims)
					memcpy(&meta, &prims[pr].c[3], 4);
				if (meta & RTX_META_TRANSPARENT)
					tmask |= 1u << s;
			}
		}
		DW8 &N = out[me];
		N.w[0] = org[0] | (org[1] << 16);
		N.w[1] = org[2] | (ex[0] << 16) | (ex[1] << 20) | (ex[2] << 24);
		N.w[2] = (base << 8) | imask;
		N.w[3] = vmask | (tmask << 8);
		for (int a = 0; a < 3; a++) {
			memcpy(&N.w[4 + 4 * a], lo8[a], 8);
			memcpy(&N.w[6 + 4 * a], hi8[a], 8);
		}
		uint32_t dep = 1;
		for (uint32_t i = 0; i < n && ok; i++)
			if (kids[i].node)
				dep = std::max(dep, 1 + emit(base + (uint32_t)slot_of[i], kids[i].t));
		return dep;
	}
};

} // namespace

/* Collapses the BVH2 (inner records `inner`, root `root_ref`, bounded objects' box lo/hi) into
 * the 8-wide entries `out` and the map entry -> primitive index of the leaf slots, leaving out
 * the primitives of the objects in skip_objs when the host records `prims` are given (skipped =
 * true then).  F receives the tree's 16-bit frame.  Returns the wide tree's depth, or 0 when it
 * cannot be built (empty tree, more than 2^24 entries, a leaf of several primitives without
 * host records). */
uint32_t rtx_wide8_build(const std::vector<DNode> &inner, uint32_t nnodes, const DPrim *prims, uint32_t root_ref,
			 const float lo[3], const float hi[3], const std::vector<uint32_t> &skip_objs, const DTreeFrame &tf,
			 double fpad, QFrame &F, bool &skipped, std::vector<DW8> &out, std::vector<uint32_t> &leafmap)
{
	out.clear();
	leafmap.clear();
	skipped = false;
	if (root_ref == RTX_EMPTY_REF)
		return 0;
	Builder b{ inner, nnodes, prims, skip_objs, QFrame{}, tf, fpad, out, leafmap };
	b.tree.reserve(2 * (size_t)nnodes + 2);
	const int32_t root = b.add(root_ref, lo, hi);
	if (!b.ok || root < 0) {
		out.clear();
		leafmap.clear();
		return 0;
	}
	skipped = prims && !skip_objs.empty();
	/* the frame: the remaining primitives' box, 65533 steps per axis (as the threaded BVH's) */
	const TNode &R = b.tree[root];
	float ext_max = 0.f;
	for (int a = 0; a < 3; a++)
		ext_max = std::max(ext_max, R.hi[a] - R.lo[a]);
	for (int a = 0; a < 3; a++) {
		b.F.qo[a] = R.lo[a];
		b.F.qs[a] = 65533.f / std::max(R.hi[a] - R.lo[a], std::max(ext_max, 1.f) * 1e-6f);
	}
	F = b.F;
	b.solve();
	out.resize(2);
	leafmap.assign(2, RTX_NONE);
	memset(out.data(), 0, 2 * sizeof(DW8));
	const uint32_t dep = b.emit(0, root);
	if (!b.ok) {
		out.clear();
		leafmap.clear();
		return 0;
	}
	return dep;
}
