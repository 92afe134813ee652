/*
 * The 8-wide compressed shadow BVH (rtx_device.h DW8), collapsed on the host from the BVH2 that
 * replaces the reference's tree (accel.c:266-315; any BVH answers is_light_blocked the same,
 * accel.c:360-387).  Every wide node opens its BVH2 subtree's top, the child of largest surface
 * area first, until it has eight children (the usual SAH-driven collapse); a leaf of several
 * primitives opens into one slot per primitive.  Child boxes are quantised to 8 bits in the
 * node's own frame on the 16-bit grid of the threaded BVH, rounded outward; slots follow the
 * children's centroid octant about the node centre, so the walk's slot order c ^ (~OCT & 7) is
 * front to back for a ray of direction octant OCT.
 */
#include <float.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <vector>

#include "rtx_internal.h"
#include "rtx_quant.h"

namespace {

struct Kid {
	uint32_t ref;  /* BVH2 device ref of a subtree (RTX_NONE: a single primitive) */
	uint32_t prim; /* record-order primitive index when ref == RTX_NONE */
	float lo[3], hi[3];
};

struct Builder {
	const std::vector<DNode> &inner;
	uint32_t nnodes;
	const DPrim *prims; /* host primitive records (leaves of several primitives only), or null */
	const QFrame &F;
	std::vector<DW8> &out;
	std::vector<uint32_t> &leafmap;
	bool ok = true;

	static bool is_leaf(uint32_t ref) { return (ref & RTX_REF_LEAF) != 0; }
	uint32_t leaf_first(uint32_t ref) const { return (ref & RTX_REF_OFF) / (uint32_t)sizeof(DNode) - nnodes; }
	static uint32_t leaf_count(uint32_t ref) { return (ref & RTX_REF_CNT) + 1; }

	/* a child ref with its box as a kid: single-primitive leaves become primitive kids */
	Kid kid(uint32_t ref, const float lo[3], const float hi[3]) const
	{
		Kid k;
		k.ref = ref;
		k.prim = RTX_NONE;
		memcpy(k.lo, lo, 12);
		memcpy(k.hi, hi, 12);
		if (is_leaf(ref) && leaf_count(ref) == 1) {
			k.prim = leaf_first(ref);
			k.ref = RTX_NONE;
		}
		return k;
	}

	/* a primitive's box from its record, padded like the leaf boxes of rtx_build_scene */
	Kid prim_kid(uint32_t i) const
	{
		const DPrim &p = prims[i];
		uint32_t meta;
		memcpy(&meta, &p.c[3], 4);
		Kid k;
		k.ref = RTX_NONE;
		k.prim = i;
		float l[3], h[3];
		for (int a = 0; a < 3; a++) {
			if ((meta >> 24) == RTX_SPHERE) {
				l[a] = p.a[a] - p.b[0];
				h[a] = p.a[a] + p.b[0];
			} else {
				const float v1 = p.a[a] + p.b[a], v2 = p.a[a] + p.c[a];
				l[a] = std::min(p.a[a], std::min(v1, v2));
				h[a] = std::max(p.a[a], std::max(v1, v2));
			}
		}
		const float ext = std::max(h[0] - l[0], std::max(h[1] - l[1], h[2] - l[2]));
		for (int a = 0; a < 3; a++) {
			k.lo[a] = l[a] - (std::fabs(l[a]) + ext) * 4e-6f - 1e-30f;
			k.hi[a] = h[a] + (std::fabs(h[a]) + ext) * 4e-6f + 1e-30f;
		}
		return k;
	}

	static float half_area(const Kid &k)
	{
		const float dx = k.hi[0] - k.lo[0], dy = k.hi[1] - k.lo[1], dz = k.hi[2] - k.lo[2];
		return dx * dy + dy * dz + dz * dx;
	}

	/* how many slots opening k adds (0: not openable) */
	uint32_t grows(const Kid &k) const
	{
		if (k.ref == RTX_NONE)
			return 0;
		if (!is_leaf(k.ref))
			return 1;
		return prims ? leaf_count(k.ref) - 1 : 0;
	}

	/* the children of the wide node made from the subtree `seed`: open the largest openable kid
	 * while it fits into eight slots */
	void open_kids(const Kid &seed, Kid kids[8], uint32_t &n) const
	{
		kids[0] = seed;
		n = 1;
		for (;;) {
			int best = -1;
			float ba = -1.f;
			for (uint32_t i = 0; i < n; i++) {
				const uint32_t g = grows(kids[i]);
				if (g && n + g <= 8 && half_area(kids[i]) > ba) {
					ba = half_area(kids[i]);
					best = (int)i;
				}
			}
			if (best < 0)
				break;
			const Kid k = kids[best];
			if (!is_leaf(k.ref)) {
				const DNode &d = inner[(k.ref & RTX_REF_OFF) / (uint32_t)sizeof(DNode)];
				const float l0[3] = { d.lo0x, d.lo0y, d.lo0z }, h0[3] = { d.hi0x, d.hi0y, d.hi0z };
				const float l1[3] = { d.lo1x, d.lo1y, d.lo1z }, h1[3] = { d.hi1x, d.hi1y, d.hi1z };
				kids[best] = kid(d.ref0, l0, h0);
				kids[n++] = kid(d.ref1, l1, h1);
			} else {
				const uint32_t first = leaf_first(k.ref), cnt = leaf_count(k.ref);
				kids[best] = prim_kid(first);
				for (uint32_t j = 1; j < cnt; j++)
					kids[n++] = prim_kid(first + j);
			}
		}
	}

	/* slot of each kid: greedy assignment of the best (kid, slot) pairs, where slot s's score is
	 * how far the kid's centroid lies towards octant s of the node centre (extent-normalised) */
	static void assign_slots(const Kid *kids, uint32_t n, int slot_of[8])
	{
		float lo[3] = { FLT_MAX, FLT_MAX, FLT_MAX }, hi[3] = { -FLT_MAX, -FLT_MAX, -FLT_MAX };
		for (uint32_t i = 0; i < n; i++)
			for (int a = 0; a < 3; a++) {
				lo[a] = std::min(lo[a], kids[i].lo[a]);
				hi[a] = std::max(hi[a], kids[i].hi[a]);
			}
		float score[8][8];
		for (uint32_t i = 0; i < n; i++) {
			float off[3];
			for (int a = 0; a < 3; a++) {
				const float ext = std::max(hi[a] - lo[a], 1e-30f);
				off[a] = (0.5f * (kids[i].lo[a] + kids[i].hi[a]) - 0.5f * (lo[a] + hi[a])) / ext;
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

	/* node entry `me` from its children; returns the depth of its subtree (1 = leaves only) */
	uint32_t emit(uint32_t me, const Kid *kids, uint32_t n)
	{
		if (out.size() + 8 > RTX_W8_MAX_ENTRIES) {
			ok = false;
			return 0;
		}
		const uint32_t base = (uint32_t)out.size();
		out.resize(base + 8);
		leafmap.resize(base + 8, RTX_NONE);
		memset(&out[base], 0, 8 * sizeof(DW8));
		int slot_of[8];
		assign_slots(kids, n, slot_of);
		/* 16-bit grid boxes of the children, the node origin and per-axis steps */
		uint32_t ql[8][3], qh[8][3], org[3], ex[3];
		for (int a = 0; a < 3; a++) {
			uint32_t mn = 0xFFFFu, mx = 0;
			for (uint32_t i = 0; i < n; i++) {
				const uint32_t q = rtx_quantise(kids[i].lo[a], kids[i].hi[a], F.qo[a], F.qs[a]);
				ql[i][a] = q & 0xFFFFu;
				qh[i][a] = q >> 16;
				mn = std::min(mn, ql[i][a]);
				mx = std::max(mx, qh[i][a]);
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
		uint32_t imask = 0, vmask = 0;
		for (uint32_t i = 0; i < n; i++) {
			const int s = slot_of[i];
			for (int a = 0; a < 3; a++) {
				const uint32_t q8 = rtx_quantise8(ql[i][a] | (qh[i][a] << 16), org[a], ex[a]);
				lo8[a][s] = (uint8_t)(q8 & 0xFFu);
				hi8[a][s] = (uint8_t)(q8 >> 8);
			}
			vmask |= 1u << s;
			if (kids[i].ref != RTX_NONE)
				imask |= 1u << s;
			else
				leafmap[base + s] = kids[i].prim;
		}
		DW8 &N = out[me];
		N.w[0] = org[0] | (org[1] << 16);
		N.w[1] = org[2] | (ex[0] << 16) | (ex[1] << 20) | (ex[2] << 24);
		N.w[2] = (base << 8) | imask;
		N.w[3] = vmask;
		for (int a = 0; a < 3; a++) {
			memcpy(&N.w[4 + 4 * a], lo8[a], 8);
			memcpy(&N.w[6 + 4 * a], hi8[a], 8);
		}
		uint32_t dep = 1;
		for (uint32_t i = 0; i < n && ok; i++) {
			if (kids[i].ref == RTX_NONE)
				continue;
			Kid sub[8];
			uint32_t m = 0;
			open_kids(kids[i], sub, m);
			if (m == 1 && sub[0].ref != RTX_NONE) { /* a leaf of more than eight primitives */
				ok = false;
				return 0;
			}
			dep = std::max(dep, 1 + emit(base + (uint32_t)slot_of[i], sub, m));
		}
		return dep;
	}
};

} // namespace

/* Collapses the BVH2 (inner records `inner`, root `root_ref`, bounded objects' box lo/hi) into
 * the 8-wide entries `out` (frame F) and the map entry -> primitive index of the leaf slots.
 * prims: the host primitive records (needed only when a leaf holds several primitives).  Returns
 * the wide tree's depth, or 0 when it cannot be built (empty tree, more than 2^24 entries, a
 * leaf of more than eight primitives or of several without host records). */
uint32_t rtx_wide8_build(const std::vector<DNode> &inner, uint32_t nnodes, const DPrim *prims, uint32_t root_ref,
			 const float lo[3], const float hi[3], const QFrame &F, std::vector<DW8> &out,
			 std::vector<uint32_t> &leafmap)
{
	out.clear();
	leafmap.clear();
	if (root_ref == RTX_EMPTY_REF)
		return 0;
	Builder b{ inner, nnodes, prims, F, out, leafmap };
	out.resize(2);
	leafmap.assign(2, RTX_NONE);
	memset(out.data(), 0, 2 * sizeof(DW8));
	Kid kids[8];
	uint32_t n = 0;
	b.open_kids(b.kid(root_ref, lo, hi), kids, n);
	if (n == 1 && kids[0].ref != RTX_NONE) {
		out.clear();
		leafmap.clear();
		return 0;
	}
	const uint32_t dep = b.emit(0, kids, n);
	if (!b.ok) {
		out.clear();
		leafmap.clear();
		return 0;
	}
	return dep;
}
