/*
 * The 8-wide compressed shadow BVH (rtx_device.h DW8) collapsed on the device, for the device
 * builders (rtx_build.hip): the same surface-area cost programme as the host collapse
 * (rtx_wide8.cpp, Ylitie, Karras and Laine's compressed wide BVH) over the BVH2 records the
 * builder left in HBM, so a GPU build never round-trips the tree through the host.
 *
 *   k_w8d_parent  parent of every BVH2 node; leaf boxes from their parent's record
 *   k_w8d_leaves / k_w8d_depth / k_w8d_bucket / k_w8d_level
 *                 bottom-up, one launch per BVH2 depth from the deepest: the emitters'
 *                 primitives left out, boxes refitted over what remains, and the cost table
 *                 C(n, 1..8) with its choices per node (a node with one side left becomes an
 *                 alias of that side, as the host collapse's join)
 *   k_w8d_emit    top-down, one launch per wide-tree level: each wide node distributes its
 *                 eight slots over the programme's choices, orders them by centroid octant,
 *                 quantises the child boxes to 8 bits in its own frame and lists its inner
 *                 children for the next level (their entry blocks follow in level order)
 *   k_w8d_scalar  the scalar-path copies (DW8S) of the inner entries
 * Levels are laid out breadth-first (the host collapse: depth-first); the walk reads either.
 * Single-primitive BVH2 leaves only (the default RTX_OPT_BVH_LEAF 1); rtx_api.cpp keeps the
 * host collapse for larger leaves.
 */
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <float.h>
#include <stdint.h>

#include <vector>

#include "rtx.h"
#include "rtx_device.h"
#include "rtx_quant.h"

#ifndef RTX_W8_C_PRIM
#define RTX_W8_C_PRIM 0.3f
#endif
#define W8D_T 256
#define W8D_EMPTY 0u
#define W8D_FULL 1u
#define W8D_ALIAS 2u

namespace {

__device__ __forceinline__ float area6(const float (&b)[6])
{
	const float dx = b[3] - b[0], dy = b[4] - b[1], dz = b[5] - b[2];
	return dx * dy + dy * dz + dz * dx;
}

/* tree node id of a BVH2 child ref: inner record index, or nnodes + primitive index */
__device__ __forceinline__ uint32_t child_id(uint32_t ref, uint32_t nnodes)
{
	return (ref & RTX_REF_OFF) / (uint32_t)sizeof(DNode);
}

struct W8Tree {
	const DNode *recs;
	uint32_t nnodes, nb;
	uint32_t *parent; /* [nnodes + nb] */
	float *box;       /* [nnodes + nb][6] lo xyz, hi xyz */
	uint32_t *state;  /* [nnodes + nb] W8D_* */
	uint32_t *eff;    /* [nnodes + nb]: the node itself (full / leaf), its alias target, or RTX_NONE */
	uint2 *ekids;     /* [nnodes]: effective children of full inner nodes */
	float *cost;      /* [nnodes + nb][8]: C(n, j) for j = 1..8 */
	int8_t *pick;     /* [nnodes + nb][8] */
};

} // namespace

__global__ __launch_bounds__(W8D_T) void k_w8d_parent(W8Tree T)
{
	const uint32_t i = blockIdx.x * W8D_T + threadIdx.x;
	if (i >= T.nnodes)
		return;
	const DNode d = T.recs[i];
	const float *f = &d.lo0x;
	const uint32_t ref[2] = { d.ref0, d.ref1 };
	for (int c = 0; c < 2; c++) {
		const uint32_t id = child_id(ref[c], T.nnodes);
		T.parent[id] = i;
		if (ref[c] & RTX_REF_LEAF) /* a primitive's box: its parent's record */
			for (int a = 0; a < 3; a++) {
				T.box[6 * (size_t)id + a] = f[6 * c + 2 * a];
				T.box[6 * (size_t)id + 3 + a] = f[6 * c + 2 * a + 1];
			}
	}
	if (i == 0)
		T.parent[0] = RTX_NONE;
}

/* a primitive's tree node: left out (an emitter) or a leaf slot of cost A * c_prim */
__device__ __forceinline__ void w8d_leaf(const W8Tree &T, uint32_t k, const uint32_t *__restrict__ skip_obj, uint32_t num_objects)
{
	const uint32_t leaf = T.nnodes + k;
	const DPrim &p = *(const DPrim *)(T.recs + leaf);
	const uint32_t obj = __float_as_uint(p.b[3]);
	const bool skip = obj < num_objects && ((skip_obj[obj >> 5] >> (obj & 31u)) & 1u);
	if (skip) {
		T.state[leaf] = W8D_EMPTY;
		T.eff[leaf] = RTX_NONE;
		return;
	}
	float b[6];
	for (int a = 0; a < 6; a++)
		b[a] = T.box[6 * (size_t)leaf + a];
	const float c = area6(b) * RTX_W8_C_PRIM;
	for (int j = 0; j < 8; j++) {
		T.cost[8 * (size_t)leaf + j] = c;
		T.pick[8 * (size_t)leaf + j] = 0;
	}
	T.state[leaf] = W8D_FULL;
	T.eff[leaf] = leaf;
}

/* an inner BVH2 node once both children are done: empty, an alias of its one remaining side, or
 * a full node with its refitted box and cost table C(n, 1..8) (the host programme,
 * rtx_wide8.cpp Builder::solve) */
__device__ __forceinline__ void w8d_node(const W8Tree &T, uint32_t node)
{
	const DNode &d = T.recs[node];
	const uint32_t ea = T.eff[child_id(d.ref0, T.nnodes)], eb = T.eff[child_id(d.ref1, T.nnodes)];
	if (ea == RTX_NONE && eb == RTX_NONE) {
		T.state[node] = W8D_EMPTY;
		T.eff[node] = RTX_NONE;
		return;
	}
	if (ea == RTX_NONE || eb == RTX_NONE) { /* one side left: the node is that side */
		T.state[node] = W8D_ALIAS;
		T.eff[node] = ea == RTX_NONE ? eb : ea;
		return;
	}
	float b[6], L[9], R[9];
	for (int a = 0; a < 3; a++) {
		b[a] = fminf(T.box[6 * (size_t)ea + a], T.box[6 * (size_t)eb + a]);
		b[3 + a] = fmaxf(T.box[6 * (size_t)ea + 3 + a], T.box[6 * (size_t)eb + 3 + a]);
	}
	for (int j = 1; j <= 8; j++) {
		L[j] = T.cost[8 * (size_t)ea + j - 1];
		R[j] = T.cost[8 * (size_t)eb + j - 1];
	}
	float D[9], C[9];
	int8_t K[9], P[9];
	for (int j = 2; j <= 8; j++) {
		D[j] = FLT_MAX;
		K[j] = 1;
		for (int q = 1; q < j; q++) {
			const float v = L[q] + R[j - q];
			if (v < D[j]) {
				D[j] = v;
				K[j] = (int8_t)q;
			}
		}
	}
	C[1] = area6(b) * 1.0f + D[8];
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
	for (int a = 0; a < 6; a++)
		T.box[6 * (size_t)node + a] = b[a];
	for (int j = 1; j <= 8; j++) {
		T.cost[8 * (size_t)node + j - 1] = C[j];
		T.pick[8 * (size_t)node + j - 1] = P[j];
	}
	T.ekids[node] = make_uint2(ea, eb);
	T.state[node] = W8D_FULL;
	T.eff[node] = node;
}

/* bottom-up, level by level (no arrival counters or device-scope fences): every primitive's
 * leaf, then each inner node's depth (its parent chain) bucketed by depth, then one launch per
 * depth from the deepest, each node's children finished by the launches before */
__global__ __launch_bounds__(W8D_T) void k_w8d_leaves(W8Tree T, const uint32_t *__restrict__ skip_obj, uint32_t num_objects)
{
	const uint32_t k = blockIdx.x * W8D_T + threadIdx.x;
	if (k < T.nb)
		w8d_leaf(T, k, skip_obj, num_objects);
}
#define W8D_MAXDEPTH 1024
/* each inner node's depth (its parent chain), counted per depth: a workgroup counts in LDS and
 * adds its counts once (one global atomic per depth per workgroup, not per node: the few depth
 * counters serialised 327K atomics, 1.6 ms) */
__global__ __launch_bounds__(W8D_T) void k_w8d_depth(W8Tree T, uint32_t *__restrict__ depth, uint32_t *__restrict__ hist)
{
	__shared__ uint32_t h[W8D_MAXDEPTH + 1];
	for (uint32_t b = threadIdx.x; b <= W8D_MAXDEPTH; b += W8D_T)
		h[b] = 0;
	__syncthreads();
	const uint32_t i = blockIdx.x * W8D_T + threadIdx.x;
	if (i < T.nnodes) {
		uint32_t d = 0;
		for (uint32_t n = T.parent[i]; n != RTX_NONE && d < W8D_MAXDEPTH; n = T.parent[n])
			d++;
		depth[i] = d;
		atomicAdd(&h[d], 1u); /* d = W8D_MAXDEPTH: too deep, the host gives up */
	}
	__syncthreads();
	for (uint32_t b = threadIdx.x; b <= W8D_MAXDEPTH; b += W8D_T)
		if (h[b])
			atomicAdd(&hist[b], h[b]);
}
/* the inner nodes bucketed by depth: a workgroup ranks its nodes per depth in LDS and reserves
 * each depth's range with one global atomic */
__global__ __launch_bounds__(W8D_T) void k_w8d_bucket(uint32_t n, const uint32_t *__restrict__ depth, uint32_t *__restrict__ cursor,
						      uint32_t *__restrict__ order)
{
	__shared__ uint32_t cnt[W8D_MAXDEPTH], base[W8D_MAXDEPTH];
	for (uint32_t b = threadIdx.x; b < W8D_MAXDEPTH; b += W8D_T)
		cnt[b] = 0;
	__syncthreads();
	const uint32_t i = blockIdx.x * W8D_T + threadIdx.x;
	const uint32_t d = i < n ? depth[i] : 0u, r = i < n ? atomicAdd(&cnt[d], 1u) : 0u;
	__syncthreads();
	for (uint32_t b = threadIdx.x; b < W8D_MAXDEPTH; b += W8D_T)
		if (cnt[b])
			base[b] = atomicAdd(&cursor[b], cnt[b]);
	__syncthreads();
	if (i < n)
		order[base[d] + r] = i;
}
__global__ __launch_bounds__(W8D_T) void k_w8d_level(W8Tree T, const uint32_t *__restrict__ nodes, uint32_t m)
{
	const uint32_t i = blockIdx.x * W8D_T + threadIdx.x;
	if (i < m)
		w8d_node(T, nodes[i]);
}

/* one wide node of a level: its slots, their order, the quantised entry, its inner children */
__global__ __launch_bounds__(W8D_T) void k_w8d_emit(W8Tree T, uint32_t m, const uint2 *__restrict__ items, uint32_t blk,
						    float qo0, float qo1, float qo2, float qs0, float qs1, float qs2,
						    DW8 *__restrict__ out, uint32_t *__restrict__ leafmap, uint32_t *__restrict__ nxt,
						    uint32_t *__restrict__ ncnt)
{
	const uint32_t k = blockIdx.x * W8D_T + threadIdx.x;
	if (k >= m)
		return;
	const uint32_t t = items[k].x, me = items[k].y, base = blk + 8 * k;
	const float qo[3] = { qo0, qo1, qo2 }, qs[3] = { qs0, qs1, qs2 };
	/* the children: eight slots over the two subtrees (Builder::children / slots) */
	uint32_t kid[8];
	bool knode[8];
	uint32_t n = 0;
	if (t >= T.nnodes) {
		kid[0] = t;
		knode[0] = false;
		n = 1;
	} else {
		const uint2 ek = T.ekids[t];
		const float *L = T.cost + 8 * (size_t)ek.x, *R = T.cost + 8 * (size_t)ek.y;
		int best = 1;
		for (int q = 2; q < 8; q++)
			if (L[q - 1] + R[8 - q - 1] < L[best - 1] + R[8 - best - 1])
				best = q;
		uint32_t st_t[16], st_j[16];
		int sp = 0;
		st_t[sp] = ek.y;
		st_j[sp++] = (uint32_t)(8 - best);
		st_t[sp] = ek.x;
		st_j[sp++] = (uint32_t)best;
		while (sp > 0 && n < 8) {
			const uint32_t x = st_t[--sp];
			int j = (int)st_j[sp];
			if (x >= T.nnodes) {
				kid[n] = x;
				knode[n++] = false;
				continue;
			}
			for (;;) {
				const int8_t p = T.pick[8 * (size_t)x + j - 1];
				if (p < 0) {
					kid[n] = x;
					knode[n++] = true;
					break;
				}
				if (p == 0) {
					j--;
					continue;
				}
				const uint2 xk = T.ekids[x];
				st_t[sp] = xk.y;
				st_j[sp++] = (uint32_t)(j - p);
				st_t[sp] = xk.x;
				st_j[sp++] = (uint32_t)p;
				break;
			}
		}
	}
	/* slots by centroid octant about the node centre (Builder::assign_slots) */
	float clo[8][3], chi[8][3];
	float lo[3] = { FLT_MAX, FLT_MAX, FLT_MAX }, hi[3] = { -FLT_MAX, -FLT_MAX, -FLT_MAX };
	for (uint32_t i = 0; i < n; i++)
		for (int a = 0; a < 3; a++) {
			clo[i][a] = T.box[6 * (size_t)kid[i] + a];
			chi[i][a] = T.box[6 * (size_t)kid[i] + 3 + a];
			lo[a] = fminf(lo[a], clo[i][a]);
			hi[a] = fmaxf(hi[a], chi[i][a]);
		}
	float score[8][8];
	for (uint32_t i = 0; i < n; i++) {
		float off[3];
		for (int a = 0; a < 3; a++) {
			const float ext = fmaxf(hi[a] - lo[a], 1e-30f);
			off[a] = (0.5f * (clo[i][a] + chi[i][a]) - 0.5f * (lo[a] + hi[a])) / ext;
		}
		for (int s = 0; s < 8; s++)
			score[i][s] = ((s & 1) ? off[0] : -off[0]) + ((s & 2) ? off[1] : -off[1]) + ((s & 4) ? off[2] : -off[2]);
	}
	int slot_of[8];
	uint32_t kid_done = 0, slot_used = 0;
	for (uint32_t r = 0; r < n; r++) {
		int bi = -1, bs = -1;
		float bv = -FLT_MAX;
		for (uint32_t i = 0; i < n; i++) {
			if ((kid_done >> i) & 1u)
				continue;
			for (int s = 0; s < 8; s++)
				if (!((slot_used >> s) & 1u) && (bi < 0 || score[i][s] > bv)) {
					bv = score[i][s];
					bi = (int)i;
					bs = s;
				}
		}
		kid_done |= 1u << bi;
		slot_used |= 1u << bs;
		slot_of[bi] = bs;
	}
	/* the entry (Builder::emit) */
	uint32_t q16[8][3], org[3], ex[3];
	for (int a = 0; a < 3; a++) {
		uint32_t mn = 0xFFFFu, mx = 0;
		for (uint32_t i = 0; i < n; i++) {
			q16[i][a] = rtx_quantise(clo[i][a], chi[i][a], qo[a], qs[a]);
			mn = min(mn, q16[i][a] & 0xFFFFu);
			mx = max(mx, q16[i][a] >> 16);
		}
		org[a] = mn;
		uint32_t e = 0;
		while (((mx - mn) + (1u << e) - 1) >> e > 255u)
			e++;
		ex[a] = e;
	}
	uint32_t lo8[3][2] = { { ~0u, ~0u }, { ~0u, ~0u }, { ~0u, ~0u } }, hi8[3][2] = {};
	uint32_t imask = 0, vmask = 0, tmask = 0;
	for (uint32_t s = 0; s < 8; s++)
		leafmap[base + s] = RTX_NONE;
	uint32_t inner = 0;
	for (uint32_t i = 0; i < n; i++) {
		const uint32_t s = (uint32_t)slot_of[i];
		for (int a = 0; a < 3; a++) {
			const uint32_t q8 = rtx_quantise8(q16[i][a], org[a], ex[a]);
			const uint32_t sh = 8 * (s & 3);
			lo8[a][s >> 2] = (lo8[a][s >> 2] & ~(0xFFu << sh)) | ((q8 & 0xFFu) << sh);
			hi8[a][s >> 2] = (hi8[a][s >> 2] & ~(0xFFu << sh)) | ((q8 >> 8) << sh);
		}
		vmask |= 1u << s;
		if (knode[i]) {
			imask |= 1u << s;
			inner++;
		} else {
			const uint32_t pr = kid[i] - T.nnodes;
			leafmap[base + s] = pr;
			if (__float_as_uint(((const DPrim *)(T.recs + kid[i]))->c[3]) & RTX_META_TRANSPARENT)
				tmask |= 1u << s;
		}
	}
	DW8 N;
	N.w[0] = org[0] | (org[1] << 16);
	N.w[1] = org[2] | (ex[0] << 16) | (ex[1] << 20) | (ex[2] << 24);
	N.w[2] = (base << 8) | imask;
	N.w[3] = vmask | (tmask << 8);
	for (int a = 0; a < 3; a++) {
		N.w[4 + 4 * a] = lo8[a][0];
		N.w[5 + 4 * a] = lo8[a][1];
		N.w[6 + 4 * a] = hi8[a][0];
		N.w[7 + 4 * a] = hi8[a][1];
	}
	out[me] = N;
	/* the inner children for the next level, in slot order */
	for (uint32_t s = 0; s < 8; s++)
		nxt[8 * k + s] = RTX_NONE;
	for (uint32_t i = 0; i < n; i++)
		if (knode[i])
			nxt[8 * k + (uint32_t)slot_of[i]] = kid[i];
	ncnt[k] = inner;
}

__global__ __launch_bounds__(W8D_T) void k_w8d_next(uint32_t m, uint32_t blk, const uint32_t *__restrict__ nxt,
						    const uint32_t *__restrict__ noff, uint2 *__restrict__ items)
{
	const uint32_t k = blockIdx.x * W8D_T + threadIdx.x;
	if (k >= m)
		return;
	uint32_t o = noff[k];
	for (uint32_t s = 0; s < 8; s++) {
		const uint32_t t = nxt[8 * k + s];
		if (t != RTX_NONE)
			items[o++] = make_uint2(t, blk + 8 * k + s);
	}
}

/* the scalar-path copies of the inner entries (rtx_device.h DW8S; planes as exact floats) */
__global__ __launch_bounds__(W8D_T) void k_w8d_scalar(uint32_t n, const DW8 *__restrict__ w8, const uint32_t *__restrict__ leafmap,
						      DW8S *__restrict__ w8s)
{
	const uint32_t i = blockIdx.x * W8D_T + threadIdx.x;
	if (i >= n)
		return;
	DW8S f;
	memset(&f, 0, sizeof(f));
	const DW8 nd = w8[i];
	if ((nd.w[3] & 0xFFu) && leafmap[i] == RTX_NONE) {
		for (int k = 0; k < 4; k++)
			f.w[k] = nd.w[k];
		f.org[0] = (float)(nd.w[0] & 0xFFFFu);
		f.org[1] = (float)(nd.w[0] >> 16);
		f.org[2] = (float)(nd.w[1] & 0xFFFFu);
		for (int k = 0; k < 6; k++)
			for (int ch = 0; ch < 8; ch++)
				f.q[ch][k] = (float)((nd.w[4 + 2 * k + (ch >> 2)] >> (8 * (ch & 3))) & 0xFFu);
	}
	w8s[i] = f;
}

/* the scalar-path copies for a tree collapsed on the host (uploaded w8 and leaf map) */
extern "C" hipError_t rtx_launch_w8_scalar(uint32_t n, const DW8 *w8, const uint32_t *leafmap, DW8S *w8s, hipStream_t st)
{
	if (!n)
		return hipSuccess;
	hipLaunchKernelGGL(k_w8d_scalar, dim3((n + W8D_T - 1) / W8D_T), dim3(W8D_T), 0, st, n, w8, leafmap, w8s);
	return hipGetLastError();
}

/* The device collapse of the BVH2 in `recs` (nnodes inner records, root record 0, then nb
 * single-primitive leaves' records) into *w8_out / *leafmap_out (device buffers of *entries_out
 * entries, the caller frees them) and the scalar copies *w8s_out.  skip_obj: bit set of the
 * objects left out (the emitters), num_objects bits.  qo / qs receive the tree's frame;
 * *depth_out = 0 when nothing is left or the tree exceeds RTX_W8_MAX_ENTRIES. */
extern "C" hipError_t rtx_w8_collapse_device(const DNode *recs, uint32_t nnodes, uint32_t nb, const uint32_t *skip_obj,
					     uint32_t num_objects, DW8 **w8_out, DW8S **w8s_out, uint32_t **leafmap_out,
					     uint32_t *entries_out, uint32_t *scalar_entries_out, uint32_t *depth_out,
					     uint32_t *wide_out, uint32_t *top_out, float qo[3], float qs[3], hipStream_t st)
{
	hipError_t e = hipSuccess;
	*w8_out = nullptr;
	*w8s_out = nullptr;
	*leafmap_out = nullptr;
	*entries_out = *depth_out = *wide_out = *top_out = 0;
	if (!nnodes || !nb)
		return hipErrorInvalidValue;
	const size_t nt = (size_t)nnodes + nb;
	W8Tree T;
	T.recs = recs;
	T.nnodes = nnodes;
	T.nb = nb;
	T.parent = T.state = T.eff = nullptr;
	T.box = T.cost = nullptr;
	T.ekids = nullptr;
	T.pick = nullptr;
	DW8 *w8 = nullptr, *w8f = nullptr;
	DW8S *w8s = nullptr;
	uint32_t *lm = nullptr, *lmf = nullptr, *nxt = nullptr, *ncnt = nullptr, *noff = nullptr, *hst = nullptr;
	uint32_t *hhist = nullptr, *dhist = nullptr, *ddepth = nullptr, *dorder = nullptr; /* the bottom-up pass's depth buckets */
	uint2 *items = nullptr, *items2 = nullptr;
	void *temp = nullptr;
	const size_t cap = 2 + 8 * (size_t)nnodes; /* entries: at most one wide node per inner record */
	size_t tb = 0;
#define TRY(x)                                  \
	do {                                    \
		if ((e = (x)) != hipSuccess)    \
			goto done;              \
	} while (0)
	TRY(hipMalloc(&T.parent, nt * 4));
	TRY(hipMalloc(&T.box, nt * 24));
	TRY(hipMalloc(&T.state, nt * 4));
	TRY(hipMalloc(&T.eff, nt * 4));
	TRY(hipMalloc(&T.ekids, (size_t)nnodes * 8));
	TRY(hipMalloc(&T.cost, nt * 32));
	TRY(hipMalloc(&T.pick, nt * 8));
	TRY(hipMalloc(&w8, cap * sizeof(DW8)));
	TRY(hipMalloc(&lm, cap * 4));
	TRY(hipMalloc(&nxt, 8 * (size_t)nnodes * 4));
	TRY(hipMalloc(&ncnt, (size_t)nnodes * 4));
	TRY(hipMalloc(&noff, (size_t)nnodes * 4));
	TRY(hipMalloc(&items, (size_t)nnodes * 8));
	TRY(hipMalloc(&items2, (size_t)nnodes * 8));
	TRY(hipHostMalloc(&hst, 16 * 4));
	TRY(hipHostMalloc(&hhist, (W8D_MAXDEPTH + 1) * 4));
	TRY(hipMalloc(&dhist, (W8D_MAXDEPTH + 1) * 4));
	TRY(hipMalloc(&ddepth, (size_t)nnodes * 4));
	TRY(hipMalloc(&dorder, (size_t)nnodes * 4));
	TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, ncnt, noff, (int)nnodes, st));
	TRY(hipMalloc(&temp, tb));
	hipLaunchKernelGGL(k_w8d_parent, dim3((nnodes + W8D_T - 1) / W8D_T), dim3(W8D_T), 0, st, T);
	TRY(hipGetLastError());
	hipLaunchKernelGGL(k_w8d_leaves, dim3((nb + W8D_T - 1) / W8D_T), dim3(W8D_T), 0, st, T, skip_obj, num_objects);
	TRY(hipMemsetAsync(dhist, 0, (W8D_MAXDEPTH + 1) * 4, st));
	hipLaunchKernelGGL(k_w8d_depth, dim3((nnodes + W8D_T - 1) / W8D_T), dim3(W8D_T), 0, st, T, ddepth, dhist);
	TRY(hipGetLastError());
	TRY(hipMemcpyAsync(hhist, dhist, (W8D_MAXDEPTH + 1) * 4, hipMemcpyDeviceToHost, st));
	TRY(hipStreamSynchronize(st));
	{
		if (hhist[W8D_MAXDEPTH]) { /* a BVH2 deeper than W8D_MAXDEPTH: no tree (the walks fall back) */
			e = hipSuccess;
			goto done;
		}
		uint32_t maxd = 0, acc = 0;
		std::vector<uint32_t> off(W8D_MAXDEPTH + 1, 0);
		for (uint32_t d = 0; d < W8D_MAXDEPTH; d++) {
			off[d] = acc;
			acc += hhist[d];
			if (hhist[d])
				maxd = d;
		}
		TRY(hipMemcpyAsync(dhist, off.data(), W8D_MAXDEPTH * 4, hipMemcpyHostToDevice, st));
		hipLaunchKernelGGL(k_w8d_bucket, dim3((nnodes + W8D_T - 1) / W8D_T), dim3(W8D_T), 0, st, nnodes, ddepth, dhist, dorder);
		TRY(hipGetLastError());
		for (uint32_t d = maxd + 1; d-- > 0;)
			if (hhist[d]) {
				hipLaunchKernelGGL(k_w8d_level, dim3((hhist[d] + W8D_T - 1) / W8D_T), dim3(W8D_T), 0, st, T, dorder + off[d],
						   hhist[d]);
				TRY(hipGetLastError());
			}
		TRY(hipStreamSynchronize(st)); /* off (host memory) stays alive until the copy has run */
	}
	/* the root: its effective node and box -> the frame (rtx_wide8_build's) */
	TRY(hipMemcpyAsync(&hst[0], T.eff, 4, hipMemcpyDeviceToHost, st));
	TRY(hipStreamSynchronize(st));
	{
		const uint32_t root = hst[0];
		if (root == RTX_NONE)
			goto done; /* nothing left: no tree (depth 0) */
		float rb[6];
		TRY(hipMemcpyAsync(rb, T.box + 6 * (size_t)root, 24, hipMemcpyDeviceToHost, st));
		TRY(hipStreamSynchronize(st));
		float ext_max = 0.f;
		for (int a = 0; a < 3; a++)
			ext_max = fmaxf(ext_max, rb[3 + a] - rb[a]);
		for (int a = 0; a < 3; a++) {
			qo[a] = rb[a];
			qs[a] = 65533.f / fmaxf(rb[3 + a] - rb[a], fmaxf(ext_max, 1.f) * 1e-6f);
		}
		TRY(hipMemsetAsync(w8, 0, 2 * sizeof(DW8), st));
		TRY(hipMemsetAsync(lm, 0xFF, 2 * 4, st));
		hst[1] = root;
		hst[2] = 0;
		TRY(hipMemcpyAsync(items, &hst[1], 8, hipMemcpyHostToDevice, st));
		uint32_t m = 1, blk = 2, depth = 0, wide = 0, top = 0;
		uint32_t last = 2; /* where the last level's children start: every node entry lies below it */
		while (m) {
			if (blk + 8 * (size_t)m > RTX_W8_MAX_ENTRIES || blk + 8 * (size_t)m > cap) {
				depth = 0;
				goto done;
			}
			const dim3 g((m + W8D_T - 1) / W8D_T);
			hipLaunchKernelGGL(k_w8d_emit, g, dim3(W8D_T), 0, st, T, m, items, blk, qo[0], qo[1], qo[2], qs[0], qs[1], qs[2], w8,
					   lm, nxt, ncnt);
			TRY(hipGetLastError());
			TRY(hipcub::DeviceScan::ExclusiveSum(temp, tb, ncnt, noff, (int)m, st));
			hipLaunchKernelGGL(k_w8d_next, g, dim3(W8D_T), 0, st, m, blk, nxt, noff, items2);
			TRY(hipGetLastError());
			TRY(hipMemcpyAsync(&hst[4], noff + (m - 1), 4, hipMemcpyDeviceToHost, st));
			TRY(hipMemcpyAsync(&hst[5], ncnt + (m - 1), 4, hipMemcpyDeviceToHost, st));
			TRY(hipStreamSynchronize(st));
			wide += m;
			depth++;
			last = blk;
			blk += 8 * m;
			if (depth == RTX_W8_TOP_LEVELS - 1) /* every entry of levels 0 .. RTX_W8_TOP_LEVELS-1 */
				top = blk;
			m = hst[4] + hst[5];
			uint2 *ti = items;
			items = items2;
			items2 = ti;
		}
		/* exact-size buffers */
		TRY(hipMalloc(&w8f, (size_t)blk * sizeof(DW8)));
		TRY(hipMalloc(&lmf, (size_t)blk * 4));
		/* the scalar copies only up to the last node entry: the deepest level's entries are leaves
		 * (children of the last level's nodes), never read through the scalar path */
		TRY(hipMalloc(&w8s, (size_t)last * sizeof(DW8S)));
		TRY(hipMemcpyAsync(w8f, w8, (size_t)blk * sizeof(DW8), hipMemcpyDeviceToDevice, st));
		TRY(hipMemcpyAsync(lmf, lm, (size_t)blk * 4, hipMemcpyDeviceToDevice, st));
		hipLaunchKernelGGL(k_w8d_scalar, dim3((last + W8D_T - 1) / W8D_T), dim3(W8D_T), 0, st, last, w8f, lmf, w8s);
		TRY(hipGetLastError());
		TRY(hipStreamSynchronize(st));
		*w8_out = w8f;
		*w8s_out = w8s;
		*leafmap_out = lmf;
		w8f = nullptr;
		w8s = nullptr;
		lmf = nullptr;
		*entries_out = blk;
		*scalar_entries_out = last;
		*top_out = std::min<uint32_t>(top ? top : blk, RTX_W8_TOP_MAX);
		*depth_out = depth;
		*wide_out = wide;
	}
done:
#undef TRY
	(void)hipFree(T.parent);
	(void)hipFree(T.box);
	(void)hipFree(T.state);
	(void)hipFree(T.eff);
	(void)hipFree(T.ekids);
	(void)hipFree(T.cost);
	(void)hipFree(T.pick);
	(void)hipFree(w8);
	(void)hipFree(lm);
	(void)hipFree(nxt);
	(void)hipFree(ncnt);
	(void)hipFree(noff);
	(void)hipFree(items);
	(void)hipFree(items2);
	(void)hipFree(temp);
	(void)hipFree(w8f);
	(void)hipFree(w8s);
	(void)hipFree(lmf);
	(void)hipHostFree(hst);
	(void)hipHostFree(hhist);
	(void)hipFree(dhist);
	(void)hipFree(ddepth);
	(void)hipFree(dorder);
	return e;
}

/* the code object of this file on the current device, loaded now (rtx_open) rather than at the
 * first launch inside an upload or a render */
extern "C" __attribute__((visibility("hidden"))) hipError_t rtx_load_wide8_dev(void)
{
	hipFuncAttributes a;
	return hipFuncGetAttributes(&a, (const void *)k_w8d_parent);
}
