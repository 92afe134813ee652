/*
 * GPU BVH build (replacing accel_init accel.c:266-315 on the device):
 * a linear BVH in the reference's own spirit (Morton codes of leaf-box centroids, sorted,
 * Karras-split hierarchy: accel.c:83-88, 183-264), built in parallel and emitted straight
 * into the device record layout the kernels traverse (rtx_device.h):
 *
 *   k_lb_morton   63-bit Morton code (21 bits/axis) of each padded leaf box's centroid,
 *                 normalised by the scene extents; value = primitive index
 *   radix sort    rocPRIM via hipCUB (64-bit keys)
 *   k_lb_karras   Karras 2012 "Maximizing parallelism in the construction of BVHs":
 *                 one thread per internal node finds its key range and split from the
 *                 longest-common-prefix function (ties broken by index, as the
 *                 reference's equal-code median split does)
 *   k_lb_refit    bottom-up boxes: each leaf climbs, the second child to arrive at a node
 *                 unions both boxes and continues (atomic arrival counters)
 *   k_lb_keep     internal nodes kept as device nodes: the root and every node covering
 *                 more than max_leaf primitives; smaller subtrees become one leaf of their
 *                 contiguous primitive range; prefix sum -> record index
 *   k_lb_depth    kept-node depth of every leaf (the shadow walk's VGPR stack bound)
 *   k_lb_emit     DNode records (child boxes, byte-offset refs, per-octant child order)
 *                 and the primitives gathered into leaf order after them
 * The host binned-SAH builder (bvh_build.cpp) stays the default: it gives the tracer fewer
 * node visits; this builder trades some of that for build time.
 */
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <float.h>
#include <stdint.h>

#include "rtx.h"
#include "rtx_device.h"

#define LB_LEAF 0x80000000u /* child encoding during the build: LB_LEAF | sorted primitive index */

__device__ __forceinline__ uint64_t spread21(uint64_t v)
{
	v &= 0x1FFFFFull;
	v = (v | (v << 32)) & 0x1F00000000FFFFull;
	v = (v | (v << 16)) & 0x1F0000FF0000FFull;
	v = (v | (v << 8)) & 0x100F00F00F00F00Full;
	v = (v | (v << 4)) & 0x10C30C30C30C30C3ull;
	v = (v | (v << 2)) & 0x1249249249249249ull;
	return v;
}

__global__ __launch_bounds__(256) void k_lb_morton(uint32_t n, const float *__restrict__ lo, const float *__restrict__ hi,
						    float bx, float by, float bz, float sx, float sy, float sz,
						    uint64_t *__restrict__ keys, uint32_t *__restrict__ vals)
{
	const uint32_t i = blockIdx.x * 256u + threadIdx.x;
	if (i >= n)
		return;
	const float c[3] = { 0.5f * (lo[3 * i] + hi[3 * i]), 0.5f * (lo[3 * i + 1] + hi[3 * i + 1]),
			     0.5f * (lo[3 * i + 2] + hi[3 * i + 2]) };
	const float b[3] = { bx, by, bz }, s[3] = { sx, sy, sz };
	uint64_t q[3];
	for (int a = 0; a < 3; a++)
		q[a] = (uint64_t)fminf(fmaxf((c[a] - b[a]) * s[a], 0.f), 2097151.f);
	keys[i] = spread21(q[0]) << 2 | spread21(q[1]) << 1 | spread21(q[2]);
	vals[i] = i;
}

/* longest common prefix of sorted keys i and j (-1 outside [0, n)) */
__device__ __forceinline__ int lcp(const uint64_t *k, int n, int i, int j)
{
	if (j < 0 || j >= n)
		return -1;
	const uint64_t x = k[i] ^ k[j];
	return x ? __clzll((long long)x) : 64 + __clz(i ^ j);
}

/* internal node i: children (LB_LEAF | prim or internal index), range, parents */
__global__ __launch_bounds__(256) void k_lb_karras(int n, const uint64_t *__restrict__ k, uint32_t *__restrict__ child,
						    uint2 *__restrict__ range, uint32_t *__restrict__ parent_int,
						    uint32_t *__restrict__ parent_leaf)
{
	const int i = (int)(blockIdx.x * 256u + threadIdx.x);
	if (i >= n - 1)
		return;
	const int d = (lcp(k, n, i, i + 1) - lcp(k, n, i, i - 1)) >= 0 ? 1 : -1;
	const int dmin = lcp(k, n, i, i - d);
	int lmax = 2;
	while (lcp(k, n, i, i + lmax * d) > dmin)
		lmax <<= 1;
	int l = 0;
	for (int t = lmax >> 1; t >= 1; t >>= 1)
		if (lcp(k, n, i, i + (l + t) * d) > dmin)
			l += t;
	const int j = i + l * d;
	const int dnode = lcp(k, n, i, j);
	int s = 0;
	for (int t = (l + 1) >> 1;; t = (t + 1) >> 1) {
		if (lcp(k, n, i, i + (s + t) * d) > dnode)
			s += t;
		if (t == 1)
			break;
	}
	const int g = i + s * d + min(d, 0);
	const int first = min(i, j), last = max(i, j);
	const uint32_t left = (first == g) ? (LB_LEAF | (uint32_t)g) : (uint32_t)g;
	const uint32_t right = (last == g + 1) ? (LB_LEAF | (uint32_t)(g + 1)) : (uint32_t)(g + 1);
	child[2 * i] = left;
	child[2 * i + 1] = right;
	range[i] = make_uint2((uint32_t)first, (uint32_t)last);
	if (left & LB_LEAF)
		parent_leaf[left & ~LB_LEAF] = (uint32_t)i;
	else
		parent_int[left] = (uint32_t)i;
	if (right & LB_LEAF)
		parent_leaf[right & ~LB_LEAF] = (uint32_t)i;
	else
		parent_int[right] = (uint32_t)i;
}

__global__ __launch_bounds__(256) void k_lb_refit(int n, const uint32_t *__restrict__ perm, const float *__restrict__ lo,
						   const float *__restrict__ hi, const uint32_t *__restrict__ child,
						   const uint32_t *__restrict__ parent_int, const uint32_t *__restrict__ parent_leaf,
						   unsigned *__restrict__ arrive, float *__restrict__ nbox)
{
	const int k = (int)(blockIdx.x * 256u + threadIdx.x);
	if (k >= n)
		return;
	uint32_t node = parent_leaf[k];
	for (;;) {
		__threadfence();
		if (atomicAdd(&arrive[node], 1u) == 0)
			return; /* the sibling's thread finishes this node */
		__threadfence();
		float b[6] = { FLT_MAX, FLT_MAX, FLT_MAX, -FLT_MAX, -FLT_MAX, -FLT_MAX };
		for (int c = 0; c < 2; c++) {
			const uint32_t ch = child[2 * node + c];
			float cb[6];
			if (ch & LB_LEAF) {
				const uint32_t p = perm[ch & ~LB_LEAF];
				for (int a = 0; a < 3; a++) {
					cb[a] = lo[3 * p + a];
					cb[3 + a] = hi[3 * p + a];
				}
			} else {
				for (int a = 0; a < 6; a++) /* written by another thread: bypass stale L1 */
					cb[a] = __hip_atomic_load(&nbox[6 * ch + a], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
			}
			for (int a = 0; a < 3; a++) {
				b[a] = fminf(b[a], cb[a]);
				b[3 + a] = fmaxf(b[3 + a], cb[3 + a]);
			}
		}
		for (int a = 0; a < 6; a++)
			__hip_atomic_store(&nbox[6 * node + a], b[a], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		if (node == 0)
			return;
		node = parent_int[node];
	}
}

__global__ __launch_bounds__(256) void k_lb_keep(int n, uint32_t max_leaf, const uint2 *__restrict__ range,
						  uint32_t *__restrict__ keep)
{
	const int i = (int)(blockIdx.x * 256u + threadIdx.x);
	if (i >= n - 1)
		return;
	keep[i] = (i == 0 || range[i].y - range[i].x + 1 > max_leaf) ? 1u : 0u;
}

/* kept internal nodes on the path from each primitive to the root */
__global__ __launch_bounds__(256) void k_lb_depth(int n, const uint32_t *__restrict__ keep,
						   const uint32_t *__restrict__ parent_int,
						   const uint32_t *__restrict__ parent_leaf, unsigned *__restrict__ depth)
{
	const int k = (int)(blockIdx.x * 256u + threadIdx.x);
	if (k >= n)
		return;
	uint32_t node = parent_leaf[k];
	unsigned dd = 0;
	for (int guard = 0; guard < 4096; guard++) {
		dd += keep[node];
		if (node == 0)
			break;
		node = parent_int[node];
	}
	atomicMax(depth, dd);
}

__device__ __forceinline__ uint32_t leaf_ref(uint32_t nnodes, uint32_t first, uint32_t cnt,
					     const uint32_t *__restrict__ perm, const DPrim *__restrict__ prims_in)
{
	uint32_t sph = 0;
	for (uint32_t q = first; q < first + cnt; q++)
		if ((__float_as_uint(prims_in[perm[q]].c[3]) >> 24) == RTX_SPHERE)
			sph = RTX_REF_SPH;
	return (nnodes + first) * (uint32_t)sizeof(DNode) | RTX_REF_LEAF | sph | (cnt - 1);
}

/* a BVH2 inner record from its children's boxes (lo xyz, hi xyz) and refs, with the per-octant
 * child order of bvh_build.cpp (split axis = largest centroid separation) */
__device__ DNode make_dnode(const float (&box)[2][6], const uint32_t (&ref)[2])
{
	DNode d;
	float *f = &d.lo0x;
	for (int c = 0; c < 2; c++)
		for (int a = 0; a < 3; a++) {
			f[6 * c + 2 * a] = box[c][a];
			f[6 * c + 2 * a + 1] = box[c][3 + a];
		}
	d.ref0 = ref[0];
	d.ref1 = ref[1];
	int ax = 0;
	float best = -1.f;
	for (int a = 0; a < 3; a++) {
		const float sep = fabsf((box[0][a] + box[0][3 + a]) - (box[1][a] + box[1][3 + a]));
		if (sep > best) {
			best = sep;
			ax = a;
		}
	}
	const bool lcg = (box[0][ax] + box[0][3 + ax]) > (box[1][ax] + box[1][3 + ax]);
	d.order = 0;
	for (uint32_t o = 0; o < 8; o++)
		d.order |= ((((o >> ax) & 1u) != 0) != lcg) ? 1u << o : 0u;
	d.pad = 0;
	return d;
}

__global__ __launch_bounds__(256) void k_lb_emit(int n_int, int n, uint32_t nnodes, const uint32_t *__restrict__ keep,
						  const uint32_t *__restrict__ idx, const uint32_t *__restrict__ child,
						  const uint2 *__restrict__ range, const float *__restrict__ nbox,
						  const uint32_t *__restrict__ perm, const float *__restrict__ lo,
						  const float *__restrict__ hi, const DPrim *__restrict__ prims_in,
						  DNode *__restrict__ recs)
{
	const int i = (int)(blockIdx.x * 256u + threadIdx.x);
	if (i < n_int && keep[i]) {
		float box[2][6];
		uint32_t ref[2];
		for (int c = 0; c < 2; c++) {
			const uint32_t ch = child[2 * i + c];
			if (ch & LB_LEAF) {
				const uint32_t q = ch & ~LB_LEAF, p = perm[q];
				for (int a = 0; a < 3; a++) {
					box[c][a] = lo[3 * p + a];
					box[c][3 + a] = hi[3 * p + a];
				}
				ref[c] = leaf_ref(nnodes, q, 1, perm, prims_in);
			} else {
				for (int a = 0; a < 6; a++)
					box[c][a] = nbox[6 * ch + a];
				ref[c] = keep[ch] ? idx[ch] * (uint32_t)sizeof(DNode)
						  : leaf_ref(nnodes, range[ch].x, range[ch].y - range[ch].x + 1, perm, prims_in);
			}
		}
		recs[idx[i]] = make_dnode(box, ref);
	}
	if (i < n) /* primitives in leaf order after the nodes */
		recs[nnodes + i] = *(const DNode *)&prims_in[perm[i]];
}

extern "C" hipError_t rtx_lbvh_build(uint32_t n, const float *d_lo, const float *d_hi, const DPrim *d_prims_in,
				     const float blo[3], const float bhi[3], uint32_t max_leaf, DNode **recs_out,
				     uint32_t *nnodes_out, uint32_t *root_out, uint32_t *depth_out, hipStream_t st)
{
	hipError_t e = hipSuccess;
	*recs_out = nullptr;
	*nnodes_out = 0;
	*depth_out = 0;
	void *temp = nullptr;
	uint64_t *keys = nullptr;
	uint32_t *vals = nullptr, *child = nullptr, *pint = nullptr, *pleaf = nullptr, *keep = nullptr, *idx = nullptr;
	uint2 *range = nullptr;
	unsigned *arrive = nullptr, *scal = nullptr;
	float *nbox = nullptr;
	const int ni = (int)n - 1 > 0 ? (int)n - 1 : 1;
#define TRY(x)                                  \
	do {                                    \
		if ((e = (x)) != hipSuccess)    \
			goto done;              \
	} while (0)
	TRY(hipMalloc(&keys, 2 * (size_t)n * sizeof(uint64_t)));
	TRY(hipMalloc(&vals, 2 * (size_t)n * sizeof(uint32_t)));
	TRY(hipMalloc(&child, 2 * (size_t)ni * sizeof(uint32_t)));
	TRY(hipMalloc(&range, (size_t)ni * sizeof(uint2)));
	TRY(hipMalloc(&pint, (size_t)ni * sizeof(uint32_t)));
	TRY(hipMalloc(&pleaf, (size_t)n * sizeof(uint32_t)));
	TRY(hipMalloc(&arrive, (size_t)ni * sizeof(unsigned)));
	TRY(hipMalloc(&nbox, 6 * (size_t)ni * sizeof(float)));
	TRY(hipMalloc(&keep, (size_t)ni * sizeof(uint32_t)));
	TRY(hipMalloc(&idx, ((size_t)ni + 1) * sizeof(uint32_t)));
	TRY(hipMalloc(&scal, 4 * sizeof(unsigned)));
	{
		float s[3];
		for (int a = 0; a < 3; a++) {
			const float ext = bhi[a] - blo[a];
			s[a] = ext > 0.f ? 2097151.f / ext : 0.f;
		}
		const dim3 gn((n + 255) / 256), gi((ni + 255) / 256);
		hipLaunchKernelGGL(k_lb_morton, gn, dim3(256), 0, st, n, d_lo, d_hi, blo[0], blo[1], blo[2], s[0], s[1], s[2],
				   keys, vals);
		TRY(hipGetLastError());
		hipcub::DoubleBuffer<uint64_t> kb(keys, keys + n);
		hipcub::DoubleBuffer<uint32_t> vb(vals, vals + n);
		size_t tb = 0;
		TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, kb, vb, (int)n, 0, 63, st));
		TRY(hipMalloc(&temp, tb));
		TRY(hipcub::DeviceRadixSort::SortPairs(temp, tb, kb, vb, (int)n, 0, 63, st));
		const uint64_t *sk = kb.Current();
		const uint32_t *perm = vb.Current();
		uint32_t nnodes = 0, root = 0, depth = 0;
		if (n > max_leaf) {
			hipLaunchKernelGGL(k_lb_karras, gi, dim3(256), 0, st, (int)n, sk, child, range, pint, pleaf);
			TRY(hipGetLastError());
			TRY(hipMemsetAsync(arrive, 0, (size_t)ni * sizeof(unsigned), st));
			hipLaunchKernelGGL(k_lb_refit, gn, dim3(256), 0, st, (int)n, perm, d_lo, d_hi, child, pint, pleaf, arrive,
					   nbox);
			hipLaunchKernelGGL(k_lb_keep, gi, dim3(256), 0, st, (int)n, max_leaf, range, keep);
			TRY(hipGetLastError());
			size_t tb2 = 0;
			TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tb2, keep, idx, ni, st));
			void *temp2 = nullptr;
			TRY(hipMalloc(&temp2, tb2));
			e = hipcub::DeviceScan::ExclusiveSum(temp2, tb2, keep, idx, ni, st);
			(void)hipFreeAsync(temp2, st);
			TRY(e);
			TRY(hipMemsetAsync(scal, 0, 4 * sizeof(unsigned), st));
			hipLaunchKernelGGL(k_lb_depth, gn, dim3(256), 0, st, (int)n, keep, pint, pleaf, scal);
			TRY(hipGetLastError());
			uint32_t last[2];
			TRY(hipMemcpyAsync(&last[0], idx + (ni - 1), 4, hipMemcpyDeviceToHost, st));
			TRY(hipMemcpyAsync(&last[1], keep + (ni - 1), 4, hipMemcpyDeviceToHost, st));
			TRY(hipMemcpyAsync(&depth, scal, 4, hipMemcpyDeviceToHost, st));
			TRY(hipStreamSynchronize(st));
			nnodes = last[0] + last[1];
			root = 0;
		} else {
			root = RTX_EMPTY_REF;
		}
		DNode *recs = nullptr;
		TRY(hipMalloc(&recs, ((size_t)nnodes + n) * sizeof(DNode)));
		/* n <= max_leaf: no internal nodes, the caller makes the root one leaf of all primitives */
		hipLaunchKernelGGL(k_lb_emit, gn, dim3(256), 0, st, n > max_leaf ? (int)n - 1 : 0, (int)n, nnodes, keep, idx,
				   child, range, nbox, perm, d_lo, d_hi, d_prims_in, recs);
		e = hipGetLastError();
		if (e == hipSuccess)
			e = hipStreamSynchronize(st);
		if (e != hipSuccess) {
			(void)hipFree(recs);
			goto done;
		}
		*recs_out = recs;
		*nnodes_out = nnodes;
		*root_out = root;
		*depth_out = depth;
	}
done:
#undef TRY
	(void)hipFree(temp);
	(void)hipFree(keys);
	(void)hipFree(vals);
	(void)hipFree(child);
	(void)hipFree(range);
	(void)hipFree(pint);
	(void)hipFree(pleaf);
	(void)hipFree(arrive);
	(void)hipFree(nbox);
	(void)hipFree(keep);
	(void)hipFree(idx);
	(void)hipFree(scal);
	return e;
}

/* ------------------------------------------------------------------------ */
/* PLOC: parallel locally-ordered clustering (Meister and Bittner 2018)      */
/* ------------------------------------------------------------------------ */
/* The clusters start as the primitives in Morton order.  Each round every cluster finds its
 * nearest neighbour among the RTX_PLOC_R clusters either side (distance: surface area of the
 * union box; ties to the lower pair index, so the order is total and the closest pair is always
 * mutual), mutual pairs merge into a new inner node at the lower one's position and the list is
 * compacted.  Tree node ids: 0..n-1 the primitives (sorted position), n.. the inner nodes in
 * creation order.  The records are then laid out depth-first like the host builder's. */
#ifndef RTX_PLOC_R
#define RTX_PLOC_R 16 /* search radius (clusters either side) */
#endif
#define PLOC_T 256

__device__ __forceinline__ float box_area6(const float *b)
{
	const float dx = b[3] - b[0], dy = b[4] - b[1], dz = b[5] - b[2];
	return dx * dy + dy * dz + dz * dx;
}

/* leaf nodes: boxes in sorted order, counts; clusters = the leaves */
__global__ __launch_bounds__(PLOC_T) void k_pl_init(uint32_t n, const uint32_t *__restrict__ perm, const float *__restrict__ lo,
						    const float *__restrict__ hi, float *__restrict__ nb6, uint32_t *__restrict__ cnt,
						    uint32_t *__restrict__ kcnt, uint32_t *__restrict__ cl, float *__restrict__ cb)
{
	const uint32_t q = blockIdx.x * PLOC_T + threadIdx.x;
	if (q >= n)
		return;
	const uint32_t p = perm[q];
	for (int a = 0; a < 3; a++) {
		nb6[6 * q + a] = cb[6 * q + a] = lo[3 * p + a];
		nb6[6 * q + 3 + a] = cb[6 * q + 3 + a] = hi[3 * p + a];
	}
	cnt[q] = 1;
	kcnt[q] = 0;
	cl[q] = q;
}

/* nearest neighbour of each cluster within the radius (boxes staged through LDS) */
__global__ __launch_bounds__(PLOC_T) void k_pl_nn(uint32_t m, const float *__restrict__ cb, uint32_t *__restrict__ nn)
{
	__shared__ float sb[PLOC_T + 2 * RTX_PLOC_R][6];
	const int b0 = (int)(blockIdx.x * PLOC_T) - RTX_PLOC_R;
	for (int k = threadIdx.x; k < PLOC_T + 2 * RTX_PLOC_R; k += PLOC_T) {
		const int j = b0 + k;
		for (int a = 0; a < 6; a++)
			sb[k][a] = (j >= 0 && j < (int)m) ? cb[6 * j + a] : 0.f;
	}
	__syncthreads();
	const int i = (int)(blockIdx.x * PLOC_T + threadIdx.x);
	if (i >= (int)m)
		return;
	const int li = i - b0;
	float bd = FLT_MAX;
	int bj = -1;
	for (int o = -RTX_PLOC_R; o <= RTX_PLOC_R; o++) {
		const int j = i + o;
		if (o == 0 || j < 0 || j >= (int)m)
			continue;
		float u[6];
		for (int a = 0; a < 3; a++) {
			u[a] = fminf(sb[li][a], sb[li + o][a]);
			u[3 + a] = fmaxf(sb[li][3 + a], sb[li + o][3 + a]);
		}
		const float d = box_area6(u);
		/* pair order (d, lower index, higher index): for a fixed i the lower index decides ties
		 * among j < i by j, and any j < i before any j > i */
		if (d < bd || (d == bd && j < bj)) {
			bd = d;
			bj = j;
		}
	}
	nn[i] = (uint32_t)bj;
}

/* merge / keep flags: merges count in the high word, surviving list entries in the low word */
__global__ __launch_bounds__(PLOC_T) void k_pl_flags(uint32_t m, const uint32_t *__restrict__ nn, uint64_t *__restrict__ fl)
{
	const uint32_t i = blockIdx.x * PLOC_T + threadIdx.x;
	if (i >= m)
		return;
	const uint32_t j = nn[i];
	const bool mutual = j < m && nn[j] == i;
	const bool merge = mutual && i < j, gone = mutual && i > j;
	fl[i] = ((uint64_t)(merge ? 1u : 0u) << 32) | (gone ? 0u : 1u);
}

__global__ __launch_bounds__(PLOC_T) void k_pl_apply(uint32_t m, uint32_t n, uint32_t next_id, uint32_t max_leaf,
						     const uint32_t *__restrict__ nn, const uint64_t *__restrict__ fl,
						     const uint64_t *__restrict__ pre, const uint32_t *__restrict__ cl,
						     const float *__restrict__ cb, uint32_t *__restrict__ cl2, float *__restrict__ cb2,
						     float *__restrict__ nb6, uint2 *__restrict__ kids, uint32_t *__restrict__ par,
						     uint32_t *__restrict__ cnt, uint32_t *__restrict__ kcnt)
{
	const uint32_t i = blockIdx.x * PLOC_T + threadIdx.x;
	if (i >= m || !(fl[i] & 1u))
		return;
	const uint32_t pos = (uint32_t)pre[i];
	if (!(fl[i] >> 32)) { /* unmerged: carried over */
		cl2[pos] = cl[i];
		for (int a = 0; a < 6; a++)
			cb2[6 * pos + a] = cb[6 * i + a];
		return;
	}
	const uint32_t j = nn[i], id = next_id + (uint32_t)(pre[i] >> 32);
	const uint32_t a_ = cl[i], b_ = cl[j];
	float u[6];
	for (int a = 0; a < 3; a++) {
		u[a] = fminf(cb[6 * i + a], cb[6 * j + a]);
		u[3 + a] = fmaxf(cb[6 * i + 3 + a], cb[6 * j + 3 + a]);
	}
	for (int a = 0; a < 6; a++) {
		nb6[6 * (size_t)id + a] = u[a];
		cb2[6 * pos + a] = u[a];
	}
	cl2[pos] = id;
	kids[id - n] = make_uint2(a_, b_);
	par[a_] = id;
	par[b_] = id;
	const uint32_t c = cnt[a_] + cnt[b_];
	cnt[id] = c;
	kcnt[id] = (c > max_leaf ? 1u : 0u) + kcnt[a_] + kcnt[b_];
}

/* depth-first position of node v among the kept inner nodes (KEPT) or of its first primitive in
 * leaf order (!KEPT): parent first, then the left subtree, then the right one */
template <bool KEPT>
__device__ __forceinline__ uint32_t pl_pos(uint32_t v, uint32_t root, const uint2 *__restrict__ kids,
					   const uint32_t *__restrict__ par, const uint32_t *__restrict__ cnt,
					   const uint32_t *__restrict__ kcnt, uint32_t n)
{
	uint32_t x = v, pos = 0;
	for (int guard = 0; x != root && guard < (1 << 20); guard++) {
		const uint32_t p = par[x];
		const uint2 k = kids[p - n];
		if (KEPT)
			pos += 1;
		if (x == k.y)
			pos += KEPT ? kcnt[k.x] : cnt[k.x];
		x = p;
	}
	return pos;
}

/* each primitive's position in leaf order (and the depth of kept nodes above it) */
__global__ __launch_bounds__(PLOC_T) void k_pl_leafpos(uint32_t n, uint32_t root, uint32_t max_leaf,
						       const uint32_t *__restrict__ perm, const uint2 *__restrict__ kids,
						       const uint32_t *__restrict__ par, const uint32_t *__restrict__ cnt,
						       const uint32_t *__restrict__ kcnt, uint32_t *__restrict__ posmap,
						       unsigned *__restrict__ depth)
{
	const uint32_t q = blockIdx.x * PLOC_T + threadIdx.x;
	if (q >= n)
		return;
	posmap[pl_pos<false>(q, root, kids, par, cnt, kcnt, n)] = perm[q];
	unsigned dd = 0;
	uint32_t x = q;
	for (int guard = 0; x != root && guard < (1 << 20); guard++) {
		x = par[x];
		dd += (x == root || cnt[x] > max_leaf) ? 1u : 0u;
	}
	atomicMax(depth, dd);
}

__global__ __launch_bounds__(PLOC_T) void k_pl_emit(uint32_t n, uint32_t n_int, uint32_t root, uint32_t max_leaf, uint32_t nnodes,
						    const uint2 *__restrict__ kids, const uint32_t *__restrict__ par,
						    const uint32_t *__restrict__ cnt, const uint32_t *__restrict__ kcnt,
						    const float *__restrict__ nb6, const uint32_t *__restrict__ posmap,
						    const DPrim *__restrict__ prims_in, DNode *__restrict__ recs)
{
	const uint32_t i = blockIdx.x * PLOC_T + threadIdx.x;
	if (i < n_int) {
		const uint32_t v = n + i;
		if (v == root || cnt[v] > max_leaf) {
			const uint2 k = kids[i];
			float box[2][6];
			uint32_t ref[2];
			for (int c = 0; c < 2; c++) {
				const uint32_t ch = c ? k.y : k.x;
				for (int a = 0; a < 6; a++)
					box[c][a] = nb6[6 * (size_t)ch + a];
				if (ch >= n && cnt[ch] > max_leaf) {
					ref[c] = pl_pos<true>(ch, root, kids, par, cnt, kcnt, n) * (uint32_t)sizeof(DNode);
				} else {
					const uint32_t first = pl_pos<false>(ch, root, kids, par, cnt, kcnt, n), m = cnt[ch];
					uint32_t sph = 0;
					for (uint32_t q = first; q < first + m; q++)
						if ((__float_as_uint(prims_in[posmap[q]].c[3]) >> 24) == RTX_SPHERE)
							sph = RTX_REF_SPH;
					ref[c] = (nnodes + first) * (uint32_t)sizeof(DNode) | RTX_REF_LEAF | sph | (m - 1);
				}
			}
			recs[pl_pos<true>(v, root, kids, par, cnt, kcnt, n)] = make_dnode(box, ref);
		}
	}
	if (i < n) /* primitives in leaf order after the nodes */
		recs[nnodes + i] = *(const DNode *)&prims_in[posmap[i]];
}

/* The PLOC build: same contract as rtx_lbvh_build (records = inner nodes depth-first, then the
 * primitives in leaf order; root record 0; n <= max_leaf leaves no inner node).  Each round
 * reads back its list length (a few dozen rounds). */
extern "C" hipError_t rtx_ploc_build(uint32_t n, const float *d_lo, const float *d_hi, const DPrim *d_prims_in,
				     const float blo[3], const float bhi[3], uint32_t max_leaf, DNode **recs_out,
				     uint32_t *nnodes_out, uint32_t *root_out, uint32_t *depth_out, uint32_t *rounds_out,
				     hipStream_t st)
{
	hipError_t e = hipSuccess;
	*recs_out = nullptr;
	*nnodes_out = 0;
	*depth_out = 0;
	*rounds_out = 0;
	void *temp = nullptr;
	uint64_t *keys = nullptr, *fl = nullptr, *pre = nullptr, *tail = nullptr;
	uint32_t *vals = nullptr, *cnt = nullptr, *kcnt = nullptr, *par = nullptr, *cl = nullptr, *cl2 = nullptr, *nn = nullptr,
		 *posmap = nullptr;
	float *nb6 = nullptr, *cb = nullptr, *cb2 = nullptr;
	uint2 *kids = nullptr;
	unsigned *scal = nullptr;
	const size_t nt = 2 * (size_t)n; /* tree nodes (2n - 1) */
#define TRY(x)                                  \
	do {                                    \
		if ((e = (x)) != hipSuccess)    \
			goto done;              \
	} while (0)
	TRY(hipMalloc(&keys, 2 * (size_t)n * sizeof(uint64_t)));
	TRY(hipMalloc(&vals, 2 * (size_t)n * sizeof(uint32_t)));
	TRY(hipMalloc(&nb6, 6 * nt * sizeof(float)));
	TRY(hipMalloc(&cnt, nt * sizeof(uint32_t)));
	TRY(hipMalloc(&kcnt, nt * sizeof(uint32_t)));
	TRY(hipMalloc(&par, nt * sizeof(uint32_t)));
	TRY(hipMalloc(&kids, (size_t)n * sizeof(uint2)));
	TRY(hipMalloc(&cl, (size_t)n * sizeof(uint32_t)));
	TRY(hipMalloc(&cl2, (size_t)n * sizeof(uint32_t)));
	TRY(hipMalloc(&cb, 6 * (size_t)n * sizeof(float)));
	TRY(hipMalloc(&cb2, 6 * (size_t)n * sizeof(float)));
	TRY(hipMalloc(&nn, (size_t)n * sizeof(uint32_t)));
	TRY(hipMalloc(&fl, (size_t)n * sizeof(uint64_t)));
	TRY(hipMalloc(&pre, (size_t)n * sizeof(uint64_t)));
	TRY(hipMalloc(&posmap, (size_t)n * sizeof(uint32_t)));
	TRY(hipHostMalloc(&tail, 2 * sizeof(uint64_t)));
	TRY(hipMalloc(&scal, 4 * sizeof(unsigned)));
	{
		float s[3];
		for (int a = 0; a < 3; a++) {
			const float ext = bhi[a] - blo[a];
			s[a] = ext > 0.f ? 2097151.f / ext : 0.f;
		}
		const dim3 gn((n + PLOC_T - 1) / PLOC_T);
		hipLaunchKernelGGL(k_lb_morton, gn, dim3(256), 0, st, n, d_lo, d_hi, blo[0], blo[1], blo[2], s[0], s[1], s[2],
				   keys, vals);
		TRY(hipGetLastError());
		hipcub::DoubleBuffer<uint64_t> kb(keys, keys + n);
		hipcub::DoubleBuffer<uint32_t> vb(vals, vals + n);
		size_t tb = 0, tb2 = 0;
		TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, kb, vb, (int)n, 0, 63, st));
		TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tb2, fl, pre, (int)n, st));
		TRY(hipMalloc(&temp, tb > tb2 ? tb : tb2));
		TRY(hipcub::DeviceRadixSort::SortPairs(temp, tb, kb, vb, (int)n, 0, 63, st));
		const uint32_t *perm = vb.Current();
		uint32_t nnodes = 0, root = 0, depth = 0;
		hipLaunchKernelGGL(k_pl_init, gn, dim3(PLOC_T), 0, st, n, perm, d_lo, d_hi, nb6, cnt, kcnt, cl, cb);
		TRY(hipGetLastError());
		uint32_t m = n, next_id = n, rounds = 0;
		while (m > 1) {
			if (++rounds > 4096) { /* a round always merges the closest pair: cannot happen */
				e = hipErrorUnknown;
				goto done;
			}
			const dim3 gm((m + PLOC_T - 1) / PLOC_T);
			hipLaunchKernelGGL(k_pl_nn, gm, dim3(PLOC_T), 0, st, m, cb, nn);
			hipLaunchKernelGGL(k_pl_flags, gm, dim3(PLOC_T), 0, st, m, nn, fl);
			TRY(hipGetLastError());
			TRY(hipcub::DeviceScan::ExclusiveSum(temp, tb2, fl, pre, (int)m, st));
			hipLaunchKernelGGL(k_pl_apply, gm, dim3(PLOC_T), 0, st, m, n, next_id, max_leaf, nn, fl, pre, cl, cb, cl2, cb2,
					   nb6, kids, par, cnt, kcnt);
			TRY(hipGetLastError());
			TRY(hipMemcpyAsync(&tail[0], pre + (m - 1), 8, hipMemcpyDeviceToHost, st));
			TRY(hipMemcpyAsync(&tail[1], fl + (m - 1), 8, hipMemcpyDeviceToHost, st));
			TRY(hipStreamSynchronize(st));
			const uint64_t tot = tail[0] + tail[1];
			if (!(tot >> 32)) {
				e = hipErrorUnknown;
				goto done;
			}
			next_id += (uint32_t)(tot >> 32);
			m = (uint32_t)tot;
			uint32_t *tc = cl;
			cl = cl2;
			cl2 = tc;
			float *tf = cb;
			cb = cb2;
			cb2 = tf;
		}
		*rounds_out = rounds;
		if (n > max_leaf) {
			root = next_id - 1; /* the last merge */
			TRY(hipMemcpyAsync(&nnodes, kcnt + root, 4, hipMemcpyDeviceToHost, st));
			TRY(hipStreamSynchronize(st));
		} else {
			nnodes = 0;
		}
		TRY(hipMemsetAsync(scal, 0, 4 * sizeof(unsigned), st));
		if (n > 1) {
			hipLaunchKernelGGL(k_pl_leafpos, gn, dim3(PLOC_T), 0, st, n, next_id - 1, max_leaf, perm, kids, par, cnt, kcnt,
					   posmap, scal);
		} else {
			TRY(hipMemcpyAsync(posmap, perm, 4, hipMemcpyDeviceToDevice, st));
		}
		TRY(hipGetLastError());
		DNode *recs = nullptr;
		TRY(hipMalloc(&recs, ((size_t)nnodes + n) * sizeof(DNode)));
		hipLaunchKernelGGL(k_pl_emit, gn, dim3(PLOC_T), 0, st, n, n > max_leaf ? n - 1 : 0u, next_id - 1, max_leaf, nnodes, kids, par, cnt, kcnt, nb6, posmap, d_prims_in, recs);
		e = hipGetLastError();
		if (e == hipSuccess)
			e = hipMemcpyAsync(&depth, scal, 4, hipMemcpyDeviceToHost, st);
		if (e == hipSuccess)
			e = hipStreamSynchronize(st);
		if (e != hipSuccess) {
			(void)hipFree(recs);
			goto done;
		}
		*recs_out = recs;
		*nnodes_out = nnodes;
		*root_out = n > max_leaf ? 0u : RTX_EMPTY_REF;
		*depth_out = n > max_leaf ? depth : 0u;
	}
done:
#undef TRY
	(void)hipFree(temp);
	(void)hipFree(keys);
	(void)hipFree(vals);
	(void)hipFree(nb6);
	(void)hipFree(cnt);
	(void)hipFree(kcnt);
	(void)hipFree(par);
	(void)hipFree(kids);
	(void)hipFree(cl);
	(void)hipFree(cl2);
	(void)hipFree(cb);
	(void)hipFree(cb2);
	(void)hipFree(nn);
	(void)hipFree(fl);
	(void)hipFree(pre);
	(void)hipFree(posmap);
	(void)hipHostFree(tail);
	(void)hipFree(scal);
	return e;
}

/* ------------------------------------------------------------------------ */
/* Binned SAH on the device: bvh_build.cpp's algorithm, level by level       */
/* ------------------------------------------------------------------------ */
/* Every level holds the active nodes (two or more primitives), each a contiguous range of the
 * position array.  Per level: node boxes and centroid bounds (atomic min / max on order-preserving
 * integer encodings of the floats, exact), the SAH bins of every axis (same bin rule, same float
 * arithmetic, so the same costs), one thread per node sweeping the bins in the host's order (axis
 * 0..2, split 0..NB-2, strict <), then a stable partition of each range by an exclusive scan of the
 * left flags.  Nodes the host would split at the centroid median (depth budget) or by index (all
 * centroids equal) split at the middle of the range.  For single-primitive leaves (the default)
 * the tree is the host builder's node for node: its records are byte-identical
 * (tests/test_gpu_build.py).  The tree then goes through the PLOC builder's depth-first emission
 * (ids 0..n-1 the final positions, n.. the inner nodes). */
#define SB_T 256
#define SB_NBMAX 64
/* the host's float arithmetic exactly: no contraction into FMAs (this file is built without
 * -ffp-contract=off) */
#pragma clang fp contract(off)
#define SB_ACC(NB) (12 + 3 * (NB) * 7) /* per node: box + centroid bounds, then per axis and bin 6 bounds + count */

__device__ __forceinline__ uint32_t f2o(float f) /* order-preserving encoding */
{
	const uint32_t b = __float_as_uint(f);
	return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float o2f(uint32_t o) { return __uint_as_float((o & 0x80000000u) ? (o & 0x7FFFFFFFu) : ~o); }

/* the host's Box::area */
__device__ __forceinline__ float sb_area(const float *lo, const float *hi)
{
	const float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
	if (dx < 0 || dy < 0 || dz < 0)
		return 0.f;
	return 2.f * (dx * dy + dy * dz + dz * dx);
}

struct SbNode {
	uint32_t b, e, id, depth;
};

/* accumulators of M nodes: mins at +FLT_MAX, maxes at -FLT_MAX, counts 0 */
__global__ __launch_bounds__(SB_T) void k_sb_reset(uint32_t M, uint32_t nb, uint32_t *__restrict__ acc)
{
	const uint32_t stride = SB_ACC(nb);
	const size_t i = (size_t)blockIdx.x * SB_T + threadIdx.x;
	if (i >= (size_t)M * stride)
		return;
	const uint32_t k = (uint32_t)(i % stride);
	uint32_t v;
	if (k < 12)
		v = (k % 6) < 3 ? f2o(FLT_MAX) : f2o(-FLT_MAX);
	else {
		const uint32_t j = (k - 12) % 7;
		v = j == 6 ? 0u : j < 3 ? f2o(FLT_MAX) : f2o(-FLT_MAX);
	}
	acc[i] = v;
}

/* the batch's node of position q (RTX_NONE: a leaf, or another batch's node) */
__device__ __forceinline__ uint32_t sb_node(uint32_t q, uint32_t n, uint32_t s0b, uint32_t sn, const uint32_t *__restrict__ seg)
{
	const uint32_t s = q < n ? seg[q] : RTX_NONE;
	return (s != RTX_NONE && s - s0b < sn) ? s - s0b : RTX_NONE;
}

/* the least and greatest batch node of the workgroup's positions (a node's positions are one
 * contiguous range, so every position between two of one node's is that node's); lo = RTX_NONE:
 * none */
__device__ __forceinline__ void sb_span(uint32_t s, uint32_t *sh, uint32_t &lo, uint32_t &hi)
{
	if (threadIdx.x == 0) {
		sh[0] = RTX_NONE;
		sh[1] = 0u;
	}
	__syncthreads();
	if (s != RTX_NONE) {
		atomicMin(&sh[0], s);
		atomicMax(&sh[1], s);
	}
	__syncthreads();
	lo = sh[0];
	hi = sh[1];
}

/* node boxes and centroid bounds.  A wave whose positions all lie in one node reduces first; a
 * workgroup whose positions all lie in one node reduces its waves in LDS and sends one set of
 * atomics (the top levels: every workgroup's positions in the root, or one of a few nodes). */
__global__ __launch_bounds__(SB_T) void k_sb_bounds(uint32_t n, uint32_t nb, uint32_t s0b, uint32_t sn,
						     const uint32_t *__restrict__ seg, const uint32_t *__restrict__ pidx,
						     const float *__restrict__ lo, const float *__restrict__ hi, uint32_t *__restrict__ acc)
{
	__shared__ uint32_t span[2], red[12];
	const uint32_t q = blockIdx.x * SB_T + threadIdx.x;
	const uint32_t s = sb_node(q, n, s0b, sn, seg);
	uint32_t smin, smax;
	sb_span(s, span, smin, smax);
	if (smin == RTX_NONE)
		return;
	float v[12];
	if (s != RTX_NONE) {
		const uint32_t p = pidx[q];
		for (int a = 0; a < 3; a++) {
			v[a] = lo[3 * (size_t)p + a];
			v[3 + a] = hi[3 * (size_t)p + a];
			v[6 + a] = v[9 + a] = 0.5f * (v[a] + v[3 + a]);
		}
	} else {
		for (int a = 0; a < 3; a++) {
			v[a] = v[6 + a] = FLT_MAX;
			v[3 + a] = v[9 + a] = -FLT_MAX;
		}
	}
	if (smin == smax) { /* one node: waves reduce, then the workgroup in LDS */
		if (threadIdx.x < 12)
			red[threadIdx.x] = (threadIdx.x % 6) < 3 ? f2o(FLT_MAX) : f2o(-FLT_MAX);
		for (int k = 0; k < 12; k++)
			for (int m = 32; m > 0; m >>= 1) {
				const float o = __shfl_xor(v[k], m);
				v[k] = ((k % 6) < 3) ? fminf(v[k], o) : fmaxf(v[k], o);
			}
		__syncthreads();
		if ((threadIdx.x & 63u) == 0)
			for (int k = 0; k < 12; k++)
				((k % 6) < 3) ? atomicMin(&red[k], f2o(v[k])) : atomicMax(&red[k], f2o(v[k]));
		__syncthreads();
		if (threadIdx.x < 12) {
			uint32_t *A = acc + (size_t)smin * SB_ACC(nb);
			const int k = (int)threadIdx.x;
			((k % 6) < 3) ? atomicMin(&A[k], red[k]) : atomicMax(&A[k], red[k]);
		}
		return;
	}
	const uint32_t s0 = __shfl(s, 0);
	if (__all(s == s0)) {
		if (s0 == RTX_NONE)
			return;
		for (int k = 0; k < 12; k++)
			for (int m = 32; m > 0; m >>= 1) {
				const float o = __shfl_xor(v[k], m);
				v[k] = ((k % 6) < 3) ? fminf(v[k], o) : fmaxf(v[k], o);
			}
		if ((threadIdx.x & 63u) == 0) {
			uint32_t *A = acc + (size_t)s0 * SB_ACC(nb);
			for (int k = 0; k < 12; k++)
				((k % 6) < 3) ? atomicMin(&A[k], f2o(v[k])) : atomicMax(&A[k], f2o(v[k]));
		}
		return;
	}
	if (s == RTX_NONE)
		return;
	uint32_t *A = acc + (size_t)s * SB_ACC(nb);
	for (int k = 0; k < 12; k++)
		((k % 6) < 3) ? atomicMin(&A[k], f2o(v[k])) : atomicMax(&A[k], f2o(v[k]));
}

/* the host's bin of a centroid coordinate */
__device__ __forceinline__ int sb_bin(float c, float clo, float k, int nb)
{
	int bi = (int)((c - clo) * k);
	return min(max(bi, 0), nb - 1);
}

/* the bins of a position's centroid, per axis: 6 bounds and a count.  A workgroup whose
 * positions lie in at most SB_LK nodes accumulates in LDS first and sends one atomic per bin
 * word it touched (the top levels: thousands of positions per bin word, which serialised on the
 * L2 atomics); otherwise every position sends its own.  Min / max of order-preserving encodings
 * and integer counts: the same result in any order. */
#define SB_LK 2
__device__ __forceinline__ uint32_t sb_ident(uint32_t k) /* bin word k's identity (k < 7 * 3 * nb) */
{
	const uint32_t j = k % 7;
	return j == 6 ? 0u : j < 3 ? f2o(FLT_MAX) : f2o(-FLT_MAX);
}
__global__ __launch_bounds__(SB_T) void k_sb_bins(uint32_t n, uint32_t nb, uint32_t s0b, uint32_t sn,
						   const uint32_t *__restrict__ seg, const uint32_t *__restrict__ pidx,
						   const float *__restrict__ lo, const float *__restrict__ hi, uint32_t *__restrict__ acc)
{
	__shared__ uint32_t span[2];
	__shared__ uint32_t L[SB_LK][3 * SB_NBMAX * 7];
	const uint32_t q = blockIdx.x * SB_T + threadIdx.x;
	const uint32_t s = sb_node(q, n, s0b, sn, seg);
	uint32_t smin, smax;
	sb_span(s, span, smin, smax);
	if (smin == RTX_NONE)
		return;
	const bool local = smax - smin < SB_LK;
	const uint32_t nw = 3 * nb * 7; /* bin words per node */
	if (local) {
		for (uint32_t i = threadIdx.x; i < SB_LK * nw; i += SB_T)
			L[i / nw][i % nw] = sb_ident(i % nw);
		__syncthreads();
	}
	if (s != RTX_NONE) {
		const uint32_t *A = acc + (size_t)s * SB_ACC(nb);
		uint32_t *D = local ? L[s - smin] : acc + (size_t)s * SB_ACC(nb) + 12;
		const uint32_t p = pidx[q];
		float b[6];
		for (int a = 0; a < 3; a++) {
			b[a] = lo[3 * (size_t)p + a];
			b[3 + a] = hi[3 * (size_t)p + a];
		}
		for (int ax = 0; ax < 3; ax++) {
			const float clo = o2f(A[6 + ax]), chi = o2f(A[9 + ax]), ext = chi - clo;
			if (!(ext > 0.f))
				continue;
			const float k = (float)nb * (1.f - 1e-6f) / ext;
			const int bi = sb_bin(0.5f * (b[ax] + b[3 + ax]), clo, k, (int)nb);
			uint32_t *B = D + ((size_t)ax * nb + bi) * 7;
			for (int a = 0; a < 3; a++) {
				atomicMin(&B[a], f2o(b[a]));
				atomicMax(&B[3 + a], f2o(b[3 + a]));
			}
			atomicAdd(&B[6], 1u);
		}
	}
	if (!local)
		return;
	__syncthreads();
	const uint32_t nl = smax - smin + 1;
	for (uint32_t i = threadIdx.x; i < nl * nw; i += SB_T) {
		const uint32_t w = i % nw, v = L[i / nw][w];
		if (v == sb_ident(w))
			continue;
		uint32_t *G = acc + (size_t)(smin + i / nw) * SB_ACC(nb) + 12 + w;
		const uint32_t j = w % 7;
		if (j == 6)
			atomicAdd(G, v);
		else if (j < 3)
			atomicMin(G, v);
		else
			atomicMax(G, v);
	}
}

/* the split of each node (bvh_build.cpp Builder::build): mode 0 = SAH (axis, bin), 1 = middle
 * of the range; nleft; the node's box into the tree; children that stay active */
__global__ __launch_bounds__(SB_T) void k_sb_split(uint32_t sn, uint32_t s0b, uint32_t nb, uint32_t max_leaf, uint32_t max_depth,
						    float c_trav, float c_isect, const SbNode *__restrict__ act,
						    const uint32_t *__restrict__ acc, uint4 *__restrict__ dec,
						    uint32_t *__restrict__ nact, float *__restrict__ nb6, uint32_t *__restrict__ cnt)
{
	const uint32_t i = blockIdx.x * SB_T + threadIdx.x; /* node s0b + i; accumulators i */
	if (i >= sn)
		return;
	const SbNode nd = act[s0b + i];
	const uint32_t n = nd.e - nd.b;
	const uint32_t *A = acc + (size_t)i * SB_ACC(nb);
	float blo[3], bhi[3], clo[3], chi[3];
	for (int a = 0; a < 3; a++) {
		blo[a] = o2f(A[a]);
		bhi[a] = o2f(A[3 + a]);
		clo[a] = o2f(A[6 + a]);
		chi[a] = o2f(A[9 + a]);
		nb6[6 * (size_t)nd.id + a] = blo[a];
		nb6[6 * (size_t)nd.id + 3 + a] = bhi[a];
	}
	cnt[nd.id] = n;
	int need = 0;
	while ((1u << need) < (n + max_leaf - 1) / max_leaf)
		need++;
	const bool force_median = (int)nd.depth + need + 1 >= (int)max_depth;
	int best_axis = -1;
	uint32_t best_split = 0, best_left = 0;
	float best_cost = FLT_MAX;
	if (!force_median) {
		for (int ax = 0; ax < 3; ax++) {
			const float ext = chi[ax] - clo[ax];
			if (!(ext > 0.f))
				continue;
			const uint32_t *B = A + 12 + (size_t)ax * nb * 7;
			float ra[SB_NBMAX];
			uint32_t rc[SB_NBMAX];
			float alo[3] = { FLT_MAX, FLT_MAX, FLT_MAX }, ahi[3] = { -FLT_MAX, -FLT_MAX, -FLT_MAX };
			uint32_t c = 0;
			for (int k = (int)nb - 1; k > 0; k--) {
				for (int a = 0; a < 3; a++) {
					alo[a] = fminf(alo[a], o2f(B[7 * k + a]));
					ahi[a] = fmaxf(ahi[a], o2f(B[7 * k + 3 + a]));
				}
				c += B[7 * k + 6];
				ra[k] = sb_area(alo, ahi);
				rc[k] = c;
			}
			for (int a = 0; a < 3; a++) {
				alo[a] = FLT_MAX;
				ahi[a] = -FLT_MAX;
			}
			c = 0;
			for (uint32_t k = 0; k + 1 < nb; k++) {
				for (int a = 0; a < 3; a++) {
					alo[a] = fminf(alo[a], o2f(B[7 * k + a]));
					ahi[a] = fmaxf(ahi[a], o2f(B[7 * k + 3 + a]));
				}
				c += B[7 * k + 6];
				if (!c || !rc[k + 1])
					continue;
				const float cost = sb_area(alo, ahi) * c + ra[k + 1] * rc[k + 1];
				if (cost < best_cost) {
					best_cost = cost;
					best_axis = ax;
					best_split = k;
					best_left = c;
				}
			}
		}
	}
	const float parea = sb_area(blo, bhi);
	const float split_cost = best_axis >= 0 && parea > 0 ? c_trav + c_isect * best_cost / parea : FLT_MAX;
	const float leaf_cost = c_isect * n;
	uint32_t mode, nleft;
	if (best_axis >= 0 && !force_median && !(n <= max_leaf && leaf_cost <= split_cost)) {
		mode = 0;
		nleft = best_left;
	} else { /* depth budget, equal centroids, or a leaf the emission collapses: the middle */
		mode = 1;
		nleft = n / 2;
	}
	dec[s0b + i] = make_uint4(mode | ((uint32_t)(best_axis < 0 ? 0 : best_axis) << 1), best_split, nleft, 0u);
	nact[s0b + i] = (nleft >= 2 ? 1u : 0u) + (n - nleft >= 2 ? 1u : 0u);
}

/* left flags of the positions (stable partition by scan) */
__global__ __launch_bounds__(SB_T) void k_sb_flags(uint32_t n, uint32_t nb, uint32_t s0b, uint32_t sn,
						    const uint32_t *__restrict__ seg, const uint32_t *__restrict__ pidx,
						    const float *__restrict__ lo, const float *__restrict__ hi,
						    const SbNode *__restrict__ act, const uint4 *__restrict__ dec,
						    const uint32_t *__restrict__ acc, uint32_t *__restrict__ flag)
{
	const uint32_t q = blockIdx.x * SB_T + threadIdx.x;
	if (q >= n)
		return;
	const uint32_t s = seg[q];
	if (s == RTX_NONE || s - s0b >= sn) /* not this batch's (flags start at 0) */
		return;
	uint32_t f = 0;
	{
		const uint4 d = dec[s];
		if (d.x & 1u) {
			f = q - act[s].b < d.z ? 1u : 0u;
		} else {
			const uint32_t ax = d.x >> 1, p = pidx[q];
			const uint32_t *A = acc + (size_t)(s - s0b) * SB_ACC(nb);
			const float clo = o2f(A[6 + ax]), ext = o2f(A[9 + ax]) - clo;
			const float k = (float)nb * (1.f - 1e-6f) / ext;
			const float c = 0.5f * (lo[3 * (size_t)p + ax] + hi[3 * (size_t)p + ax]);
			f = (uint32_t)sb_bin(c, clo, k, (int)nb) <= d.y ? 1u : 0u;
		}
	}
	flag[q] = f;
}

/* children: tree ids (a one-primitive child is its position), parents, next level's nodes */
__global__ __launch_bounds__(SB_T) void k_sb_children(uint32_t M, uint32_t n, uint32_t id_base, const SbNode *__restrict__ act,
						       const uint4 *__restrict__ dec, const uint32_t *__restrict__ off,
						       SbNode *__restrict__ next, uint2 *__restrict__ kids, uint32_t *__restrict__ par)
{
	const uint32_t i = blockIdx.x * SB_T + threadIdx.x;
	if (i >= M)
		return;
	const SbNode nd = act[i];
	const uint32_t nl = dec[i].z;
	uint32_t o = off[i], ch[2];
	const uint32_t b[2] = { nd.b, nd.b + nl }, e[2] = { nd.b + nl, nd.e };
	for (int c = 0; c < 2; c++) {
		if (e[c] - b[c] >= 2) {
			ch[c] = id_base + o;
			SbNode x;
			x.b = b[c];
			x.e = e[c];
			x.id = ch[c];
			x.depth = nd.depth + 1;
			next[o++] = x;
		} else {
			ch[c] = b[c];
		}
		par[ch[c]] = nd.id;
	}
	kids[nd.id - n] = make_uint2(ch[0], ch[1]);
}

/* stable partition; each position's node in the next level (RTX_NONE: a leaf) */
__global__ __launch_bounds__(SB_T) void k_sb_scatter(uint32_t n, const uint32_t *__restrict__ seg, const uint32_t *__restrict__ pidx,
						      const SbNode *__restrict__ act, const uint4 *__restrict__ dec,
						      const uint32_t *__restrict__ flag, const uint32_t *__restrict__ scan,
						      const uint32_t *__restrict__ off, uint32_t *__restrict__ pidx2,
						      uint32_t *__restrict__ seg2)
{
	const uint32_t q = blockIdx.x * SB_T + threadIdx.x;
	if (q >= n)
		return;
	const uint32_t s = seg[q];
	if (s == RTX_NONE) {
		pidx2[q] = pidx[q];
		seg2[q] = RTX_NONE;
		return;
	}
	const SbNode nd = act[s];
	const uint32_t nl = dec[s].z, lrank = scan[q] - scan[nd.b];
	const bool left = flag[q] != 0;
	const uint32_t pos = left ? nd.b + lrank : nd.b + nl + (q - nd.b - lrank);
	pidx2[pos] = pidx[q];
	const uint32_t o = off[s];
	uint32_t ns = RTX_NONE;
	if (left) {
		if (nl >= 2)
			ns = o;
	} else if (nd.e - nd.b - nl >= 2) {
		ns = o + (nl >= 2 ? 1u : 0u);
	}
	seg2[pos] = ns;
}

/* leaves (positions): their boxes, counts */
__global__ __launch_bounds__(SB_T) void k_sb_leaves(uint32_t n, const uint32_t *__restrict__ pidx, const float *__restrict__ lo,
						     const float *__restrict__ hi, float *__restrict__ nb6, uint32_t *__restrict__ cnt,
						     uint32_t *__restrict__ kcnt)
{
	const uint32_t q = blockIdx.x * SB_T + threadIdx.x;
	if (q >= n)
		return;
	const uint32_t p = pidx[q];
	for (int a = 0; a < 3; a++) {
		nb6[6 * (size_t)q + a] = lo[3 * (size_t)p + a];
		nb6[6 * (size_t)q + 3 + a] = hi[3 * (size_t)p + a];
	}
	cnt[q] = 1;
	kcnt[q] = 0;
}

/* kept inner nodes per subtree, one level at a time from the deepest */
__global__ __launch_bounds__(SB_T) void k_sb_kcnt(uint32_t M, uint32_t n, uint32_t max_leaf, uint32_t root,
						   const SbNode *__restrict__ lev, const uint2 *__restrict__ kids,
						   const uint32_t *__restrict__ cnt, uint32_t *__restrict__ kcnt)
{
	const uint32_t i = blockIdx.x * SB_T + threadIdx.x;
	if (i >= M)
		return;
	const uint32_t v = lev[i].id;
	const uint2 k = kids[v - n];
	kcnt[v] = ((v == root || cnt[v] > max_leaf) ? 1u : 0u) + kcnt[k.x] + kcnt[k.y];
}

extern "C" hipError_t rtx_sah_build(uint32_t n, const float *d_lo, const float *d_hi, const DPrim *d_prims_in,
				    uint32_t max_leaf, uint32_t bins, uint32_t max_depth, float c_trav, float c_isect,
				    DNode **recs_out, uint32_t *nnodes_out, uint32_t *root_out, uint32_t *depth_out,
				    uint32_t *levels_out, hipStream_t st)
{
	hipError_t e = hipSuccess;
	*recs_out = nullptr;
	*nnodes_out = 0;
	*depth_out = 0;
	*levels_out = 0;
	if (bins < 2 || bins > SB_NBMAX)
		return hipErrorInvalidValue;
	void *temp = nullptr;
	uint32_t *pidx = nullptr, *pidx2 = nullptr, *seg = nullptr, *seg2 = nullptr, *flag = nullptr, *scan = nullptr,
		 *acc = nullptr, *nact = nullptr, *off = nullptr, *cnt = nullptr, *kcnt = nullptr, *par = nullptr, *posmap = nullptr;
	SbNode *lev = nullptr; /* every level's nodes, one after the other (the inner nodes, n - 1 of them) */
	uint4 *dec = nullptr;
	uint2 *kids = nullptr;
	float *nb6 = nullptr;
	unsigned *scal = nullptr;
	uint32_t *tail = nullptr;
	const size_t nt = 2 * (size_t)n;
	const uint32_t nb = bins;
	std::vector<uint32_t> lev_off;
	/* accumulators for at most this many nodes at a time: a level holds nodes of two or more
	 * primitives, so never more than n / 2 of them (3 spheres: one node, not 65,536 x 2.8 KB) */
	const uint32_t chunk = std::min<uint32_t>(1u << 16, std::max<uint32_t>(1u, n / 2));
#define TRY(x)                                  \
	do {                                    \
		if ((e = (x)) != hipSuccess)    \
			goto done;              \
	} while (0)
	TRY(hipMalloc(&pidx, (size_t)n * 4));
	TRY(hipMalloc(&pidx2, (size_t)n * 4));
	TRY(hipMalloc(&seg, (size_t)n * 4));
	TRY(hipMalloc(&seg2, (size_t)n * 4));
	TRY(hipMalloc(&flag, (size_t)n * 4));
	TRY(hipMalloc(&scan, ((size_t)n + 1) * 4));
	TRY(hipMalloc(&acc, (size_t)chunk * SB_ACC(nb) * 4));
	TRY(hipMalloc(&nact, (size_t)n * 4));
	TRY(hipMalloc(&off, ((size_t)n + 1) * 4));
	TRY(hipMalloc(&dec, (size_t)n * sizeof(uint4)));
	TRY(hipMalloc(&lev, (size_t)n * sizeof(SbNode)));
	TRY(hipMalloc(&kids, (size_t)n * sizeof(uint2)));
	TRY(hipMalloc(&par, nt * 4));
	TRY(hipMalloc(&cnt, nt * 4));
	TRY(hipMalloc(&kcnt, nt * 4));
	TRY(hipMalloc(&nb6, 6 * nt * sizeof(float)));
	TRY(hipMalloc(&posmap, (size_t)n * 4));
	TRY(hipMalloc(&scal, 4 * sizeof(unsigned)));
	TRY(hipHostMalloc(&tail, 4 * sizeof(uint32_t)));
	{
		const dim3 gn((n + SB_T - 1) / SB_T);
		size_t tb = 0, tb2 = 0;
		TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, flag, scan, (int)n + 1, st));
		TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tb2, nact, off, (int)n + 1, st));
		TRY(hipMalloc(&temp, tb > tb2 ? tb : tb2));
		/* positions = input order; one active node (the root, id n) over all of them */
		{
			std::vector<uint32_t> io(n);
			for (uint32_t k = 0; k < n; k++)
				io[k] = k;
			TRY(hipMemcpyAsync(pidx, io.data(), (size_t)n * 4, hipMemcpyHostToDevice, st));
			TRY(hipMemsetAsync(seg, 0, (size_t)n * 4, st));
			SbNode r{ 0u, n, n, 1u };
			TRY(hipMemcpyAsync(lev, &r, sizeof(r), hipMemcpyHostToDevice, st));
			TRY(hipStreamSynchronize(st));
		}
		uint32_t nnodes = 0, root = RTX_EMPTY_REF, depth = 0;
		if (n > max_leaf && n >= 2) {
			uint32_t M = 1, base = 0, id_next = n + 1;
			lev_off.push_back(0);
			while (M) {
				if (lev_off.size() > 4096) { /* a level always splits every node: cannot happen */
					e = hipErrorUnknown;
					goto done;
				}
				SbNode *act = lev + base;
				TRY(hipMemsetAsync(flag, 0, (size_t)n * 4, st));
				/* the level's nodes in batches of at most `chunk` (the accumulators) */
				for (uint32_t s0b = 0; s0b < M; s0b += chunk) {
					const uint32_t sn = std::min(chunk, M - s0b);
					const size_t na = (size_t)sn * SB_ACC(nb);
					hipLaunchKernelGGL(k_sb_reset, dim3((uint32_t)((na + SB_T - 1) / SB_T)), dim3(SB_T), 0, st, sn, nb, acc);
					hipLaunchKernelGGL(k_sb_bounds, gn, dim3(SB_T), 0, st, n, nb, s0b, sn, seg, pidx, d_lo, d_hi, acc);
					hipLaunchKernelGGL(k_sb_bins, gn, dim3(SB_T), 0, st, n, nb, s0b, sn, seg, pidx, d_lo, d_hi, acc);
					hipLaunchKernelGGL(k_sb_split, dim3((sn + SB_T - 1) / SB_T), dim3(SB_T), 0, st, sn, s0b, nb, max_leaf,
							   max_depth, c_trav, c_isect, act, acc, dec, nact, nb6, cnt);
					hipLaunchKernelGGL(k_sb_flags, gn, dim3(SB_T), 0, st, n, nb, s0b, sn, seg, pidx, d_lo, d_hi, act, dec, acc,
							   flag);
					TRY(hipGetLastError());
				}
				const dim3 gm((M + SB_T - 1) / SB_T);
				TRY(hipMemsetAsync(nact + M, 0, 4, st));
				TRY(hipcub::DeviceScan::ExclusiveSum(temp, tb2, nact, off, (int)M + 1, st));
				TRY(hipcub::DeviceScan::ExclusiveSum(temp, tb, flag, scan, (int)n, st));
				hipLaunchKernelGGL(k_sb_children, gm, dim3(SB_T), 0, st, M, n, id_next, act, dec, off, lev + base + M, kids, par);
				hipLaunchKernelGGL(k_sb_scatter, gn, dim3(SB_T), 0, st, n, seg, pidx, act, dec, flag, scan, off, pidx2, seg2);
				TRY(hipGetLastError());
				TRY(hipMemcpyAsync(&tail[0], off + M, 4, hipMemcpyDeviceToHost, st));
				TRY(hipStreamSynchronize(st));
				std::swap(pidx, pidx2);
				std::swap(seg, seg2);
				base += M;
				id_next += tail[0];
				M = tail[0];
				lev_off.push_back(base);
			}
			root = n;
			nnodes = base; /* every inner node is kept at max_leaf 1; counted exactly below */
			hipLaunchKernelGGL(k_sb_leaves, gn, dim3(SB_T), 0, st, n, pidx, d_lo, d_hi, nb6, cnt, kcnt);
			for (size_t l = lev_off.size() - 1; l-- > 0;) {
				const uint32_t m = lev_off[l + 1] - lev_off[l];
				hipLaunchKernelGGL(k_sb_kcnt, dim3((m + SB_T - 1) / SB_T), dim3(SB_T), 0, st, m, n, max_leaf, root,
						   lev + lev_off[l], kids, cnt, kcnt);
			}
			TRY(hipGetLastError());
			TRY(hipMemcpyAsync(&nnodes, kcnt + root, 4, hipMemcpyDeviceToHost, st));
			TRY(hipMemsetAsync(scal, 0, 4 * sizeof(unsigned), st));
			hipLaunchKernelGGL(k_pl_leafpos, gn, dim3(PLOC_T), 0, st, n, root, max_leaf, pidx, kids, par, cnt, kcnt, posmap, scal);
			TRY(hipGetLastError());
			TRY(hipMemcpyAsync(&depth, scal, 4, hipMemcpyDeviceToHost, st));
			TRY(hipStreamSynchronize(st));
			depth += 1; /* the host builder's count: the leaves' level */
		} else {
			TRY(hipMemcpyAsync(posmap, pidx, (size_t)n * 4, hipMemcpyDeviceToDevice, st));
		}
		DNode *recs = nullptr;
		TRY(hipMalloc(&recs, ((size_t)nnodes + n) * sizeof(DNode)));
		/* k_pl_emit: inner ids n .. n + (n - 2), root n */
		hipLaunchKernelGGL(k_pl_emit, gn, dim3(PLOC_T), 0, st, n, root != RTX_EMPTY_REF ? n - 1 : 0u, root, max_leaf, nnodes, kids,
				   par, cnt, kcnt, nb6, posmap, d_prims_in, recs);
		e = hipGetLastError();
		if (e == hipSuccess)
			e = hipStreamSynchronize(st);
		if (e != hipSuccess) {
			(void)hipFree(recs);
			goto done;
		}
		*recs_out = recs;
		*nnodes_out = nnodes;
		*root_out = root != RTX_EMPTY_REF ? 0u : RTX_EMPTY_REF;
		*depth_out = root != RTX_EMPTY_REF ? depth : 0u;
		*levels_out = (uint32_t)(lev_off.empty() ? 0 : lev_off.size() - 1);
	}
done:
#undef TRY
	(void)hipFree(temp);
	(void)hipFree(pidx);
	(void)hipFree(pidx2);
	(void)hipFree(seg);
	(void)hipFree(seg2);
	(void)hipFree(flag);
	(void)hipFree(scan);
	(void)hipFree(acc);
	(void)hipFree(nact);
	(void)hipFree(off);
	(void)hipFree(dec);
	(void)hipFree(lev);
	(void)hipFree(kids);
	(void)hipFree(par);
	(void)hipFree(cnt);
	(void)hipFree(kcnt);
	(void)hipFree(nb6);
	(void)hipFree(posmap);
	(void)hipFree(scal);
	(void)hipHostFree(tail);
	return e;
}

/* the record index of each of nobj objects (the emitters) among n primitive records: out[j] = k
 * where record k's object id (DPrim b[3]) is objs[j]; out left RTX_NONE for an object without
 * a record.  One thread per record; each object has at most one record, so no races. */
__global__ void k_find_prims(const DPrim *__restrict__ prims, uint32_t n, const uint32_t *__restrict__ objs, uint32_t nobj,
			     uint32_t *__restrict__ out)
{
	const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
	if (k >= n)
		return;
	const uint32_t obj = __float_as_uint(prims[k].b[3]);
	for (uint32_t j = 0; j < nobj; j++)
		if (objs[j] == obj)
			out[j] = k;
}

extern "C" hipError_t rtx_launch_find_prims(const DPrim *prims, uint32_t n, const uint32_t *objs, uint32_t nobj, uint32_t *out,
					     hipStream_t stream)
{
	if (!n || !nobj)
		return hipSuccess;
	hipLaunchKernelGGL(k_find_prims, dim3((n + 255) / 256), dim3(256), 0, stream, prims, n, objs, nobj, out);
	return hipGetLastError();
}

/* the code object of this file on the current device, loaded now (rtx_open) rather than at the
 * first launch inside an upload or a render */
extern "C" __attribute__((visibility("hidden"))) hipError_t rtx_load_build(void)
{
	hipFuncAttributes a;
	return hipFuncGetAttributes(&a, (const void *)k_sb_reset);
}
