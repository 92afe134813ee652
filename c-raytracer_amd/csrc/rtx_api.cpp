/*
 * C-ABI of include/rtx.h: device context, scene flattening + BVH upload
 * (replaces accel_init, accel.c:266-315), render (replaces render_init +
 * render, render.c:61-116 / 345-368), statistics, known-answer entry.
 */
#include <hip/hip_runtime.h>

#include <float.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <vector>

#include "bvh_build.h"
#include "rtx.h"
#include "rtx_device.h"
#include "rtx_frame.h"
#include "rtx_kat.h"
#include "rtx_quant.h"
#include "rtx_internal.h"

extern "C" size_t rtx_trace_lds_bytes(uint32_t stack_size);
extern "C" size_t rtx_shadow_lds_bytes(uint32_t stack_size);
extern "C" hipError_t rtx_trace_occupancy(uint32_t stack_size, int *blocks_per_cu);
extern "C" hipError_t rtx_launch_trace(const DScene *S, const DFrame *F, const DParams *P, float *rgb, float *z,
				       DTask *tasks, uint32_t task_cap, float4 *staging, uint32_t staging_cap,
				       float4 *sp_out, uint32_t sp_cap, uint2 *tile_rec, uint32_t tile_begin,
				       uint32_t tile_end, unsigned long long *ctr, uint32_t waves, int count,
				       hipStream_t stream);
extern "C" hipError_t rtx_launch_shadow(const DScene *S, const DParams *P, const float4 *sp, const uint32_t *perm,
					uint32_t n_sp, uint32_t per_wave, uint32_t slot_b, float4 *contrib,
					unsigned long long *ctr, int count, uint32_t cus, hipStream_t stream);
extern "C" hipError_t rtx_launch_post(uint32_t w, uint32_t h, const rtx_post *pp, float *rgb, const float *z,
				      int *rad, float4 *pv, unsigned *scratch, hipStream_t stream);
extern "C" hipError_t rtx_spsort_temp_bytes(uint32_t n, size_t *bytes);
extern "C" hipError_t rtx_ploc_build(uint32_t n, const float *d_lo, const float *d_hi, const DPrim *d_prims_in,
				     const float blo[3], const float bhi[3], uint32_t max_leaf, DNode **recs_out,
				     uint32_t *nnodes_out, uint32_t *root_out, uint32_t *depth_out, uint32_t *rounds_out,
				     hipStream_t st);
extern "C" hipError_t rtx_sah_build(uint32_t n, const float *d_lo, const float *d_hi, const DPrim *d_prims_in,
				    uint32_t max_leaf, uint32_t bins, uint32_t max_depth, float c_trav, float c_isect,
				    DNode **recs_out, uint32_t *nnodes_out, uint32_t *root_out, uint32_t *depth_out,
				    uint32_t *levels_out, hipStream_t st);
extern "C" hipError_t rtx_w8_collapse_device(const DNode *recs, uint32_t nnodes, uint32_t nb, const uint32_t *skip_obj,
					     uint32_t num_objects, DW8 **w8_out, DW8S **w8s_out, uint32_t **leafmap_out,
					     uint32_t *entries_out, uint32_t *scalar_entries_out, uint32_t *depth_out,
					     uint32_t *wide_out, uint32_t *top_out, float qo[3], float qs[3], hipStream_t st);
extern "C" hipError_t rtx_launch_w8_scalar(uint32_t n, const DW8 *w8, const uint32_t *leafmap, DW8S *w8s, hipStream_t st);
extern "C" hipError_t rtx_lbvh_build(uint32_t n, const float *d_lo, const float *d_hi, const DPrim *d_prims_in,
				     const float blo[3], const float bhi[3], uint32_t max_leaf, DNode **recs_out,
				     uint32_t *nnodes_out, uint32_t *root_out, uint32_t *depth_out, hipStream_t st);
extern "C" hipError_t rtx_launch_spsort(const float4 *sp, uint32_t n, const float lo[3], const float hi[3],
					uint32_t *keys0, uint32_t *keys1, uint32_t *vals0, uint32_t *vals1, void *temp,
					size_t temp_bytes, const uint32_t **perm, hipStream_t stream);
extern "C" hipError_t rtx_launch_accum(const DFrame *F, const DParams *P, const uint2 *tile_rec,
				       const float4 *contrib, uint32_t tile_begin, uint32_t ntiles, float *rgb,
				       hipStream_t stream);
extern "C" hipError_t rtx_launch_kat(int kind, uint32_t n, const float *in, float *out, int u32mode,
				     hipStream_t stream);
extern "C" hipError_t rtx_launch_find_prims(const DPrim *prims, uint32_t n, const uint32_t *objs, uint32_t nobj, uint32_t *out,
					     hipStream_t stream);
extern "C" hipError_t rtx_launch_kat_shadow(int kind, uint32_t n, const float *in, float *out, hipStream_t stream);
extern "C" hipError_t rtx_launch_w8_fill(const DPrim *prims, const DMaterial *mats, const uint32_t *leafmap, uint32_t n, DW8 *out,
					  hipStream_t stream);
extern "C" hipError_t rtx_shadow_grid_lanes(uint32_t cus, uint32_t *lanes);

/* the code objects of the library's device files (each file's rtx_load_*) */
extern "C" hipError_t rtx_load_build(void);
extern "C" hipError_t rtx_load_wide8_dev(void);
extern "C" hipError_t rtx_load_shadow(void);
extern "C" hipError_t rtx_load_trace(void);
extern "C" hipError_t rtx_load_sort(void);
extern "C" hipError_t rtx_load_post(void);
extern "C" hipError_t rtx_load_gather(void);

static thread_local char g_err[512] = "";

/* measurement builds (EXTRA=-DRTX_MEASURE=1): host-side phase times of an upload on stderr */
#if RTX_MEASURE
struct PhaseClock {
	std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
	void mark(const char *what, hipStream_t st)
	{
		(void)hipStreamSynchronize(st);
		const auto n = std::chrono::steady_clock::now();
		fprintf(stderr, "[rtx upload] %-24s %8.2f ms\n", what, std::chrono::duration<double, std::milli>(n - t).count());
		t = n;
	}
};
#define PHASE(clk, what, st) clk.mark(what, st)
#else
struct PhaseClock {};
#define PHASE(clk, what, st) ((void)clk)
#endif

int rtx_fail(int code, const char *fmt, ...)
{
	va_list ap;
	va_start(ap, fmt);
	vsnprintf(g_err, sizeof(g_err), fmt, ap);
	va_end(ap);
	return code;
}


extern "C" const char *rtx_last_error(void)
{
	return g_err;
}

extern "C" void rtx_params_default(rtx_params *p)
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
	p->count_traversal = 0;
}

extern "C" int rtx_device_count(int *count)
{
	if (!count)
		return fail(RTX_ERR_ARG, "null count");
	int n = 0;
	hipError_t e = hipGetDeviceCount(&n);
	*count = (e == hipSuccess) ? n : 0;
	return RTX_OK;
}


static void free_scene(rtx_ctx *c)
{
	dfree(c->d_nodes);
	dfree(c->d_planes);
	dfree(c->d_mats);
	dfree(c->d_emitters);
	dfree(c->d_lin);
	dfree(c->d_cull);
	dfree(c->d_qnodes);
	dfree(c->d_top);
	dfree(c->d_w8);
	dfree(c->d_w8s);
	c->have_scene = false;
	c->sp_tile_seen = 0.0;
	c->sp_tile_key = SpKey{};
}

extern "C" void rtx_close(rtx_ctx *c)
{
	if (!c)
		return;
	(void)hipSetDevice(c->device);
	if (c->stream)
		(void)hipStreamSynchronize(c->stream);
	free_scene(c);
	dfree(c->d_tasks);
	dfree(c->d_ostk);
	c->ostk_bytes = 0;
	dfree(c->d_w8spill);
	c->w8spill_bytes = 0;
	dfree(c->d_sortbuf);
	dfree(c->d_sorttmp);
	dfree(c->d_post_rad);
	dfree(c->d_post_pv);
	dfree(c->d_post_scratch);
	dfree(c->d_staging);
	dfree(c->d_sp);
	dfree(c->d_contrib);
	dfree(c->d_tile_rec);
	for (auto &e : c->ev)
		if (e)
			(void)hipEventDestroy(e);
	dfree(c->d_ctr);
	dfree(c->d_rgb);
	dfree(c->d_z);
	if (c->ev0)
		(void)hipEventDestroy(c->ev0);
	if (c->ev1)
		(void)hipEventDestroy(c->ev1);
	if (c->stream)
		(void)hipStreamDestroy(c->stream);
	delete c;
}

extern "C" int rtx_open(int device, rtx_ctx **out)
{
	if (!out)
		return fail(RTX_ERR_ARG, "null out");
	*out = nullptr;
	int n = 0;
	if (hipGetDeviceCount(&n) != hipSuccess || n <= 0)
		return fail(RTX_ERR_NODEV, "no HIP device available");
	if (device < 0 || device >= n)
		return fail(RTX_ERR_NODEV, "device %d out of range (%d devices)", device, n);
	hipDeviceProp_t prop;
	HIP_TRY(hipGetDeviceProperties(&prop, device));
	if (!strstr(prop.gcnArchName, "gfx950"))
		return fail(RTX_ERR_NODEV, "device %d is %s, this build targets gfx950 only", device, prop.gcnArchName);
	rtx_ctx *c = new rtx_ctx();
	c->device = device;
	c->cus = prop.multiProcessorCount;
	hipError_t e;
	if ((e = hipSetDevice(device)) != hipSuccess || (e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)) != hipSuccess ||
	    (e = hipEventCreate(&c->ev0)) != hipSuccess || (e = hipEventCreate(&c->ev1)) != hipSuccess ||
	    (e = hipEventCreate(&c->ev[0])) != hipSuccess || (e = hipEventCreate(&c->ev[1])) != hipSuccess ||
	    (e = hipEventCreate(&c->ev[2])) != hipSuccess || (e = hipEventCreate(&c->ev[3])) != hipSuccess ||
	    (e = hipEventCreate(&c->ev[4])) != hipSuccess ||
	    (e = hipMalloc(&c->d_ctr, sizeof(unsigned long long) * RTX_C_N)) != hipSuccess) {
		rtx_close(c);
		return fail(RTX_ERR_HIP, "context setup failed: %s", hipGetErrorString(e));
	}
	/* one-time device set-up here rather than inside the first upload or render: every code object
	 * of the library loaded on this device (the runtime loads one at its first launch otherwise,
	 * ~30 ms inside the first BVH build), and the runtime's pageable-copy path primed */
	for (hipError_t (*load)(void) : { rtx_load_build, rtx_load_wide8_dev, rtx_load_shadow, rtx_load_trace, rtx_load_sort,
					  rtx_load_post, rtx_load_gather })
		if ((e = load()) != hipSuccess) {
			rtx_close(c);
			return fail(RTX_ERR_HIP, "loading the device code failed: %s", hipGetErrorString(e));
		}
	{
		std::vector<uint8_t> h((size_t)4 << 20, 0);
		void *d = nullptr;
		e = hipMalloc(&d, h.size());
		if (e == hipSuccess)
			e = hipMemcpyAsync(d, h.data(), h.size(), hipMemcpyHostToDevice, c->stream);
		if (e == hipSuccess)
			e = hipMemcpyAsync(h.data(), d, 64, hipMemcpyDeviceToHost, c->stream);
		if (e == hipSuccess)
			e = hipStreamSynchronize(c->stream);
		if (d)
			(void)hipFree(d);
		if (e != hipSuccess) {
			rtx_close(c);
			return fail(RTX_ERR_HIP, "context setup failed: %s", hipGetErrorString(e));
		}
	}
	*out = c;
	return RTX_OK;
}


/* DQNode preorder of the subtree at device ref `ref` (rtx_device.h): the node itself with the
 * box it has in its parent, then its left and right subtrees.  An inner node's link is the
 * index after its subtree (subtree sizes from `size`, filled by thread_sizes); a leaf keeps
 * its device ref. */
static uint32_t thread_sizes(const std::vector<DNode> &recs, uint32_t ref, std::vector<uint32_t> &size)
{
	if (ref & RTX_REF_LEAF)
		return 1;
	const uint32_t i = (ref & RTX_REF_OFF) / (uint32_t)sizeof(DNode);
	const DNode &n = recs[i];
	size[i] = 1 + thread_sizes(recs, n.ref0, size) + thread_sizes(recs, n.ref1, size);
	return size[i];
}


/* one plane pair quantised conservatively (rtx_quant.h) */
static uint32_t quantise(float lo, float hi, float qo, float qs) { return rtx_quantise(lo, hi, qo, qs); }

static void thread_emit(const std::vector<DNode> &recs, const std::vector<uint32_t> &size, const QFrame &F,
			uint32_t ref, const float lo[3], const float hi[3], std::vector<DQNode> &out, uint32_t dep,
			std::vector<uint32_t> &depth)
{
	DQNode t;
	t.x = quantise(lo[0], hi[0], F.qo[0], F.qs[0]);
	t.y = quantise(lo[1], hi[1], F.qo[1], F.qs[1]);
	t.z = quantise(lo[2], hi[2], F.qo[2], F.qs[2]);
	const uint32_t me = (uint32_t)out.size();
	if (ref & RTX_REF_LEAF) {
		t.link = ref;
		out.push_back(t);
		depth.push_back(dep);
		return;
	}
	const uint32_t i = (ref & RTX_REF_OFF) / (uint32_t)sizeof(DNode);
	t.link = (me + size[i]) << 6;
	out.push_back(t);
	depth.push_back(dep);
	const DNode &n = recs[i];
	const float l0[3] = { n.lo0x, n.lo0y, n.lo0z }, h0[3] = { n.hi0x, n.hi0y, n.hi0z };
	const float l1[3] = { n.lo1x, n.lo1y, n.lo1z }, h1[3] = { n.hi1x, n.hi1y, n.hi1z };
	thread_emit(recs, size, F, n.ref0, l0, h0, out, dep + 1, depth);
	thread_emit(recs, size, F, n.ref1, l1, h1, out, dep + 1, depth);
}

/* the quantised threaded BVH and its frame: the bounded objects' box, 65533 steps per axis */
static void thread_bvh(const std::vector<DNode> &inner, uint32_t root_ref, const float lo[3], const float hi[3],
		       std::vector<DQNode> &out, QFrame &F, std::vector<uint32_t> &depth)
{
	out.clear();
	depth.clear();
	float ext_max = 0.f;
	for (int a = 0; a < 3; a++)
		ext_max = std::max(ext_max, hi[a] - lo[a]);
	for (int a = 0; a < 3; a++) {
		F.qo[a] = lo[a];
		const float ext = std::max(hi[a] - lo[a], std::max(ext_max, 1.f) * 1e-6f);
		F.qs[a] = 65533.f / ext;
	}
	if (root_ref == RTX_EMPTY_REF)
		return;
	std::vector<uint32_t> size(inner.size(), 0);
	const uint32_t total = thread_sizes(inner, root_ref, size);
	out.reserve(total);
	thread_emit(inner, size, F, root_ref, lo, hi, out, 0, depth);
}

/* the LDS copy of the threaded BVH's top levels (rtx_device.h RTX_QTOP_CUT): every node
 * shallower than the deepest cut that keeps at most RTX_TOP_MAX records */
static uint32_t thread_top(const std::vector<DQNode> &q, const std::vector<uint32_t> &depth, std::vector<uint32_t> &top)
{
	top.clear();
	if (q.empty())
		return 0;
	std::vector<size_t> hist(66, 0);
	for (uint32_t dj : depth)
		hist[std::min<uint32_t>(dj, 65)]++;
	uint32_t D = 1; /* the top = nodes of depth < D */
	size_t cnt = hist[0];
	while (D < 65 && hist[D] && cnt + hist[D] <= RTX_TOP_MAX) {
		cnt += hist[D];
		D++;
	}
	std::vector<uint32_t> id(q.size(), RTX_NONE);
	uint32_t nt = 0;
	for (size_t j = 0; j < q.size(); j++)
		if (depth[j] < D)
			id[j] = nt++;
	top.assign(5 * (size_t)nt, 0);
	for (size_t j = 0; j < q.size(); j++) {
		if (id[j] == RTX_NONE)
			continue;
		uint32_t *T = &top[4 * (size_t)id[j]];
		T[0] = q[j].x;
		T[1] = q[j].y;
		T[2] = q[j].z;
		const uint32_t link = q[j].link;
		if (link & RTX_REF_LEAF) {
			T[3] = link;
		} else if (depth[j] == D - 1) {
			T[3] = (((uint32_t)j + 1) << 6) | RTX_QTOP_CUT;
			top[4 * (size_t)nt + id[j]] = link >> 6;
		} else {
			/* the node after an above-cut subtree is a sibling's or an ancestor's: in the top */
			const uint32_t e = link >> 6;
			T[3] = (e < q.size() ? id[e] : nt) << 6;
		}
	}
	return nt;
}

int rtx_build_scene(rtx_ctx *c, const rtx_scene_desc *sc, HostScene &hs)
{
	if (!sc->num_materials || !sc->materials)
		return fail(RTX_ERR_SCENE, "scene has no materials");
	if (sc->num_objects && !sc->objects)
		return fail(RTX_ERR_ARG, "objects pointer is null");
	if (sc->num_emitters && !sc->emitters)
		return fail(RTX_ERR_ARG, "emitters pointer is null");
	HIP_TRY(hipSetDevice(c->device));
	PhaseClock clk0;
	free_scene(c);
	PHASE(clk0, "free the old scene", c->stream);
	hs.builder = c->builder;

	if (sc->num_materials > RTX_META_MAT)
		return fail(RTX_ERR_SCENE, "too many materials (%u)", sc->num_materials);
	std::vector<DMaterial> mats(sc->num_materials);
	for (uint32_t i = 0; i < sc->num_materials; i++) {
		const rtx_material &m = sc->materials[i];
		DMaterial &d = mats[i];
		memset(&d, 0, sizeof(d));
		memcpy(d.ks, m.ks, 12);
		memcpy(d.ka, m.ka, 12);
		memcpy(d.kr, m.kr, 12);
		memcpy(d.kt, m.kt, 12);
		memcpy(d.ke, m.ke, 12);
		d.shininess = m.shininess;
		d.ior = m.refractive_index;
		d.tex = m.texture;
		d.periodic = m.periodic;
		memcpy(d.color, m.color, sizeof(d.color));
		d.scale = m.scale;
		d.mortar = m.mortar_width;
		d.nfs = m.noise_feature_scale;
		d.ns = m.noise_scale;
		d.fs = m.frequency_scale;
		d.flags = (m.emittant ? RTX_MF_EMITTANT : 0) | (m.reflective ? RTX_MF_REFLECTIVE : 0) |
			  (m.transparent ? RTX_MF_TRANSPARENT : 0);
	}

	std::vector<uint32_t> bounded;
	std::vector<DPlane> planes;
	std::vector<uint32_t> plane_of(sc->num_objects, RTX_NONE);
	for (uint32_t i = 0; i < sc->num_objects; i++) {
		const rtx_object &o = sc->objects[i];
		if (o.material < 0 || (uint32_t)o.material >= sc->num_materials)
			return fail(RTX_ERR_SCENE, "object %u: material index %d out of range", i, o.material);
		if (o.type == RTX_PLANE) {
			DPlane p;
			memset(&p, 0, sizeof(p));
			memcpy(p.n, o.n, 12);
			p.d = o.d;
			p.eps = o.epsilon;
			p.obj = i;
			p.mat = (uint32_t)o.material;
			p.transparent = (mats[o.material].flags & RTX_MF_TRANSPARENT) ? 1u : 0u;
			memcpy(p.kt, mats[o.material].kt, 12);
			plane_of[i] = (uint32_t)planes.size();
			planes.push_back(p);
		} else if (o.type == RTX_SPHERE || o.type == RTX_TRIANGLE) {
			bounded.push_back(i);
		} else {
			return fail(RTX_ERR_SCENE, "object %u: unknown type %d", i, o.type);
		}
	}

	/* leaf boxes (sphere_get_corners / triangle_get_corners), padded so the traversal's
	 * FMA slab test is conservative: in world space for the bounded objects' box (the
	 * shade-point sort's frame), then in the trees' frame (rtx_frame.cpp) for the builders */
	const uint32_t nb = (uint32_t)bounded.size();
	std::vector<float> lo(3 * (size_t)nb), hi(3 * (size_t)nb);
	PHASE(clk0, "materials + planes", c->stream);
	rtx_world_boxes(sc, bounded, lo.data(), hi.data(), c->bound_lo, c->bound_hi);
	PHASE(clk0, "world boxes", c->stream);
	PhaseClock clk;
	const auto tf0 = std::chrono::steady_clock::now();
	DTreeFrame &tf = hs.tf;
	hs.frame_ratio = c->opt_frame == RTX_FRAME_AUTO ? rtx_frame_choose(sc, bounded, c->bound_lo, c->bound_hi, tf) : 1.0;
	if (c->opt_frame != RTX_FRAME_AUTO)
		rtx_frame_choose(sc, {}, c->bound_lo, c->bound_hi, tf); /* the identity */
	float tlo[3], thi[3]; /* the bounded objects' box in the trees' frame */
	memcpy(tlo, c->bound_lo, 12);
	memcpy(thi, c->bound_hi, 12);
	/* the objects' centre and radius for the far-origin test (rtx_math.h tf_far), in every frame */
	rtx_frame_far(c->bound_lo, c->bound_hi, tf);
	if (tf.rotated) {
		const double pad = hs.frame_pad = rtx_frame_pad(rtx_frame_radius(c->bound_lo, c->bound_hi, tf));
		rtx_frame_boxes(sc, bounded, tf, pad, lo.data(), hi.data(), tlo, thi);
	}
	hs.frame_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tf0).count();
	BvhConfig cfg;
	cfg.max_leaf = c->opt_leaf; /* RTX_OPT_BVH_LEAF (default 1) */

	/* one 64-byte primitive record (rtx_device.h DPrim) of bounded object oi */
	auto make_prim = [&](uint32_t oi) {
		const rtx_object &o = sc->objects[oi];
		DPrim p;
		memset(&p, 0, sizeof(p));
		uint32_t meta = ((uint32_t)o.type << 24) | (uint32_t)o.material;
		if (mats[o.material].flags & RTX_MF_TRANSPARENT)
			meta |= RTX_META_TRANSPARENT;
		memcpy(p.a, o.p0, 12);
		p.a[3] = o.epsilon;
		if (o.type == RTX_SPHERE) {
			p.b[0] = o.radius;
		} else {
			memcpy(p.b, o.e1, 12);
			memcpy(p.c, o.e2, 12);
			memcpy(p.d, o.n, 12);
		}
		memcpy(&p.b[3], &oi, 4);
		memcpy(&p.c[3], &meta, 4);
		return p;
	};
	auto is_sphere = [](const DPrim &p) {
		uint32_t meta;
		memcpy(&meta, &p.c[3], 4);
		return (meta >> 24) == RTX_SPHERE;
	};

	std::vector<DEmitter> emit(sc->num_emitters);
	for (uint32_t i = 0; i < sc->num_emitters; i++) {
		uint32_t oi = sc->emitters[i];
		if (oi >= sc->num_objects)
			return fail(RTX_ERR_SCENE, "emitter %u: object %u out of range", i, oi);
		const rtx_object &o = sc->objects[oi];
		if (o.type == RTX_PLANE)
			return fail(RTX_ERR_SCENE, "Plane cannot be emittant");
		DEmitter &e = emit[i];
		memset(&e, 0, sizeof(e));
		e.obj = oi;
		e.type = (uint32_t)o.type;
		e.num_lights = o.num_lights;
		const rtx_material &m = sc->materials[o.material];
		float inv = 1.f / (float)o.num_lights; /* render.c:175 */
		for (int a = 0; a < 3; a++)
			e.li[a] = m.ke[a] * inv;
		memcpy(e.p0, o.p0, 12);
		memcpy(e.p1, o.p1, 12);
		memcpy(e.p2, o.p2, 12);
		e.radius = o.radius;
		memcpy(e.e1, o.e1, 12);
		memcpy(e.e2, o.e2, 12);
		e.eps = o.epsilon;
		e.prim = RTX_NONE;
		e.transparent = (mats[o.material].flags & RTX_MF_TRANSPARENT) ? 1u : 0u;
		memcpy(e.kt, mats[o.material].kt, 12);
		rtx_world_box(o, e.wlo, e.whi);
	}

	const auto tb0 = std::chrono::steady_clock::now();
	uint32_t nnodes = 0, root_ref = RTX_EMPTY_REF, depth = 0;
	/* RTX_WALK_AUTO: a scene whose threaded BVH2 fits the LDS top records is walked from LDS alone
	 * (scene3, 3 spheres: 102 ms vs 114 ms over the 8-wide tree); larger ones over the 8-wide tree */
	const bool small = (uint64_t)2 * nb <= RTX_TOP_MAX + 1;
	/* a tiny scene (RTX_WALK_LINEAR): k_shadow tests its few bounded objects one by one like the planes
	 * (scene1 / scene3: 3 spheres, one of them the light), no walk */
	const bool linear = nb && (c->opt_walk == RTX_WALK_LINEAR || (c->opt_walk == RTX_WALK_AUTO && nb <= RTX_SHADOW_LINEAR_MAX));
	const bool want_w8 = nb && !linear && (c->opt_walk == RTX_WALK_W8 || (c->opt_walk == RTX_WALK_AUTO && !small));
	std::vector<DNode> inner; /* host copy of the inner-node records (threaded BVH2, host collapse) */
	std::vector<DPrim> prims_dl; /* device builders: the primitive records read back (host collapse) */
	const DPrim *host_prims = nullptr; /* the primitive records in leaf order on the host */
	hs.device = c->device;
	int rc;
	if ((c->builder == RTX_BUILD_LBVH_GPU || c->builder == RTX_BUILD_PLOC_GPU || c->builder == RTX_BUILD_SAH_GPU) && nb) {
		/* GPU builders (rtx_build.hip): primitives uploaded in input order, records emitted on the device */
		std::vector<DPrim> prims_in(nb);
		rtx_host_parallel(nb, [&](size_t b, size_t e, unsigned) {
			for (size_t k = b; k < e; k++)
				prims_in[k] = make_prim(bounded[k]);
		});
		uint32_t sph = 0;
		for (uint32_t k = 0; k < nb && !sph; k++)
			if (sc->objects[bounded[k]].type == RTX_SPHERE)
				sph = RTX_REF_SPH;
		float *d_lo = nullptr, *d_hi = nullptr;
		DPrim *d_in = nullptr;
		DNode *recs = nullptr;
		PHASE(clk, "frame + boxes + records", c->stream);
		if ((rc = upload(d_lo, lo, c->stream)) || (rc = upload(d_hi, hi, c->stream)) || (rc = upload(d_in, prims_in, c->stream))) {
			dfree(d_lo);
			dfree(d_hi);
			dfree(d_in);
			return rc;
		}
		PHASE(clk, "upload boxes + records", c->stream);
		uint32_t rounds = 0;
		hipError_t e = c->builder == RTX_BUILD_PLOC_GPU
				       ? rtx_ploc_build(nb, d_lo, d_hi, d_in, tlo, thi, cfg.max_leaf, &recs, &nnodes,
							&root_ref, &depth, &rounds, c->stream)
			       : c->builder == RTX_BUILD_SAH_GPU
				       ? rtx_sah_build(nb, d_lo, d_hi, d_in, cfg.max_leaf, cfg.bins, cfg.max_depth, cfg.c_trav, cfg.c_isect,
						       &recs, &nnodes, &root_ref, &depth, &rounds, c->stream)
				       : rtx_lbvh_build(nb, d_lo, d_hi, d_in, tlo, thi, cfg.max_leaf, &recs, &nnodes,
							&root_ref, &depth, c->stream);
		dfree(d_lo);
		dfree(d_hi);
		dfree(d_in);
		if (e != hipSuccess)
			return fail(RTX_ERR_HIP, "GPU BVH build failed: %s", hipGetErrorString(e));
		PHASE(clk, "device BVH2 build", c->stream);
		c->d_nodes = recs;
		hs.recs_on_device = true;
		if (root_ref == RTX_EMPTY_REF) /* nb <= max_leaf: a single leaf */
			root_ref = RTX_REF_LEAF | sph | (nb - 1);
		if (((uint64_t)nnodes + nb) * sizeof(DNode) > 0xFFFFFFC0ull)
			return fail(RTX_ERR_SCENE, "scene too large: %u BVH nodes + %u primitives exceed 4 GB of records", nnodes,
				    nb);
		/* the 8-wide tree collapsed where the records are (single-primitive leaves) */
		if (want_w8 && cfg.max_leaf == 1 && nnodes) {
			std::vector<uint32_t> skip((sc->num_objects + 31) / 32 + 1, 0u);
			for (uint32_t i = 0; i < sc->num_emitters; i++)
				skip[sc->emitters[i] >> 5] |= 1u << (sc->emitters[i] & 31u);
			uint32_t *d_skip = nullptr;
			if ((rc = upload(d_skip, skip, c->stream)))
				return rc;
			uint32_t ent = 0, dep = 0, wide = 0, top = 0;
			e = rtx_w8_collapse_device(recs, nnodes, nb, d_skip, sc->num_objects, &hs.dev_w8, &hs.dev_w8s, &hs.dev_w8leaf, &ent,
						   &hs.w8s_entries, &dep, &wide, &top, hs.w8f.qo, hs.w8f.qs, c->stream);
			dfree(d_skip);
			if (e != hipSuccess)
				return fail(RTX_ERR_HIP, "8-wide BVH collapse on the device failed: %s", hipGetErrorString(e));
			PHASE(clk, "device 8-wide collapse", c->stream);
			if (dep) {
				hs.w8_on_device = true;
				hs.w8depth = dep;
				hs.w8_entries = ent;
				hs.w8_wide = wide;
				hs.w8top = top;
				hs.w8noemit = sc->num_emitters > 0;
			}
		}
		/* the host needs the records only for the host collapse or the threaded BVH2 */
		if (!hs.w8_on_device) {
			inner.resize(nnodes);
			if (nnodes)
				HIP_TRY(hipMemcpy(inner.data(), recs, nnodes * sizeof(DNode), hipMemcpyDeviceToHost));
			prims_dl.resize(nb);
			HIP_TRY(hipMemcpy(prims_dl.data(), recs + nnodes, (size_t)nb * sizeof(DPrim), hipMemcpyDeviceToHost));
			host_prims = prims_dl.data();
		}
		/* the emitters' record indices (the 8-wide closest-hit walk tests them apart from the tree),
		 * found on the device */
		if (!emit.empty()) {
			std::vector<uint32_t> objs(emit.size()), at(emit.size(), RTX_NONE);
			for (size_t i = 0; i < emit.size(); i++)
				objs[i] = emit[i].obj;
			uint32_t *d_objs = nullptr, *d_at = nullptr;
			if ((rc = upload(d_objs, objs, c->stream)) || (rc = upload(d_at, at, c->stream))) {
				dfree(d_objs);
				return rc;
			}
			e = rtx_launch_find_prims((const DPrim *)(recs + nnodes), nb, d_objs, (uint32_t)objs.size(), d_at, c->stream);
			if (e == hipSuccess)
				e = hipMemcpyAsync(at.data(), d_at, at.size() * sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream);
			if (e == hipSuccess)
				e = hipStreamSynchronize(c->stream);
			dfree(d_objs);
			dfree(d_at);
			if (e != hipSuccess)
				return fail(RTX_ERR_HIP, "emitter record lookup failed: %s", hipGetErrorString(e));
			for (size_t i = 0; i < emit.size(); i++)
				emit[i].prim = at[i];
			PHASE(clk, "emitter records", c->stream);
		}
	} else {
		BvhOutput bvh;
		bvh_build(BvhInput{ nb, lo.data(), hi.data() }, cfg, bvh);
		std::vector<DPrim> prims(nb);
		for (uint32_t k = 0; k < nb; k++)
			prims[k] = make_prim(bounded[bvh.order[k]]);
		/* nodes and primitives in one array of 64-byte records: the shadow walk addresses both
		 * through one base pointer (record num_nodes + i = primitive i) */
		nnodes = (uint32_t)bvh.nodes.size();
		if (((uint64_t)nnodes + nb) * sizeof(DNode) > 0xFFFFFFC0ull)
			return fail(RTX_ERR_SCENE, "scene too large: %u BVH nodes + %u primitives exceed 4 GB of records", nnodes,
				    nb);
		/* builder refs (node index | RTX_LEAF_BIT leaf) -> device refs (record byte offset | leaf bits) */
		auto dref = [nnodes, &prims, &is_sphere](uint32_t r) -> uint32_t {
			if (r == RTX_EMPTY_REF)
				return r;
			if (r & RTX_LEAF_BIT) {
				const uint32_t first = (r >> 4) & 0x7FFFFFFu, cnt = (r & 15u) + 1;
				uint32_t sph = 0;
				for (uint32_t k = first; k < first + cnt; k++)
					if (is_sphere(prims[k]))
						sph = RTX_REF_SPH;
				return (nnodes + first) * (uint32_t)sizeof(DNode) | RTX_REF_LEAF | sph | (cnt - 1);
			}
			return r * (uint32_t)sizeof(DNode);
		};
		std::vector<DNode> recs(nnodes + (size_t)nb);
		for (uint32_t i = 0; i < nnodes; i++) {
			recs[i] = bvh.nodes[i];
			recs[i].ref0 = dref(recs[i].ref0);
			recs[i].ref1 = dref(recs[i].ref1);
		}
		if (nb)
			memcpy(recs.data() + nnodes, prims.data(), nb * sizeof(DPrim));
		/* the emitters' record indices (the 8-wide closest-hit walk tests them apart from the tree) */
		{
			std::vector<uint32_t> rec_of(sc->num_objects, RTX_NONE);
			for (uint32_t k = 0; k < nb; k++)
				rec_of[bounded[bvh.order[k]]] = k;
			for (DEmitter &e : emit)
				e.prim = rec_of[e.obj];
		}
		root_ref = dref(bvh.root_ref);
		depth = bvh.depth;
		inner.assign(recs.begin(), recs.begin() + nnodes);
		hs.recs = std::move(recs);
		host_prims = (const DPrim *)(hs.recs.data() + nnodes);
	}
	/* the shadow walk's BVH (RTX_OPT_SHADOW_WALK): the 8-wide compressed tree by default, which
	 * walks any depth (collapsed on the device above, else here from the host records); the
	 * threaded BVH2 for small scenes (its top levels in LDS), for measurement, and when the 8-wide
	 * tree cannot be built (over 2^24 entries) */
	if (!hs.w8_on_device && want_w8) {
		/* with the host records the emitters are left out of the tree (k_shadow tests them linearly) */
		std::vector<uint32_t> emit_objs;
		for (const DEmitter &e : emit)
			emit_objs.push_back(e.obj);
		hs.w8depth = rtx_wide8_build(inner, nnodes, host_prims, root_ref, tlo, thi, emit_objs, tf, hs.frame_pad, hs.w8f,
					     hs.w8noemit, hs.w8, hs.w8leaf);
	}
	if (hs.w8.empty() && !hs.w8_on_device)
		hs.w8depth = 0;
	/* does the 8-wide tree hold spheres?  (the emitters it leaves out do not count) */
	if (hs.w8depth) {
		std::vector<char> is_emit(sc->num_objects, 0);
		for (const DEmitter &e : emit)
			is_emit[e.obj] = 1;
		hs.w8sph = false;
		for (uint32_t k = 0; k < nb && !hs.w8sph; k++)
			hs.w8sph = sc->objects[bounded[k]].type == RTX_SPHERE && !(hs.w8noemit && is_emit[bounded[k]]);
	}
	if (linear) {
		for (uint32_t k = 0; k < nb; k++) {
			const rtx_object &o = sc->objects[bounded[k]];
			DEmitter e;
			memset(&e, 0, sizeof(e));
			e.obj = bounded[k];
			e.type = (uint32_t)o.type;
			memcpy(e.p0, o.p0, 12);
			memcpy(e.p1, o.p1, 12);
			memcpy(e.p2, o.p2, 12);
			e.radius = o.radius;
			memcpy(e.e1, o.e1, 12);
			memcpy(e.e2, o.e2, 12);
			e.eps = o.epsilon;
			e.transparent = (mats[o.material].flags & RTX_MF_TRANSPARENT) ? 1u : 0u;
			memcpy(e.kt, mats[o.material].kt, 12);
			e.prim = RTX_NONE;
			rtx_world_box(o, e.wlo, e.whi);
			hs.lin.push_back(e);
		}
	} else if (!hs.w8depth) {
		std::vector<uint32_t> qdepth;
		thread_bvh(inner, nb ? root_ref : RTX_EMPTY_REF, tlo, thi, hs.qnodes, hs.qf, qdepth);
		if (hs.qnodes.size() >= (1u << 26))
			return fail(RTX_ERR_SCENE, "scene too large: %zu threaded BVH nodes (max 2^26)", hs.qnodes.size());
		hs.ntop = thread_top(hs.qnodes, qdepth, hs.qtop);
	}
	PHASE(clk, "host trees", c->stream);
	hs.build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tb0).count();
	hs.mats = std::move(mats);
	hs.planes = std::move(planes);
	hs.emit = std::move(emit);
	hs.nnodes = nnodes;
	hs.nb = nb;
	hs.root_ref = nb ? root_ref : RTX_EMPTY_REF;
	hs.depth = depth;
	memcpy(hs.bound_lo, c->bound_lo, 12);
	memcpy(hs.bound_hi, c->bound_hi, 12);
	memcpy(hs.ambient, sc->ambient, 12);
	hs.num_emitters = sc->num_emitters;
	return RTX_OK;
}

/* the built scene onto c's device (c->d_nodes already holds the records when the device
 * builder ran on c, or a group copied them to it); device buffers in hs (the 8-wide tree
 * collapsed on the device) change hands to c */
int rtx_upload_built(rtx_ctx *c, HostScene &hs)
{
	DevTree t{ hs.dev_w8, hs.dev_w8s, hs.dev_w8leaf, hs.device };
	hs.dev_w8 = nullptr;
	hs.dev_w8s = nullptr;
	hs.dev_w8leaf = nullptr;
	const int rc = rtx_upload_built(c, hs, &t);
	/* whatever was not handed over goes back to hs, whose destructor frees it */
	hs.dev_w8 = t.w8;
	hs.dev_w8s = t.w8s;
	hs.dev_w8leaf = t.leaf;
	return rc;
}

/* k_shadow's cone cull (DScene.cull, RTX_OPT_SHADOW_CULL): the bounding spheres of the 8-wide
 * tree's second level in world coordinates, from the root entry and its child nodes read back from
 * the device.  Every primitive of the tree lies in one of these boxes (a root slot's children, or
 * the root slot itself when it is a leaf); the spheres are formed in double from the quantised
 * boxes (which contain the primitives' float boxes) and padded for the kernel's float test. */
static int build_cull(rtx_ctx *c, const HostScene &hs, uint32_t num_w8, uint32_t *n_out)
{
	*n_out = 0;
	if (!c->d_w8 || num_w8 < 2)
		return RTX_OK;
	DW8 root, kid[8];
	HIP_TRY(hipMemcpyAsync(&root, c->d_w8, sizeof(DW8), hipMemcpyDeviceToHost, c->stream));
	HIP_TRY(hipStreamSynchronize(c->stream));
	const uint32_t base = root.w[2] >> 8, imask = root.w[2] & 0xFFu, vmask = root.w[3] & 0xFFu;
	if (!vmask)
		return RTX_OK;
	if ((uint64_t)base + 8 > num_w8)
		return fail(RTX_ERR_STATE, "8-wide root's children at %u beyond %u entries", base, num_w8);
	HIP_TRY(hipMemcpyAsync(kid, c->d_w8 + base, sizeof(kid), hipMemcpyDeviceToHost, c->stream));
	HIP_TRY(hipStreamSynchronize(c->stream));
	std::vector<float4> sph;
	auto add_box = [&](const DW8 &N, int slot) {
		const double org[3] = { (double)(N.w[0] & 0xFFFFu), (double)(N.w[0] >> 16), (double)(N.w[1] & 0xFFFFu) };
		const int ex[3] = { (int)((N.w[1] >> 16) & 15u), (int)((N.w[1] >> 20) & 15u), (int)((N.w[1] >> 24) & 15u) };
		double ctr[3], r2 = 0;
		for (int a = 0; a < 3; a++) {
			const uint32_t lo8 = (N.w[4 + 4 * a + (slot >> 2)] >> (8 * (slot & 3))) & 0xFFu;
			const uint32_t hi8 = (N.w[6 + 4 * a + (slot >> 2)] >> (8 * (slot & 3))) & 0xFFu;
			const double lo = (org[a] + std::ldexp((double)lo8, ex[a])) / (double)hs.w8f.qs[a] + (double)hs.w8f.qo[a];
			const double hi = (org[a] + std::ldexp((double)hi8, ex[a])) / (double)hs.w8f.qs[a] + (double)hs.w8f.qo[a];
			ctr[a] = 0.5 * (lo + hi);
			r2 += 0.25 * (hi - lo) * (hi - lo);
		}
		double w[3], m = 0;
		for (int a = 0; a < 3; a++) /* the frame's x' = R (x - c): x = R^T x' + c */
			w[a] = hs.tf.rotated ? (double)hs.tf.c[a] + hs.tf.r[0][a] * ctr[0] + hs.tf.r[1][a] * ctr[1] + hs.tf.r[2][a] * ctr[2]
					      : ctr[a];
		for (int a = 0; a < 3; a++)
			m = std::max(m, std::fabs(w[a]));
		const double r = std::sqrt(r2);
		sph.push_back(make_float4((float)w[0], (float)w[1], (float)w[2], (float)(r * (1 + 1e-5) + 1e-5 * m + 1e-6)));
	};
	for (int s = 0; s < 8; s++) {
		if (!((vmask >> s) & 1u))
			continue;
		if ((imask >> s) & 1u) {
			const DW8 &K = kid[s];
			for (int s2 = 0; s2 < 8; s2++)
				if ((K.w[3] >> s2) & 1u)
					add_box(K, s2);
		} else {
			add_box(root, s);
		}
	}
	if (sph.empty() || sph.size() > RTX_CULL_MAX)
		return RTX_OK;
	int rc = upload(c->d_cull, sph, c->stream);
	if (rc)
		return rc;
	*n_out = (uint32_t)sph.size();
	return RTX_OK;
}

int rtx_upload_built(rtx_ctx *c, const HostScene &hs, DevTree *take)
{
	int rc;
	PhaseClock clk;
	/* a failure below leaves the context without a scene (RTX_ERR_STATE on render), never with a
	 * mix of old and new buffers */
	c->have_scene = false;
	c->sp_tile_seen = 0.0; /* the next render sizes its chunks from the static bound */
	c->sp_tile_key = SpKey{};
	HIP_TRY(hipSetDevice(c->device));
	if (!(hs.recs_on_device && c->d_nodes) && (rc = upload(c->d_nodes, hs.recs, c->stream)))
		return rc;
	PHASE(clk, "upload: set device", c->stream);
	if ((rc = upload(c->d_qnodes, hs.qnodes, c->stream)) || (rc = upload(c->d_top, hs.qtop, c->stream)))
		return rc;
	PHASE(clk, "upload threaded BVH2", c->stream);
	if ((rc = upload(c->d_planes, hs.planes, c->stream)))
		return rc;
	PHASE(clk, "upload planes", c->stream);
	if ((rc = upload(c->d_mats, hs.mats, c->stream)) || (rc = upload(c->d_emitters, hs.emit, c->stream)) || (rc = upload(c->d_lin, hs.lin, c->stream)))
		return rc;
	PHASE(clk, "upload scene tables", c->stream);
	const bool have_w8 = hs.w8_on_device || !hs.w8.empty();
	const uint32_t num_w8 = hs.w8_on_device ? hs.w8_entries : (uint32_t)hs.w8.size();
	uint32_t *d_map = nullptr; /* entry -> primitive index of the 8-wide tree's leaf entries */
	if (hs.w8_on_device) { /* collapsed on the device (or peer-copied to it): the buffers change hands */
		if (!take || take->device != c->device)
			return fail(RTX_ERR_STATE, "8-wide tree on device %d uploaded to device %d", take ? take->device : -1, c->device);
		dfree(c->d_w8);
		dfree(c->d_w8s);
		c->d_w8 = take->w8;
		c->d_w8s = take->w8s;
		d_map = take->leaf;
		take->w8 = nullptr;
		take->w8s = nullptr;
		take->leaf = nullptr;
		PHASE(clk, "8-wide tree handover", c->stream);
	} else {
		if ((rc = upload(c->d_w8, hs.w8, c->stream)))
			return rc;
		if ((rc = upload(d_map, hs.w8leaf, c->stream)))
			return rc;
		dfree(c->d_w8s);
		/* the scalar-path node copies (rtx_device.h DW8S) */
		hipError_t e = hipMalloc(&c->d_w8s, std::max<size_t>(num_w8, 1) * sizeof(DW8S));
		if (e == hipSuccess)
			e = rtx_launch_w8_scalar(num_w8, c->d_w8, d_map, c->d_w8s, c->stream);
		if (e != hipSuccess) {
			dfree(d_map);
			return fail(RTX_ERR_HIP, "8-wide BVH scalar copies failed: %s", hipGetErrorString(e));
		}
	}
	PHASE(clk, "upload host parts", c->stream);
	if (have_w8) { /* the 8-wide tree's leaf entries: copies of their primitive records */
		hipError_t e = rtx_launch_w8_fill((const DPrim *)(c->d_nodes + hs.nnodes), c->d_mats, d_map, num_w8, c->d_w8, c->stream);
		if (e == hipSuccess)
			e = hipStreamSynchronize(c->stream);
		dfree(d_map);
		if (e != hipSuccess)
			return fail(RTX_ERR_HIP, "8-wide BVH leaf fill failed: %s", hipGetErrorString(e));
	}
	dfree(d_map);
	PHASE(clk, "8-wide leaf fill", c->stream);
	uint32_t ncull = 0; /* the cone cull needs the emitters out of the tree (else a light's own leaf meets every cone) */
	if (have_w8 && hs.w8noemit && hs.lin.empty() && (rc = build_cull(c, hs, num_w8, &ncull)))
		return rc;
	memcpy(c->bound_lo, hs.bound_lo, 12);
	memcpy(c->bound_hi, hs.bound_hi, 12);
	DScene &S = c->scene;
	memset(&S, 0, sizeof(S));
	S.nodes = c->d_nodes;
	S.num_nodes = hs.nnodes;
	S.prims = (const DPrim *)(c->d_nodes + hs.nnodes);
	S.planes = c->d_planes;
	S.mats = c->d_mats;
	S.emitters = c->d_emitters;
	S.lin = hs.lin.empty() ? nullptr : c->d_lin;
	S.num_lin = (uint32_t)hs.lin.size();
	S.qnodes = hs.qnodes.empty() ? nullptr : c->d_qnodes;
	S.num_qnodes = (uint32_t)hs.qnodes.size();
	memcpy(S.qo, hs.qf.qo, 12);
	memcpy(S.qs, hs.qf.qs, 12);
	S.top = hs.ntop ? c->d_top : nullptr;
	S.num_top = hs.ntop;
	S.w8 = have_w8 ? c->d_w8 : nullptr;
	S.num_w8 = num_w8;
	S.w8depth = hs.w8depth;
	S.w8top = hs.w8_on_device ? hs.w8top : 0u; /* the device collapse's breadth-first layout only */
	memcpy(S.w8qo, hs.w8f.qo, 12);
	memcpy(S.w8qs, hs.w8f.qs, 12);
	S.w8noemit = hs.w8noemit ? 1u : 0u;
	S.w8sph = hs.w8sph ? 1u : 0u;
	S.w8s = have_w8 ? c->d_w8s : nullptr;
	S.root_ref = hs.root_ref;
	S.num_prims = hs.nb;
	S.num_planes = (uint32_t)hs.planes.size();
	S.num_emitters = hs.num_emitters;
	S.stack_size = std::max<uint32_t>(hs.depth + 1, 4);
	S.tf = hs.tf;
	S.cull = ncull ? (const float *)c->d_cull : nullptr;
	S.num_cull = ncull;
	c->total_lights = 0;
	for (const DEmitter &e : hs.emit)
		c->total_lights += e.num_lights;
	memcpy(S.ambient, hs.ambient, 12);
	c->have_scene = true;
	c->stats.build_ms = hs.build_ms;
	c->stats.bvh_nodes = hs.nnodes;
	c->stats.bvh_depth = hs.depth;
	c->stats.builder = (uint32_t)hs.builder;
	c->stats.bvh_prims = hs.nb;
	c->stats.shadow_walk = S.lin ? RTX_WALK_LINEAR : S.w8 ? RTX_WALK_W8 : RTX_WALK_BVH2;
	c->stats.tree_rotated = hs.tf.rotated;
	c->stats.frame_cost = hs.frame_ratio;
	c->stats.frame_ms = hs.frame_ms;
	if (S.w8) {
		uint32_t inner_nodes = hs.w8_wide;
		if (!hs.w8_on_device)
			for (const DW8 &e : hs.w8)
				inner_nodes += e.w[3] != 0;
		c->stats.wide_nodes = inner_nodes;
		c->stats.wide_depth = S.w8depth;
		c->stats.wide_entries = S.num_w8;
	} else {
		c->stats.wide_nodes = 0;
		c->stats.wide_depth = 0;
		c->stats.wide_entries = 0;
	}
	return RTX_OK;
}

extern "C" int rtx_upload_scene(rtx_ctx *c, const rtx_scene_desc *sc)
{
	if (!c || !sc)
		return fail(RTX_ERR_ARG, "null argument");
	HostScene hs;
	int rc = rtx_build_scene(c, sc, hs);
	if (rc)
		return rc;
	return rtx_upload_built(c, hs);
}

int rtx_render_common(rtx_ctx *c, const rtx_frame *fr, const rtx_params *p, float *d_rgb, float *d_z,
			 hipStream_t stream)
{
	if (!c->have_scene)
		return fail(RTX_ERR_STATE, "rtx_render before rtx_upload_scene");
	if (!fr || !p)
		return fail(RTX_ERR_ARG, "null frame/params");
	if (!fr->width || !fr->height)
		return fail(RTX_ERR_ARG, "empty frame %ux%u", fr->width, fr->height);
	if (!p->tile_stride || p->tile_offset >= p->tile_stride)
		return fail(RTX_ERR_ARG, "bad tile sharding %u/%u", p->tile_offset, p->tile_stride);
	DFrame F;
	F.width = fr->width;
	F.height = fr->height;
	memcpy(F.corner, fr->corner, 12);
	memcpy(F.step_x, fr->step_x, 12);
	memcpy(F.step_y, fr->step_y, 12);
	memcpy(F.origin, fr->origin, 12);
	DParams P;
	memset(&P, 0, sizeof(P));
	P.max_bounces = p->max_bounces;
	P.min_intensity_sqr = p->min_intensity_sqr;
	P.reflection = p->reflection;
	P.gi = p->gi;
	P.samples = p->samples;
	P.attenuation = p->attenuation;
	P.att_offset = p->attenuation_offset;
	P.rng = p->rng;
	P.seed = p->seed;
	P.u32conv = p->u32conv;
	P.tile_offset = p->tile_offset;
	P.tile_stride = p->tile_stride;
	P.tiles_x = (fr->width + RTX_TILE_W - 1) / RTX_TILE_W;
	const uint64_t tiles_y = (fr->height + RTX_TILE_H - 1) / RTX_TILE_H;
	const uint64_t total = (uint64_t)P.tiles_x * tiles_y;
	P.ntiles = p->tile_offset < total ? (uint32_t)((total - p->tile_offset + p->tile_stride - 1) / p->tile_stride) : 0;

	int per_cu = 0;
	HIP_TRY(rtx_trace_occupancy(c->scene.stack_size, &per_cu));
	if (per_cu <= 0)
		return fail(RTX_ERR_HIP, "trace kernel does not fit (LDS %zu B)", rtx_trace_lds_bytes(c->scene.stack_size));
	const uint32_t waves = (uint32_t)std::min<uint64_t>((uint64_t)per_cu * c->cus, std::max<uint32_t>(P.ntiles, 1));
	/* LIFO task stack: each batch pops <= 64 and pushes <= 128, depth <= max_bounces */
	if (P.max_bounces > RTX_MAX_BOUNCES)
		return fail(RTX_ERR_ARG, "max_bounces %u above the supported %u", P.max_bounces, RTX_MAX_BOUNCES);
	const uint32_t mb = P.max_bounces;
	const uint32_t task_cap = 64u * (mb + 3u);
	/* shade points per tile: 64 px x (primary + GI samples) + secondary-ray allowance */
	const uint64_t gi_n = P.gi == RTX_GI_PATH ? (uint64_t)P.samples : 0u;
	uint64_t staging_cap = 64ull * (1 + gi_n) + 64ull * 4 * std::min<uint32_t>(mb, 16u) * (gi_n ? 2 : 1) + 64;
	uint64_t avg_tile = 64ull * (1 + gi_n) * 5 / 4 + 64;
	/* a render of the same scene and settings before: its shade points per tile (x 1.25, + 64)
	 * instead of the bound above; an overflow still halves the chunk and retries */
	/* every setting the shade points per tile depend on: the scene (reset by an upload), the
	 * frame and camera, the ray-tree and GI settings and the shard */
	SpKey sp_key{};
	sp_key.v[0] = (uint32_t)P.gi;
	sp_key.v[1] = P.samples;
	sp_key.v[2] = P.max_bounces;
	sp_key.v[3] = (uint32_t)P.reflection;
	sp_key.v[4] = P.tile_offset;
	sp_key.v[5] = P.tile_stride;
	sp_key.v[6] = F.width;
	sp_key.v[7] = F.height;
	memcpy(&sp_key.v[8], &P.min_intensity_sqr, 4);
	memcpy(&sp_key.v[9], F.corner, 12);
	memcpy(&sp_key.v[12], F.step_x, 12);
	memcpy(&sp_key.v[15], F.step_y, 12);
	memcpy(&sp_key.v[18], F.origin, 12);
	sp_key.set = 1;
	if (c->sp_tile_key == sp_key && c->sp_tile_seen > 0.0)
		avg_tile = std::min<uint64_t>(avg_tile, (uint64_t)(c->sp_tile_seen * 1.25) + 64);
	if (c->opt_sp_tile) /* RTX_OPT_SP_PER_TILE: tests drive the overflow path with a low figure */
		avg_tile = c->opt_sp_tile;
	size_t free_b = 0, total_b = 0;
	HIP_TRY(hipMemGetInfo(&free_b, &total_b));
	/* shade points of a chunk: up to a third of free HBM (96 GB cap; 288 GB per MI355X), shared
	 * out among the contexts rendering on this device at once (rtx_group_open_loopback) */
	const uint64_t budget = std::min<uint64_t>(96ull << 30, free_b / 3) / std::max<uint32_t>(c->mem_share, 1u);
	/* 128 B per shade point: its record (96), its light term (16) and its sort keys / values (16) */
	uint32_t chunk_cap = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(P.ntiles, budget / (avg_tile * 128)));
	if (c->opt_chunk) /* RTX_OPT_CHUNK_TILES */
		chunk_cap = std::min(chunk_cap, c->opt_chunk);
	uint32_t chunk_tiles = chunk_cap;

	auto grow = [](auto *&ptr, size_t &have, size_t need) -> hipError_t {
		if (need <= have)
			return hipSuccess;
		dfree(ptr);
		have = 0;
		hipError_t e = hipMalloc(&ptr, need);
		if (e == hipSuccess)
			have = need;
		return e;
	};
	HIP_TRY(grow(c->d_tasks, c->task_bytes, (size_t)waves * task_cap * sizeof(DTask)));
	if (c->scene.stack_size > RTX_TRACE_LSTK) /* the closest-hit stack entries beyond the LDS part */
		HIP_TRY(grow(c->d_ostk, c->ostk_bytes,
			     (size_t)waves * 64 * (c->scene.stack_size - RTX_TRACE_LSTK) * sizeof(uint32_t)));
	c->scene.ostk = c->d_ostk;
	c->scene.w8spill = nullptr;
	c->scene.w8spill_lanes = 0;
	c->scene.trace_w8 = (c->scene.w8 && c->opt_trace_walk != RTX_WALK_BVH2) ? 1u : 0u;
	c->stats.trace_walk = c->scene.trace_w8 ? RTX_WALK_W8 : RTX_WALK_BVH2;
	c->scene.w8lstk = c->opt_lstk;
	if (c->scene.w8 && c->scene.w8depth > c->scene.w8lstk + 1) {
		/* 8-wide trees deeper than the LDS lane stacks: the deeper entries of every lane of the
		 * largest k_shadow grid (one group per level at most) */
		uint32_t lanes = 0;
		HIP_TRY(rtx_shadow_grid_lanes((uint32_t)c->cus, &lanes));
		HIP_TRY(grow(c->d_w8spill, c->w8spill_bytes,
			     (size_t)lanes * (c->scene.w8depth - 1 - c->scene.w8lstk) * sizeof(uint32_t)));
		c->scene.w8spill = c->d_w8spill;
		c->scene.w8spill_lanes = lanes;
	}

	HIP_TRY(hipEventRecord(c->ev0, stream));
	double t_trace = 0, t_sort = 0, t_shadow = 0, t_accum = 0;
	uint64_t shade_points = 0;
	uint32_t chunks = 0;
	unsigned long long tot[RTX_C_N] = {}; /* counters of the chunks that completed */
	/* shadow kernel: lane slots of slot_b = pow2ceil(lights) (<= 64) lanes per point; ~16 packets per wave */
	uint32_t slot_b = 1;
	while (slot_b < 64 && slot_b < c->total_lights)
		slot_b <<= 1;
	{
		/* a point's lanes in slots of pow2ceil(lights) (one point per 64-lane packet from 64 lights
		 * up) leave lanes idle when the count is awkward (100 lights: 64 + 36 of 128 lanes); below
		 * 90 % use, points take consecutive 4-lane slots and straddle packets instead (k_shadow
		 * sums a point's slots in slot order, so the result does not depend on its neighbours) */
		const uint32_t n = std::max<uint32_t>(c->total_lights, 1);
		const uint32_t used = slot_b * ((n + slot_b - 1) / slot_b);
		if (n > 4 && (double)n / used < 0.9)
			slot_b = 4;
	}
	if (c->opt_slot) /* RTX_OPT_SHADOW_SLOT */
		slot_b = c->opt_slot;
	const uint32_t slots_per_point = (std::max<uint32_t>(c->total_lights, 1) + slot_b - 1) / slot_b;
	const uint32_t grab = c->opt_grab; /* lane slots per k_shadow queue grab (1024 -> 4096: 903 -> 885 ms) */
	const uint32_t per_wave = std::max<uint32_t>(1, std::min<uint32_t>(64, grab / (slot_b * slots_per_point)));
	const bool spsort = c->opt_spsort;
	bool overflowed = false; /* a chunk of this frame overflowed the shade-point array */
	for (uint32_t begin = 0; begin < P.ntiles;) {
		const uint32_t end = std::min<uint32_t>(P.ntiles, begin + chunk_tiles);
		const uint64_t sp_cap64 = std::min<uint64_t>((uint64_t)(end - begin) * avg_tile + staging_cap, 0xFFFFFFF0ull);
		const uint32_t sp_cap = (uint32_t)sp_cap64;
		HIP_TRY(grow(c->d_staging, c->staging_bytes, (size_t)waves * staging_cap * 6 * sizeof(float4)));
		HIP_TRY(grow(c->d_sp, c->sp_bytes, (size_t)sp_cap * 6 * sizeof(float4)));
		HIP_TRY(grow(c->d_contrib, c->contrib_bytes, (size_t)sp_cap * sizeof(float4)));
		HIP_TRY(grow(c->d_tile_rec, c->tile_rec_bytes, (size_t)(end - begin) * sizeof(uint2)));
		HIP_TRY(hipMemsetAsync(c->d_ctr, 0, sizeof(unsigned long long) * RTX_C_N, stream));
		HIP_TRY(hipEventRecord(c->ev[0], stream));
		HIP_TRY(rtx_launch_trace(&c->scene, &F, &P, d_rgb, d_z, c->d_tasks, task_cap, c->d_staging,
					 (uint32_t)staging_cap, c->d_sp, sp_cap, c->d_tile_rec, begin, end, c->d_ctr,
					 std::min<uint32_t>(waves, end - begin), p->count_traversal, stream));
		HIP_TRY(hipEventRecord(c->ev[1], stream));
		unsigned long long head[RTX_C_N];
		HIP_TRY(hipMemcpyAsync(head, c->d_ctr, sizeof(head), hipMemcpyDeviceToHost, stream));
		HIP_TRY(hipStreamSynchronize(stream));
		if (head[RTX_C_TASKOVERFLOW])
			return fail(RTX_ERR_STATE, "reflection/refraction task stack overflow (%u entries per wave)", task_cap);
		if (head[RTX_C_OVERFLOW]) {
			if (staging_cap >= (1ull << 26))
				return fail(RTX_ERR_STATE, "shade-point staging overflow (%llu shade points per tile)",
					    (unsigned long long)staging_cap);
			staging_cap *= 2; /* retry the chunk (counters reset) with room for larger ray trees */
			continue;
		}
		if (head[RTX_C_SPOVERFLOW]) {
			if (end - begin == 1)
				return fail(RTX_ERR_STATE, "shade-point array overflow on a single tile");
			chunk_tiles = std::max<uint32_t>(1, (end - begin) / 2);
			overflowed = true;
			continue;
		}
		const uint32_t n_sp = (uint32_t)head[RTX_C_SPCOUNT];
		shade_points += n_sp;
		/* shade points in Morton order of their position (rtx_sort.hip); RTX_SPSORT=0 keeps
		 * emission order (same image, bit for bit) */
		const uint32_t *perm = nullptr;
		if (n_sp > 1 && c->scene.root_ref != RTX_EMPTY_REF && spsort) {
			/* keys and values (two ping-pong buffers each) sized for the chunk's capacity, like the
			 * shade-point array: a later render with more points per chunk (its chunks sized from
			 * this one's count) then reuses them instead of reallocating inside its frame */
			size_t tmp = 0;
			const size_t cap = std::max<size_t>(n_sp, c->sp_bytes / (6 * sizeof(float4)));
			HIP_TRY(rtx_spsort_temp_bytes((uint32_t)std::min<size_t>(cap, 0xFFFFFFF0u), &tmp));
			HIP_TRY(grow(c->d_sortbuf, c->sortbuf_bytes, cap * 4 * sizeof(uint32_t)));
			HIP_TRY(grow(c->d_sorttmp, c->sorttmp_bytes, tmp));
			const size_t q = c->sortbuf_bytes / (4 * sizeof(uint32_t)); /* the buffer's capacity in points */
			uint32_t *b = c->d_sortbuf;
			HIP_TRY(rtx_launch_spsort(c->d_sp, n_sp, c->bound_lo, c->bound_hi, b, b + q, b + 2 * q, b + 3 * q, c->d_sorttmp,
						  c->sorttmp_bytes, &perm, stream));
		}
		HIP_TRY(hipEventRecord(c->ev[4], stream));
		DScene Ssh = c->scene; /* RTX_OPT_SHADOW_CULL: 0 no cull spheres, 2 the lane slots cull too */
		if (!c->opt_cull)
			Ssh.num_cull = 0;
		Ssh.cull_slots = c->opt_cull == 2 ? 1u : 0u;
		HIP_TRY(rtx_launch_shadow(&Ssh, &P, c->d_sp, perm, n_sp, per_wave, slot_b, c->d_contrib, c->d_ctr,
					  p->count_traversal, (uint32_t)c->cus, stream));
		HIP_TRY(hipEventRecord(c->ev[2], stream));
		HIP_TRY(rtx_launch_accum(&F, &P, c->d_tile_rec, c->d_contrib, begin, end - begin, d_rgb, stream));
		HIP_TRY(hipEventRecord(c->ev[3], stream));
		unsigned long long ctr[RTX_C_N];
		HIP_TRY(hipMemcpyAsync(ctr, c->d_ctr, sizeof(ctr), hipMemcpyDeviceToHost, stream));
		HIP_TRY(hipStreamSynchronize(stream));
		for (int k = RTX_C_CLOSEST; k < RTX_C_N; k++)
			tot[k] += ctr[k];
		float a = 0, b = 0, cc = 0, so = 0;
		HIP_TRY(hipEventElapsedTime(&a, c->ev[0], c->ev[1]));
		HIP_TRY(hipEventElapsedTime(&so, c->ev[1], c->ev[4]));
		HIP_TRY(hipEventElapsedTime(&b, c->ev[4], c->ev[2]));
		HIP_TRY(hipEventElapsedTime(&cc, c->ev[2], c->ev[3]));
		t_trace += a;
		t_sort += so;
		t_shadow += b;
		t_accum += cc;
		chunks++;
		begin = end;
		/* a chunk an overflow halved grows back by a quarter per chunk that fits, so a dense region of
		 * the image does not overflow (and re-trace) every other chunk */
		if (overflowed)
			chunk_tiles = std::min<uint32_t>(chunk_cap, chunk_tiles + std::max<uint32_t>(1, chunk_tiles / 4));
	}
	HIP_TRY(hipEventRecord(c->ev1, stream));
	HIP_TRY(hipStreamSynchronize(stream));
	if (P.ntiles) {
		c->sp_tile_seen = (double)shade_points / P.ntiles;
		c->sp_tile_key = sp_key;
	}
	const unsigned long long *ctr = tot;
	rtx_stats &st = c->stats;
	st.closest_rays = ctr[RTX_C_CLOSEST];
	st.shadow_rays = ctr[RTX_C_SHADOW];
	/* the threaded walk counts box tests; a node visit is a BVH2 inner node (two box tests) */
	st.shadow_node_visits = ctr[RTX_C_SBOXES] / 2;
	st.shadow_tri_tests = ctr[RTX_C_STRIS];
	st.shadow_sphere_tests = ctr[RTX_C_SSPHERES];
	st.shadow_plane_tests = ctr[RTX_C_SPLANES];
	st.shadow_box_tests = ctr[RTX_C_SBOXES];
	st.shadow_global_box_tests = ctr[RTX_C_SGBOXES];
	st.shadow_wave_steps = ctr[RTX_C_SSTEPS];
	st.shadow_wave_walks = ctr[RTX_C_SWALKS];
	st.shadow_leaf_rounds = ctr[RTX_C_SLEAFR];
	st.shadow_uniform_steps = ctr[RTX_C_SUNIF];
	st.far_closest_rays = ctr[RTX_C_FARC];
	st.far_shadow_rays = ctr[RTX_C_FARS];
	st.shadow_stack_spills = ctr[RTX_C_SSPILL];
	st.shadow_cone_clear = ctr[RTX_C_SCLEAR];
	st.node_visits = ctr[RTX_C_NODES] + st.shadow_node_visits;
	st.tri_tests = ctr[RTX_C_TRIS] + ctr[RTX_C_STRIS];
	st.sphere_tests = ctr[RTX_C_SPHERES] + ctr[RTX_C_SSPHERES];
	st.plane_tests = ctr[RTX_C_PLANES] + ctr[RTX_C_SPLANES];
	st.shade_points = shade_points;
	st.kernel_ms = t_trace + t_sort + t_shadow + t_accum;
	st.sort_ms = t_sort;
	st.trace_ms = t_trace;
	st.shadow_ms = t_shadow;
	st.accum_ms = t_accum;
	st.waves = waves;
	st.chunks = chunks;
	return RTX_OK;
}

extern "C" int rtx_render_device(rtx_ctx *c, const rtx_frame *fr, const rtx_params *p, void *d_rgb, void *d_z,
				 void *stream)
{
	if (!c)
		return fail(RTX_ERR_ARG, "null context");
	HIP_TRY(hipSetDevice(c->device));
	return rtx_render_common(c, fr, p, (float *)d_rgb, (float *)d_z, stream ? (hipStream_t)stream : c->stream);
}

extern "C" int rtx_render(rtx_ctx *c, const rtx_frame *fr, const rtx_params *p, float *rgb, float *z)
{
	if (!c || !fr || !p)
		return fail(RTX_ERR_ARG, "null argument");
	HIP_TRY(hipSetDevice(c->device));
	const size_t px = (size_t)fr->width * fr->height;
	if (px > c->fb_pixels) {
		dfree(c->d_rgb);
		dfree(c->d_z);
		HIP_TRY(hipMalloc(&c->d_rgb, px * 3 * sizeof(float)));
		HIP_TRY(hipMalloc(&c->d_z, px * sizeof(float)));
		c->fb_pixels = px;
	}
	/* pixels of tiles outside this shard keep the caller's values */
	if (p->tile_stride > 1) {
		if (rgb)
			HIP_TRY(hipMemcpyAsync(c->d_rgb, rgb, px * 12, hipMemcpyHostToDevice, c->stream));
		if (z)
			HIP_TRY(hipMemcpyAsync(c->d_z, z, px * 4, hipMemcpyHostToDevice, c->stream));
	}
	int rc = rtx_render_common(c, fr, p, rgb ? c->d_rgb : nullptr, z ? c->d_z : nullptr, c->stream);
	if (rc)
		return rc;
	if (rgb)
		HIP_TRY(hipMemcpy(rgb, c->d_rgb, px * 12, hipMemcpyDeviceToHost));
	if (z)
		HIP_TRY(hipMemcpy(z, c->d_z, px * 4, hipMemcpyDeviceToHost));
	return RTX_OK;
}

static int post_common(rtx_ctx *c, uint32_t w, uint32_t h, const rtx_post *pp, float *d_rgb, const float *d_z,
		       hipStream_t stream)
{
	if (!w || !h || (uint64_t)w * h > 0xFFFFFFFFull)
		return fail(RTX_ERR_ARG, "bad postprocess size %ux%u", w, h);
	if (pp->mist && (pp->mist_falloff < RTX_FALLOFF_QUAD || pp->mist_falloff > RTX_FALLOFF_INV_QUAD))
		return fail(RTX_ERR_ARG, "bad mist falloff %d", pp->mist_falloff);
	if (pp->dof < RTX_DOF_NONE || pp->dof > RTX_DOF_CAMERA)
		return fail(RTX_ERR_ARG, "bad dof mode %d", pp->dof);
	const size_t n = (size_t)w * h;
	if (n > c->post_pixels) {
		dfree(c->d_post_rad);
		dfree(c->d_post_pv);
		c->post_pixels = 0;
		HIP_TRY(hipMalloc(&c->d_post_rad, n * sizeof(int)));
		HIP_TRY(hipMalloc(&c->d_post_pv, n * sizeof(float4)));
		c->post_pixels = n;
	}
	if (!c->d_post_scratch)
		HIP_TRY(hipMalloc(&c->d_post_scratch, 4 * sizeof(unsigned)));
	HIP_TRY(rtx_launch_post(w, h, pp, d_rgb, d_z, c->d_post_rad, c->d_post_pv, c->d_post_scratch, stream));
	HIP_TRY(hipStreamSynchronize(stream));
	return RTX_OK;
}

extern "C" int rtx_postprocess_device(rtx_ctx *c, uint32_t w, uint32_t h, const rtx_post *pp, void *d_rgb,
				      const void *d_z, void *stream)
{
	if (!c || !pp || !d_rgb || !d_z)
		return fail(RTX_ERR_ARG, "null argument");
	HIP_TRY(hipSetDevice(c->device));
	return post_common(c, w, h, pp, (float *)d_rgb, (const float *)d_z,
			   stream ? (hipStream_t)stream : c->stream);
}

extern "C" int rtx_postprocess(rtx_ctx *c, uint32_t w, uint32_t h, const rtx_post *pp, float *rgb, const float *z)
{
	if (!c || !pp || !rgb || !z)
		return fail(RTX_ERR_ARG, "null argument");
	if (!w || !h)
		return fail(RTX_ERR_ARG, "bad postprocess size %ux%u", w, h);
	HIP_TRY(hipSetDevice(c->device));
	const size_t px = (size_t)w * h;
	if (px > c->fb_pixels) {
		dfree(c->d_rgb);
		dfree(c->d_z);
		c->fb_pixels = 0;
		HIP_TRY(hipMalloc(&c->d_rgb, px * 3 * sizeof(float)));
		HIP_TRY(hipMalloc(&c->d_z, px * sizeof(float)));
		c->fb_pixels = px;
	}
	HIP_TRY(hipMemcpyAsync(c->d_rgb, rgb, px * 12, hipMemcpyHostToDevice, c->stream));
	HIP_TRY(hipMemcpyAsync(c->d_z, z, px * 4, hipMemcpyHostToDevice, c->stream));
	int rc = post_common(c, w, h, pp, c->d_rgb, c->d_z, c->stream);
	if (rc)
		return rc;
	HIP_TRY(hipMemcpy(rgb, c->d_rgb, px * 12, hipMemcpyDeviceToHost));
	return RTX_OK;
}

extern "C" int rtx_set_builder(rtx_ctx *c, int builder)
{
	if (!c)
		return fail(RTX_ERR_ARG, "null argument");
	if (builder != RTX_BUILD_SAH_HOST && builder != RTX_BUILD_LBVH_GPU && builder != RTX_BUILD_PLOC_GPU &&
	    builder != RTX_BUILD_SAH_GPU)
		return fail(RTX_ERR_ARG, "unknown BVH builder %d", builder);
	c->builder = builder;
	return RTX_OK;
}

extern "C" int rtx_set_option(rtx_ctx *c, int option, int64_t value)
{
	if (!c)
		return fail(RTX_ERR_ARG, "null argument");
	switch (option) {
	case RTX_OPT_SHADOW_WALK:
		if (value != RTX_WALK_AUTO && value != RTX_WALK_BVH2 && value != RTX_WALK_W8 && value != RTX_WALK_LINEAR)
			return fail(RTX_ERR_ARG, "shadow walk %lld is not AUTO, BVH2, W8 or LINEAR", (long long)value);
		c->opt_walk = (int)value;
		return RTX_OK;
	case RTX_OPT_BVH_LEAF:
		if (value < 1 || value > RTX_MAX_LEAF)
			return fail(RTX_ERR_ARG, "BVH leaf size %lld outside 1..%d", (long long)value, RTX_MAX_LEAF);
		c->opt_leaf = (uint32_t)value;
		return RTX_OK;
	case RTX_OPT_SPSORT:
		if (value != 0 && value != 1)
			return fail(RTX_ERR_ARG, "RTX_OPT_SPSORT takes 0 or 1, not %lld", (long long)value);
		c->opt_spsort = value != 0;
		return RTX_OK;
	case RTX_OPT_SHADOW_SLOT:
		if (value < 0 || value > 64 || (value & (value - 1)))
			return fail(RTX_ERR_ARG, "shadow slot %lld is not 0 or a power of two <= 64", (long long)value);
		c->opt_slot = (uint32_t)value;
		return RTX_OK;
	case RTX_OPT_SHADOW_LDS_STACK:
		if (value < 1 || value > RTX_W8_STACK)
			return fail(RTX_ERR_ARG, "shadow LDS stack %lld outside 1..%d", (long long)value, RTX_W8_STACK);
		c->opt_lstk = (uint32_t)value;
		return RTX_OK;
	case RTX_OPT_TRACE_WALK:
		if (value != RTX_WALK_AUTO && value != RTX_WALK_W8 && value != RTX_WALK_BVH2)
			return fail(RTX_ERR_ARG, "closest-hit walk %lld is not AUTO, W8 or BVH2", (long long)value);
		c->opt_trace_walk = (int)value;
		return RTX_OK;
	case RTX_OPT_TREE_FRAME:
		if (value != RTX_FRAME_AUTO && value != RTX_FRAME_WORLD)
			return fail(RTX_ERR_ARG, "tree frame %lld is not AUTO or WORLD", (long long)value);
		c->opt_frame = (int)value;
		return RTX_OK;
	case RTX_OPT_SHADOW_GRAB:
		if (value < 1 || value > (1 << 24))
			return fail(RTX_ERR_ARG, "shadow grab %lld outside 1..2^24", (long long)value);
		c->opt_grab = (uint32_t)value;
		return RTX_OK;
	case RTX_OPT_CHUNK_TILES:
		if (value < 0 || value > 0xFFFFFFFFll)
			return fail(RTX_ERR_ARG, "chunk tiles %lld outside 0..2^32-1", (long long)value);
		c->opt_chunk = (uint32_t)value;
		return RTX_OK;
	case RTX_OPT_SP_PER_TILE:
		if (value < 0 || value > (1 << 20))
			return fail(RTX_ERR_ARG, "shade points per tile %lld outside 0..2^20", (long long)value);
		c->opt_sp_tile = (uint32_t)value;
		return RTX_OK;
	case RTX_OPT_SHADOW_CULL:
		if (value < 0 || value > 2)
			return fail(RTX_ERR_ARG, "shadow cull %lld is not 0, 1 or 2", (long long)value);
		c->opt_cull = (int)value;
		return RTX_OK;
	}
	return fail(RTX_ERR_ARG, "unknown option %d", option);
}

extern "C" int rtx_read_wide_tree(rtx_ctx *c, void *entries, uint32_t capacity, uint32_t *count, float frame[6])
{
	if (!c || !count)
		return fail(RTX_ERR_ARG, "null argument");
	if (!c->have_scene)
		return fail(RTX_ERR_STATE, "rtx_read_wide_tree before rtx_upload_scene");
	const DScene &S = c->scene;
	*count = S.w8 ? S.num_w8 : 0u;
	if (frame) {
		memcpy(frame, S.w8qo, 12);
		memcpy(frame + 3, S.w8qs, 12);
	}
	if (entries && S.w8 && capacity) {
		HIP_TRY(hipSetDevice(c->device));
		HIP_TRY(hipMemcpy(entries, S.w8, (size_t)std::min(capacity, S.num_w8) * sizeof(DW8), hipMemcpyDeviceToHost));
	}
	return RTX_OK;
}

extern "C" int rtx_get_stats(const rtx_ctx *c, rtx_stats *out)
{
	if (!c || !out)
		return fail(RTX_ERR_ARG, "null argument");
	*out = c->stats;
	return RTX_OK;
}

extern "C" int rtx_kat(int kind, uint32_t n, const float *in, float *out, const rtx_params *params)
{
	if (kind < 0 || kind >= RTX_KAT_NKINDS)
		return fail(RTX_ERR_ARG, "bad KAT kind %d", kind);
	if (!n)
		return RTX_OK;
	if (!in || !out)
		return fail(RTX_ERR_ARG, "null buffers");
	int ndev = 0;
	if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
		return fail(RTX_ERR_NODEV, "no HIP device available");
	const size_t bi = (size_t)n * rtx_kat_in_width[kind] * 4, bo = (size_t)n * rtx_kat_out_width[kind] * 4;
	float *din = nullptr, *dout = nullptr;
	HIP_TRY(hipMalloc(&din, bi));
	if (hipMalloc(&dout, bo) != hipSuccess) {
		(void)hipFree(din);
		return fail(RTX_ERR_NOMEM, "KAT output allocation failed");
	}
	int rc = RTX_OK;
	hipError_t e = hipMemcpy(din, in, bi, hipMemcpyHostToDevice);
	if (e == hipSuccess)
		e = kind >= RTX_KAT_FIRST_SHADOW ? rtx_launch_kat_shadow(kind, n, din, dout, nullptr)
						 : rtx_launch_kat(kind, n, din, dout, params ? params->u32conv : RTX_U32_SAT, nullptr);
	if (e == hipSuccess)
		e = hipMemcpy(out, dout, bo, hipMemcpyDeviceToHost);
	if (e != hipSuccess)
		rc = fail(RTX_ERR_HIP, "KAT failed: %s", hipGetErrorString(e));
	(void)hipFree(din);
	(void)hipFree(dout);
	return rc;
}
