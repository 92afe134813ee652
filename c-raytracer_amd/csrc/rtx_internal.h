/*
 * Library-internal declarations shared by rtx_api.cpp (single-device C-ABI) and rtx_group.cpp
 * (multi-device C-ABI): the device context, a host-built scene, and the render entry.
 * Not installed; nothing outside librtx includes it.
 */
#ifndef RTX_INTERNAL_H
#define RTX_INTERNAL_H

#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

#include "rtx.h"
#include "rtx_device.h"

/* sets the calling thread's rtx_last_error() message, returns code */
int rtx_fail(int code, const char *fmt, ...);
#define fail rtx_fail

#define HIP_TRY(expr)                                                                                   \
	do {                                                                                            \
		hipError_t e_ = (expr);                                                                 \
		if (e_ != hipSuccess)                                                                   \
			return fail(RTX_ERR_HIP, "%s failed: %s", #expr, hipGetErrorString(e_));        \
	} while (0)

template <class T> static inline void dfree(T *&p)
{
	if (p)
		(void)hipFree(p);
	p = nullptr;
}

/* a host vector into a fresh device buffer, copied on `stream` (the context's own: no
 * synchronisation with the null stream) and complete on return */
template <class T> static inline int upload(T *&dst, const std::vector<T> &v, hipStream_t stream)
{
#if RTX_MEASURE
	const auto t0 = std::chrono::steady_clock::now();
#endif
	dfree(dst);
	size_t n = std::max<size_t>(v.size(), 1);
	HIP_TRY(hipMalloc(&dst, n * sizeof(T)));
#if RTX_MEASURE
	const auto t1 = std::chrono::steady_clock::now();
#endif
	if (!v.empty()) {
		HIP_TRY(hipMemcpyAsync(dst, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, stream));
		HIP_TRY(hipStreamSynchronize(stream));
	}
#if RTX_MEASURE
	const auto t2 = std::chrono::steady_clock::now();
	const double a = std::chrono::duration<double, std::milli>(t1 - t0).count(), b = std::chrono::duration<double, std::milli>(t2 - t1).count();
	if (a + b > 1.0)
		fprintf(stderr, "[rtx upload]   upload of %zu B: free + malloc %.2f ms, copy %.2f ms\n", v.size() * sizeof(T), a, b);
#endif
	return RTX_OK;
}

/* the settings a render's shade points per tile depend on (rtx_ctx.sp_tile_key) */
struct SpKey {
	uint32_t v[21] = {};
	uint32_t set = 0;
	bool operator==(const SpKey &o) const { return set && o.set && std::equal(v, v + 21, o.v); }
};

struct rtx_ctx {
	int device = 0;
	int builder = RTX_BUILD_SAH_GPU; /* the host's SAH tree, built on the device (29 vs 343 ms on the dragon) */
	hipStream_t stream = nullptr;
	hipEvent_t ev0 = nullptr, ev1 = nullptr;
	int cus = 0;
	/* scene */
	DNode *d_nodes = nullptr;
	DPlane *d_planes = nullptr;
	DMaterial *d_mats = nullptr;
	DEmitter *d_emitters = nullptr;
	DEmitter *d_lin = nullptr; /* RTX_WALK_LINEAR: the bounded objects as shadow-test records */
	DQNode *d_qnodes = nullptr;
	uint32_t *d_top = nullptr;
	DW8 *d_w8 = nullptr;
	DW8S *d_w8s = nullptr;
	uint32_t *d_w8spill = nullptr; /* k_shadow lane-stack spill of deep 8-wide trees (DScene.w8spill) */
	float4 *d_cull = nullptr;      /* the 8-wide tree's top-level bounding spheres (DScene.cull) */
	size_t w8spill_bytes = 0;
	DScene scene{};
	bool have_scene = false;
	/* work buffers (grow-only) */
	DTask *d_tasks = nullptr;
	size_t task_bytes = 0;
	uint32_t *d_ostk = nullptr; /* k_trace lane-stack overflow (DScene.ostk) */
	size_t ostk_bytes = 0;
	float4 *d_staging = nullptr;
	size_t staging_bytes = 0;
	float4 *d_sp = nullptr;
	size_t sp_bytes = 0;
	float4 *d_contrib = nullptr;
	size_t contrib_bytes = 0;
	uint2 *d_tile_rec = nullptr;
	size_t tile_rec_bytes = 0;
	/* shade points per tile seen by the last render of this scene with the same GI / bounce
	 * settings: sizes the next render's chunks (the static estimate is 5x too high on scene6) */
	double sp_tile_seen = 0.0;
	SpKey sp_tile_key{};
	uint32_t *d_sortbuf = nullptr; /* keys0 | keys1 | vals0 | vals1 (shade-point sort) */
	size_t sortbuf_bytes = 0;
	void *d_sorttmp = nullptr;
	size_t sorttmp_bytes = 0;
	int *d_post_rad = nullptr; /* postprocess: per-pixel DoF radius, pv, scratch */
	float4 *d_post_pv = nullptr;
	size_t post_pixels = 0;
	unsigned *d_post_scratch = nullptr;
	float bound_lo[3] = { 0, 0, 0 }, bound_hi[3] = { 0, 0, 0 }; /* bounded objects' box */
	hipEvent_t ev[5] = { nullptr, nullptr, nullptr, nullptr, nullptr };
	uint32_t total_lights = 0;
	unsigned long long *d_ctr = nullptr;
	float *d_rgb = nullptr, *d_z = nullptr;
	size_t fb_pixels = 0;
	rtx_stats stats{};
	/* rtx_set_option (include/rtx.h RTX_OPT_*) */
	int opt_walk = RTX_WALK_AUTO;
	uint32_t opt_leaf = 1;
	bool opt_spsort = true;
	uint32_t opt_slot = 0;
	uint32_t opt_grab = 4096;
	uint32_t opt_lstk = RTX_W8_STACK;
	int opt_trace_walk = RTX_WALK_AUTO;
	int opt_frame = RTX_FRAME_AUTO;
	uint32_t opt_chunk = 0;   /* most tiles per chunk (0: as many as the shade-point budget allows) */
	uint32_t opt_sp_tile = 0; /* shade points per tile a chunk is sized for (0: the estimate / last render's count) */
	int opt_cull = 1;         /* RTX_OPT_SHADOW_CULL: 0 off, 1 wave-uniform packets, 2 lane slots too */
	uint32_t mem_share = 1;   /* contexts sharing this device's HBM at once (a loopback group's n): the shade-point
	                           * budget of a render is a third of the free HBM divided by it */
};

struct QFrame {
	float qo[3], qs[3];
};

/* a scene flattened and its BVHs built (on the host, or on the building context's device), ready
 * to upload to one or more devices.  Device buffers it still owns are freed with it. */
struct HostScene {
	int builder = RTX_BUILD_SAH_HOST;
	int device = 0;               /* the building context's device */
	bool recs_on_device = false;  /* device builder: the building context holds the records */
	std::vector<DNode> recs;      /* inner nodes then primitives (64-byte records) */
	uint32_t nnodes = 0, nb = 0, root_ref = RTX_EMPTY_REF, depth = 0;
	std::vector<DQNode> qnodes;   /* threaded BVH2 */
	QFrame qf{};
	std::vector<uint32_t> qtop;
	uint32_t ntop = 0;
	std::vector<DW8> w8;          /* 8-wide BVH entries (leaf entries filled on the device) */
	std::vector<uint32_t> w8leaf; /* entry -> primitive index (RTX_NONE: node or hole) */
	uint32_t w8depth = 0;
	QFrame w8f{};                 /* its 16-bit frame */
	bool w8noemit = false;        /* emitters left out of it */
	/* collapsed on the device (rtx_wide8_dev.hip): the buffers, handed to the context on upload
	 * (rtx_upload_built clears these pointers when it takes them) */
	bool w8_on_device = false;
	DW8 *dev_w8 = nullptr;
	DW8S *dev_w8s = nullptr;
	uint32_t *dev_w8leaf = nullptr;
	uint32_t w8_entries = 0, w8_wide = 0;
	uint32_t w8s_entries = 0; /* device collapse: scalar-path copies allocated (entries below the last node entry) */
	uint32_t w8top = 0; /* entries of the 8-wide tree's top levels (rtx_device.h DScene.w8top) */
	bool w8sph = true;  /* the 8-wide tree holds spheres (DScene.w8sph) */
	std::vector<DPlane> planes;
	std::vector<DMaterial> mats;
	std::vector<DEmitter> emit;
	std::vector<DEmitter> lin;    /* RTX_WALK_LINEAR: every bounded object as a shadow-test record */
	float bound_lo[3] = { 0, 0, 0 }, bound_hi[3] = { 0, 0, 0 }, ambient[3] = { 0, 0, 0 };
	uint32_t num_emitters = 0;
	DTreeFrame tf{};              /* the frame every tree's boxes are in (rtx_frame.cpp) */
	double frame_ratio = 1.0;     /* its sampled leaf-box cost over the identity's */
	double frame_pad = 0;         /* the leaf boxes' padding for the ray transform (rtx_frame.cpp) */
	double frame_ms = 0;          /* choosing it and the leaf boxes in it */
	double build_ms = 0;
	HostScene() = default;
	HostScene(const HostScene &) = delete;
	HostScene &operator=(const HostScene &) = delete;
	~HostScene()
	{
		if (dev_w8 || dev_w8s || dev_w8leaf) {
			(void)hipSetDevice(device);
			dfree(dev_w8);
			dfree(dev_w8s);
			dfree(dev_w8leaf);
		}
	}
};

/* flatten sc and build its BVHs (on c's device for the device builder), then upload to c */
int rtx_build_scene(rtx_ctx *c, const rtx_scene_desc *sc, HostScene &hs);
int rtx_upload_built(rtx_ctx *c, HostScene &hs);
/* a device-collapsed 8-wide tree's buffers on one device (hs.w8_on_device): the building device's
 * own, or a device group's peer copies of them */
struct DevTree {
	DW8 *w8 = nullptr;
	DW8S *w8s = nullptr;
	uint32_t *leaf = nullptr;
	int device = 0;
};
/* upload a built scene to c, taking the device tree from `take` (c's device; c owns the buffers
 * after the call and take's pointers are cleared once handed over: on failure the caller frees
 * whatever take still holds).  hs is only read, so several contexts may upload one scene at once
 * from their own host threads. */
int rtx_upload_built(rtx_ctx *c, const HostScene &hs, DevTree *take);
/* rtx_wide8.cpp: the 8-wide shadow BVH collapsed from the BVH2 (0 = not built); boxes it takes
 * from primitive records (leaves of several primitives) in the trees' frame tf, padded by fpad */
uint32_t rtx_wide8_build(const std::vector<DNode> &inner, uint32_t nnodes, const DPrim *prims, uint32_t root_ref,
			 const float lo[3], const float hi[3], const std::vector<uint32_t> &skip_objs, const DTreeFrame &tf,
			 double fpad, QFrame &F, bool &skipped, std::vector<DW8> &out, std::vector<uint32_t> &leafmap);
/* one frame (or tile shard) into device buffers on stream */
int rtx_render_common(rtx_ctx *c, const rtx_frame *fr, const rtx_params *p, float *d_rgb, float *d_z, hipStream_t stream);

#endif
