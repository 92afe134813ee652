/*
 * Multi-device C-ABI (include/rtx.h rtx_group_*): one frame rendered by n MI355X devices of
 * one process.  Replaces the reference's parallel point, the OpenMP row loop of render()
 * (render.c:349-352), with a tile deal over devices:
 *
 *   open     peer access enabled between device 0 and every other device (the tree copies
 *            then go device to device over xGMI, not through host memory)
 *   upload   the scene is flattened and its BVHs built ONCE, on device 0 (rtx_build_scene,
 *            the work of accel_init, accel.c:266-315: device SAH build + 8-wide collapse); the
 *            other devices copy the device-built records and tree from it, one host thread
 *            per device, each on its own stream
 *   render   device r renders tiles t = r (mod n) on its own host thread (rtx_render_common
 *            with tile_offset r, tile_stride n), into its own HBM framebuffer
 *   gather   devices r > 0 pack their shard into 16-byte {r, g, b, z} tile records
 *            (rtx_gather.hip), and one grouped ncclSend / ncclRecv moves them to device 0
 *            over xGMI (RCCL, one communicator per device, ncclCommInitAll); device 0
 *            unpacks them into its frame, which is copied to the caller.
 *
 * At 1080p a shard is 4.1 MB / n per device; the gather is a few tens of microseconds of
 * link time.  With n = 1 no communicator is created.
 *
 * rtx_group_open_loopback: n shards as n contexts on one device, the gather a device-to-device
 * copy instead of RCCL; the rest of the path is the one above (tests/test_gpu_group.py runs it
 * at n = 2, 3, 8 on a one-GPU box against rtx_render).
 *
 * rtx_group_open_rccl_self: the other half a one-GPU box can check, the RCCL calls themselves.
 * One device with a one-rank communicator (ncclCommInitAll); the gather packs shard 0 too and
 * moves it through the same grouped ncclSend / ncclRecv (rank 0 to itself) into a receive buffer
 * filled with NaN bytes beforehand, then unpacks it over the frame, so the image is the
 * one-device image only if RCCL delivered every record.
 */
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <string.h>
#include <string>
#include <thread>
#include <vector>

#include "rtx_internal.h"
#include "rtx_tiles.h"

extern "C" hipError_t rtx_launch_tile_pack(const float *rgb, const float *z, uint32_t w, uint32_t h, uint32_t off,
					   uint32_t stride, float4 *out, hipStream_t stream);
extern "C" hipError_t rtx_launch_tile_unpack(const float4 *in, uint32_t w, uint32_t h, uint32_t off, uint32_t stride,
					     float *rgb, float *z, hipStream_t stream);

#define NCCL_TRY(expr)                                                                                  \
	do {                                                                                            \
		ncclResult_t r_ = (expr);                                                               \
		if (r_ != ncclSuccess)                                                                  \
			return fail(RTX_ERR_HIP, "%s failed: %s", #expr, ncclGetErrorString(r_));       \
	} while (0)

struct rtx_group {
	int n = 0;
	bool loopback = false;         /* rtx_group_open_loopback: every context on one device */
	bool rccl_self = false;        /* rtx_group_open_rccl_self: shard 0 sent to itself over RCCL */
	std::vector<uint32_t> peer;    /* peer access between device r and device 0 enabled */
	std::vector<rtx_ctx *> ctx;
	std::vector<ncclComm_t> comm;  /* n > 1 or rccl_self: one per device, rank r = ctx[r] */
	std::vector<float4 *> d_buf;   /* r > 0 (rccl_self: r = 0): shard r's packed records on device r */
	std::vector<float4 *> d_recv;  /* the same shards' records received on device 0 */
	std::vector<size_t> buf_cap;   /* capacity of d_buf[r] in records */
	std::vector<size_t> recv_cap;  /* capacity of d_recv[r] in records */
	rtx_stats stats{};
};

extern "C" void rtx_group_close(rtx_group *g)
{
	if (!g)
		return;
	for (int r = 0; r < (int)g->ctx.size(); r++) {
		if (!g->ctx[r])
			continue;
		(void)hipSetDevice(g->ctx[r]->device);
		if (r < (int)g->d_buf.size())
			dfree(g->d_buf[r]);
	}
	if (!g->ctx.empty() && g->ctx[0]) {
		(void)hipSetDevice(g->ctx[0]->device);
		for (auto &p : g->d_recv)
			dfree(p);
	}
	for (ncclComm_t c : g->comm)
		if (c)
			(void)ncclCommDestroy(c);
	for (rtx_ctx *c : g->ctx)
		rtx_close(c);
	delete g;
}

/* let device `dev` access `peer`'s memory (already enabled counts); false when the pair has no
 * peer path (copies then stage through the host, which is slower but correct) */
static bool enable_peer(int dev, int peer)
{
	int can = 0;
	if (hipDeviceCanAccessPeer(&can, dev, peer) != hipSuccess || !can)
		return false;
	if (hipSetDevice(dev) != hipSuccess)
		return false;
	hipError_t e = hipDeviceEnablePeerAccess(peer, 0);
	if (e == hipErrorPeerAccessAlreadyEnabled) {
		(void)hipGetLastError(); /* clear the sticky "already enabled" */
		return true;
	}
	return e == hipSuccess;
}

/* the caller's current device, restored on every way out of rtx_group_open (enable_peer and the
 * contexts' set-up switch devices) */
struct DeviceGuard {
	int dev = -1;
	DeviceGuard() { (void)hipGetDevice(&dev); }
	~DeviceGuard()
	{
		if (dev >= 0)
			(void)hipSetDevice(dev);
	}
};

extern "C" int rtx_group_open(int n, const int *devices, rtx_group **out)
{
	if (!out)
		return fail(RTX_ERR_ARG, "null out");
	*out = nullptr;
	if (n < 1 || n > 64)
		return fail(RTX_ERR_ARG, "group of %d devices (1..64)", n);
	DeviceGuard keep;
	std::vector<int> dev(n);
	for (int r = 0; r < n; r++) {
		dev[r] = devices ? devices[r] : r;
		for (int q = 0; q < r; q++)
			if (dev[q] == dev[r])
				return fail(RTX_ERR_ARG, "device %d listed twice", dev[r]);
	}
	rtx_group *g = new rtx_group();
	g->n = n;
	g->ctx.assign(n, nullptr);
	g->d_buf.assign(n, nullptr);
	g->d_recv.assign(n, nullptr);
	g->buf_cap.assign(n, 0);
	g->recv_cap.assign(n, 0);
	for (int r = 0; r < n; r++) {
		int rc = rtx_open(dev[r], &g->ctx[r]);
		if (rc) {
			rtx_group_close(g);
			return rc;
		}
	}
	g->peer.assign(n, 1u);
	for (int r = 1; r < n; r++) /* the upload's tree copies go device to device */
		g->peer[r] = enable_peer(dev[r], dev[0]) && enable_peer(dev[0], dev[r]);
	if (n > 1) {
		g->comm.assign(n, nullptr);
		ncclResult_t e = ncclCommInitAll(g->comm.data(), n, dev.data());
		if (e != ncclSuccess) {
			g->comm.assign(n, nullptr);
			rtx_group_close(g);
			return fail(RTX_ERR_HIP, "ncclCommInitAll over %d devices failed: %s", n, ncclGetErrorString(e));
		}
	}
	for (int r = 0; r < n; r++) {
		g->ctx[r]->stats.transport = n > 1 ? RTX_TRANSPORT_RCCL : RTX_TRANSPORT_NONE;
		g->ctx[r]->stats.peer_access = g->peer[r];
	}
	*out = g;
	return RTX_OK;
}

extern "C" int rtx_group_open_loopback(int n, int device, rtx_group **out)
{
	if (!out)
		return fail(RTX_ERR_ARG, "null out");
	*out = nullptr;
	if (n < 1 || n > 64)
		return fail(RTX_ERR_ARG, "loopback group of %d shards (1..64)", n);
	DeviceGuard keep;
	rtx_group *g = new rtx_group();
	g->n = n;
	g->loopback = true;
	g->ctx.assign(n, nullptr);
	g->d_buf.assign(n, nullptr);
	g->d_recv.assign(n, nullptr);
	g->buf_cap.assign(n, 0);
	g->recv_cap.assign(n, 0);
	g->peer.assign(n, 1u);
	for (int r = 0; r < n; r++) {
		int rc = rtx_open(device, &g->ctx[r]);
		if (rc) {
			rtx_group_close(g);
			return rc;
		}
		g->ctx[r]->stats.transport = n > 1 ? RTX_TRANSPORT_LOOPBACK : RTX_TRANSPORT_NONE;
		g->ctx[r]->stats.peer_access = 1u;
		g->ctx[r]->mem_share = (uint32_t)n; /* the n contexts render on this one device at once */
	}
	*out = g;
	return RTX_OK;
}

extern "C" int rtx_group_open_rccl_self(int device, rtx_group **out)
{
	int rc = rtx_group_open(1, &device, out);
	if (rc)
		return rc;
	rtx_group *g = *out;
	DeviceGuard keep;
	g->comm.assign(1, nullptr);
	ncclResult_t e = ncclCommInitAll(g->comm.data(), 1, &device);
	if (e != ncclSuccess) {
		g->comm.assign(1, nullptr);
		rtx_group_close(g);
		*out = nullptr;
		return fail(RTX_ERR_HIP, "ncclCommInitAll on device %d failed: %s", device, ncclGetErrorString(e));
	}
	g->rccl_self = true;
	g->ctx[0]->stats.transport = RTX_TRANSPORT_RCCL_SELF;
	return RTX_OK;
}

extern "C" int rtx_group_size(const rtx_group *g) { return g ? g->n : 0; }

extern "C" int rtx_group_member_info(const rtx_group *g, int r, rtx_group_member *out)
{
	if (!g || !out)
		return fail(RTX_ERR_ARG, "null argument");
	if (r < 0 || r >= g->n)
		return fail(RTX_ERR_ARG, "member %d of a group of %d", r, g->n);
	memset(out, 0, sizeof(*out));
	const int dev = g->ctx[r]->device, dev0 = g->ctx[0]->device;
	out->device = dev;
	out->comm_rank = out->comm_device = -1;
	if (r < (int)g->comm.size() && g->comm[r]) {
		NCCL_TRY(ncclCommCount(g->comm[r], &out->comm_count));
		NCCL_TRY(ncclCommUserRank(g->comm[r], &out->comm_rank));
		NCCL_TRY(ncclCommCuDevice(g->comm[r], &out->comm_device));
	}
	int can = 0;
	if (dev == dev0) {
		out->can_access_peer0 = out->peer0_can_access = 1u;
	} else {
		HIP_TRY(hipDeviceCanAccessPeer(&can, dev, dev0));
		out->can_access_peer0 = can ? 1u : 0u;
		HIP_TRY(hipDeviceCanAccessPeer(&can, dev0, dev));
		out->peer0_can_access = can ? 1u : 0u;
	}
	out->peer_enabled = g->peer[r];
	out->transport = g->ctx[r]->stats.transport;
	HIP_TRY(hipDeviceGetPCIBusId(out->pci_bus_id, (int)sizeof(out->pci_bus_id), dev));
	return RTX_OK;
}

extern "C" int rtx_group_set_builder(rtx_group *g, int builder)
{
	if (!g)
		return fail(RTX_ERR_ARG, "null group");
	for (rtx_ctx *c : g->ctx) {
		int rc = rtx_set_builder(c, builder);
		if (rc)
			return rc;
	}
	return RTX_OK;
}

extern "C" int rtx_group_set_option(rtx_group *g, int option, int64_t value)
{
	if (!g)
		return fail(RTX_ERR_ARG, "null group");
	for (rtx_ctx *c : g->ctx) {
		int rc = rtx_set_option(c, option, value);
		if (rc)
			return rc;
	}
	return RTX_OK;
}

/* a device buffer of `bytes` on device dst, copied from src on device sd on dst's stream (xGMI
 * with peer access; a plain device-to-device copy when sd == dst, the loopback group) */
template <class T> static int peer_copy(T *&out, int dst, const T *src, int sd, size_t bytes, hipStream_t s)
{
	out = nullptr;
	if (!src || !bytes)
		return RTX_OK;
	HIP_TRY(hipSetDevice(dst));
	HIP_TRY(hipMalloc(&out, bytes));
	hipError_t e = sd == dst ? hipMemcpyAsync(out, src, bytes, hipMemcpyDeviceToDevice, s)
				 : hipMemcpyPeerAsync(out, dst, src, sd, bytes, s);
	if (e != hipSuccess) {
		dfree(out);
		return fail(RTX_ERR_HIP, "peer copy of %zu bytes from device %d to %d failed: %s", bytes, sd, dst, hipGetErrorString(e));
	}
	return RTX_OK;
}

/* device r of the group takes copies of what device 0's build left in HBM, on its own host thread:
 * the records, the 8-wide tree (entries, scalar copies, leaf map), then the host parts */
static int upload_copy(rtx_group *g, int r, const HostScene &hs, const DevTree &src)
{
	rtx_ctx *c0 = g->ctx[0], *c = g->ctx[r];
	const auto t0 = std::chrono::steady_clock::now();
	HIP_TRY(hipSetDevice(c->device));
	dfree(c->d_nodes);
	c->have_scene = false;
	const size_t rec_bytes = ((size_t)hs.nnodes + hs.nb) * sizeof(DNode);
	const size_t ent = hs.w8_on_device ? hs.w8_entries : 0;
	DevTree t;
	t.device = c->device;
	int rc = RTX_OK;
	if ((!hs.recs_on_device || !(rc = peer_copy(c->d_nodes, c->device, c0->d_nodes, c0->device, rec_bytes, c->stream))) &&
	    !(rc = peer_copy(t.w8, c->device, src.w8, src.device, ent * sizeof(DW8), c->stream)) &&
	    !(rc = peer_copy(t.w8s, c->device, src.w8s, src.device, (ent ? hs.w8s_entries : 0) * sizeof(DW8S), c->stream)) &&
	    !(rc = peer_copy(t.leaf, c->device, src.leaf, src.device, ent * sizeof(uint32_t), c->stream))) {
		hipError_t e = hipStreamSynchronize(c->stream);
		if (e != hipSuccess)
			rc = fail(RTX_ERR_HIP, "device %d: scene copies: %s", c->device, hipGetErrorString(e));
	}
	c->stats.upload_copy_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
	if (!rc)
		rc = rtx_upload_built(c, hs, &t); /* takes the copies */
	(void)hipSetDevice(c->device); /* copies a failure left behind */
	dfree(t.w8);
	dfree(t.w8s);
	dfree(t.leaf);
	return rc;
}

extern "C" int rtx_group_upload_scene(rtx_group *g, const rtx_scene_desc *sc)
{
	if (!g || !sc)
		return fail(RTX_ERR_ARG, "null argument");
	/* built once, on device 0 (the device builder and the 8-wide collapse, as rtx_upload_scene);
	 * the other devices get device-to-device copies of what the build left in HBM, and the host
	 * parts (materials, planes, emitters, any host-built tree) from the host */
	HostScene hs;
	rtx_ctx *c0 = g->ctx[0];
	int rc = rtx_build_scene(c0, sc, hs);
	if (rc)
		return rc;
	const DevTree src{ hs.dev_w8, hs.dev_w8s, hs.dev_w8leaf, c0->device };
	/* devices 1..n-1 copy from device 0 concurrently, one host thread each; hs is only read */
	std::vector<int> rcs(g->n, RTX_OK);
	std::vector<std::string> errs(g->n);
	{
		std::vector<std::thread> th;
		for (int r = 1; r < g->n; r++)
			th.emplace_back([&, r] {
				rcs[r] = upload_copy(g, r, hs, src);
				if (rcs[r])
					errs[r] = rtx_last_error();
			});
		for (auto &t : th)
			t.join();
	}
	for (int r = 1; r < g->n; r++)
		if (rcs[r])
			return fail(rcs[r], "device %d: %s", g->ctx[r]->device, errs[r].c_str());
	/* device 0 last: it takes the original buffers (hs frees whatever a failure left), after every
	 * copy of them has completed */
	c0->stats.upload_copy_ms = 0.0;
	return rtx_upload_built(c0, hs);
}

static int grow_recs(float4 *&p, size_t &have, size_t need)
{
	if (need <= have)
		return RTX_OK;
	dfree(p);
	have = 0;
	HIP_TRY(hipMalloc(&p, need * sizeof(float4)));
	have = need;
	return RTX_OK;
}

static int ensure_fb(rtx_ctx *c, size_t px)
{
	if (px <= c->fb_pixels)
		return RTX_OK;
	dfree(c->d_rgb);
	dfree(c->d_z);
	HIP_TRY(hipMalloc(&c->d_rgb, px * 3 * sizeof(float)));
	HIP_TRY(hipMalloc(&c->d_z, px * sizeof(float)));
	c->fb_pixels = px;
	return RTX_OK;
}

extern "C" int rtx_group_render(rtx_group *g, const rtx_frame *fr, const rtx_params *p, float *rgb, float *z)
{
	if (!g || !fr || !p)
		return fail(RTX_ERR_ARG, "null argument");
	if (p->tile_offset != 0 || p->tile_stride != 1)
		return fail(RTX_ERR_ARG, "rtx_group_render shards the frame itself (tile_offset 0, tile_stride 1 expected)");
	for (rtx_ctx *c : g->ctx)
		if (!c->have_scene)
			return fail(RTX_ERR_STATE, "render before rtx_group_upload_scene");
	const int n = g->n;
	const uint32_t w = fr->width, h = fr->height;
	const size_t px = (size_t)w * h;
	for (rtx_ctx *c : g->ctx) {
		HIP_TRY(hipSetDevice(c->device));
		int rc = ensure_fb(c, px);
		if (rc)
			return rc;
	}
	/* every shard on its own host thread (rtx_render_common synchronises its stream) */
	std::vector<int> rcs(n, RTX_OK);
	std::vector<std::string> errs(n);
	auto shard = [&](int r) {
		rtx_ctx *c = g->ctx[r];
		if (hipSetDevice(c->device) != hipSuccess) {
			rcs[r] = RTX_ERR_HIP;
			errs[r] = "hipSetDevice failed";
			return;
		}
		rtx_params pr = *p;
		pr.tile_offset = (uint32_t)r;
		pr.tile_stride = (uint32_t)n;
		rcs[r] = rtx_render_common(c, fr, &pr, c->d_rgb, c->d_z, c->stream);
		if (rcs[r])
			errs[r] = rtx_last_error();
	};
	if (n == 1) {
		shard(0);
	} else {
		std::vector<std::thread> th;
		for (int r = 0; r < n; r++)
			th.emplace_back(shard, r);
		for (auto &t : th)
			t.join();
	}
	for (int r = 0; r < n; r++)
		if (rcs[r])
			return fail(rcs[r], "device %d: %s", g->ctx[r]->device, errs[r].c_str());

	const auto tg0 = std::chrono::steady_clock::now();
	rtx_ctx *c0 = g->ctx[0];
	const int r0 = g->rccl_self ? 0 : 1; /* the first shard that travels */
	if (n > 1 || g->rccl_self) {
		/* pack on every shard device, then one grouped send/recv to device 0 */
		for (int r = r0; r < n; r++) {
			rtx_ctx *c = g->ctx[r];
			const size_t recs = rtx_tile_pack_count(w, h, (uint32_t)r, (uint32_t)n);
			/* each buffer keeps its own capacity, so a failed allocation (capacity 0, null
			 * pointer) is retried on the next call instead of being used */
			HIP_TRY(hipSetDevice(c->device));
			int rc = grow_recs(g->d_buf[r], g->buf_cap[r], recs);
			if (rc)
				return rc;
			HIP_TRY(hipSetDevice(c0->device));
			if ((rc = grow_recs(g->d_recv[r], g->recv_cap[r], recs)))
				return rc;
			HIP_TRY(hipSetDevice(c->device));
			HIP_TRY(rtx_launch_tile_pack(c->d_rgb, c->d_z, w, h, (uint32_t)r, (uint32_t)n, g->d_buf[r], c->stream));
		}
		if (g->loopback) { /* the test transport: a device-to-device copy per shard, then device 0 waits */
			for (int r = 1; r < n; r++) {
				const size_t recs = rtx_tile_pack_count(w, h, (uint32_t)r, (uint32_t)n);
				if (!recs)
					continue;
				HIP_TRY(hipMemcpyAsync(g->d_recv[r], g->d_buf[r], recs * sizeof(float4), hipMemcpyDeviceToDevice,
						       g->ctx[r]->stream));
				HIP_TRY(hipStreamSynchronize(g->ctx[r]->stream));
			}
		} else {
			if (g->rccl_self) { /* what RCCL does not deliver stays NaN and fails the comparison */
				HIP_TRY(hipSetDevice(c0->device));
				HIP_TRY(hipMemsetAsync(g->d_recv[0], 0xFF, rtx_tile_pack_count(w, h, 0, 1) * sizeof(float4), c0->stream));
			}
			NCCL_TRY(ncclGroupStart());
			for (int r = r0; r < n; r++) {
				const size_t floats = rtx_tile_pack_count(w, h, (uint32_t)r, (uint32_t)n) * 4;
				if (!floats)
					continue;
				NCCL_TRY(ncclSend(g->d_buf[r], floats, ncclFloat, 0, g->comm[r], g->ctx[r]->stream));
				NCCL_TRY(ncclRecv(g->d_recv[r], floats, ncclFloat, r, g->comm[0], c0->stream));
			}
			NCCL_TRY(ncclGroupEnd());
		}
		HIP_TRY(hipSetDevice(c0->device));
		for (int r = r0; r < n; r++)
			HIP_TRY(rtx_launch_tile_unpack(g->d_recv[r], w, h, (uint32_t)r, (uint32_t)n, c0->d_rgb, c0->d_z, c0->stream));
		for (int r = 1; r < n; r++) {
			HIP_TRY(hipSetDevice(g->ctx[r]->device));
			HIP_TRY(hipStreamSynchronize(g->ctx[r]->stream));
		}
		HIP_TRY(hipSetDevice(c0->device));
		HIP_TRY(hipStreamSynchronize(c0->stream));
	}
	const double gather_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tg0).count();
	HIP_TRY(hipSetDevice(c0->device));
	if (rgb)
		HIP_TRY(hipMemcpy(rgb, c0->d_rgb, px * 12, hipMemcpyDeviceToHost));
	if (z)
		HIP_TRY(hipMemcpy(z, c0->d_z, px * 4, hipMemcpyDeviceToHost));

	/* statistics: counts summed, times of the slowest device */
	rtx_stats s = c0->stats;
	for (int r = 1; r < n; r++) {
		const rtx_stats &o = g->ctx[r]->stats;
		s.closest_rays += o.closest_rays;
		s.shadow_rays += o.shadow_rays;
		s.node_visits += o.node_visits;
		s.tri_tests += o.tri_tests;
		s.sphere_tests += o.sphere_tests;
		s.plane_tests += o.plane_tests;
		s.shadow_node_visits += o.shadow_node_visits;
		s.shadow_tri_tests += o.shadow_tri_tests;
		s.shadow_sphere_tests += o.shadow_sphere_tests;
		s.shadow_plane_tests += o.shadow_plane_tests;
		s.shade_points += o.shade_points;
		s.shadow_box_tests += o.shadow_box_tests;
		s.shadow_global_box_tests += o.shadow_global_box_tests;
		s.shadow_wave_steps += o.shadow_wave_steps;
		s.shadow_wave_walks += o.shadow_wave_walks;
		s.shadow_leaf_rounds += o.shadow_leaf_rounds;
		s.shadow_uniform_steps += o.shadow_uniform_steps;
		s.far_closest_rays += o.far_closest_rays;
		s.far_shadow_rays += o.far_shadow_rays;
		s.shadow_stack_spills += o.shadow_stack_spills;
		s.shadow_cone_clear += o.shadow_cone_clear;
		s.waves += o.waves;
		s.chunks += o.chunks;
		s.kernel_ms = std::max(s.kernel_ms, o.kernel_ms);
		s.trace_ms = std::max(s.trace_ms, o.trace_ms);
		s.shadow_ms = std::max(s.shadow_ms, o.shadow_ms);
		s.accum_ms = std::max(s.accum_ms, o.accum_ms);
		s.sort_ms = std::max(s.sort_ms, o.sort_ms);
		s.upload_copy_ms = std::max(s.upload_copy_ms, o.upload_copy_ms);
		s.peer_access = s.peer_access && o.peer_access;
	}
	s.gather_ms = n > 1 || g->rccl_self ? gather_ms : 0.0;
	s.devices = (uint32_t)n;
	g->stats = s;
	return RTX_OK;
}

extern "C" int rtx_group_get_stats(const rtx_group *g, rtx_stats *out)
{
	if (!g || !out)
		return fail(RTX_ERR_ARG, "null argument");
	*out = g->stats;
	return RTX_OK;
}

extern "C" int rtx_group_device_stats(const rtx_group *g, int r, rtx_stats *out)
{
	if (!g || !out)
		return fail(RTX_ERR_ARG, "null argument");
	if (r < 0 || r >= g->n)
		return fail(RTX_ERR_ARG, "device %d of a group of %d", r, g->n);
	*out = g->ctx[r]->stats;
	return RTX_OK;
}

/* ---- tile records: host reference and device entry points (rtx_tiles.h) ---- */

extern "C" size_t rtx_tile_pack_count(uint32_t w, uint32_t h, uint32_t off, uint32_t stride)
{
	if (!stride || off >= stride)
		return 0;
	return (size_t)rtx_shard_tiles(w, h, off, stride) * RTX_TILE_PX;
}

extern "C" int rtx_tile_pack_host(const float *rgb, const float *z, uint32_t w, uint32_t h, uint32_t off, uint32_t stride,
				  float *out)
{
	if (!rgb || !z || !out || !stride || off >= stride)
		return fail(RTX_ERR_ARG, "bad tile pack arguments");
	const size_t nrec = rtx_tile_pack_count(w, h, off, stride);
	const uint32_t tx = rtx_tiles_x(w);
	for (size_t i = 0; i < nrec; i++) {
		uint32_t x, y;
		rtx_shard_pixel((uint32_t)i, tx, off, stride, &x, &y);
		float *o = out + 4 * i;
		if (x < w && y < h) {
			const size_t p = (size_t)y * w + x;
			o[0] = rgb[3 * p];
			o[1] = rgb[3 * p + 1];
			o[2] = rgb[3 * p + 2];
			o[3] = z[p];
		} else {
			o[0] = o[1] = o[2] = o[3] = 0.f;
		}
	}
	return RTX_OK;
}

extern "C" int rtx_tile_unpack_host(const float *in, uint32_t w, uint32_t h, uint32_t off, uint32_t stride, float *rgb,
				    float *z)
{
	if (!in || !rgb || !z || !stride || off >= stride)
		return fail(RTX_ERR_ARG, "bad tile unpack arguments");
	const size_t nrec = rtx_tile_pack_count(w, h, off, stride);
	const uint32_t tx = rtx_tiles_x(w);
	for (size_t i = 0; i < nrec; i++) {
		uint32_t x, y;
		rtx_shard_pixel((uint32_t)i, tx, off, stride, &x, &y);
		if (x >= w || y >= h)
			continue;
		const size_t p = (size_t)y * w + x;
		rgb[3 * p] = in[4 * i];
		rgb[3 * p + 1] = in[4 * i + 1];
		rgb[3 * p + 2] = in[4 * i + 2];
		z[p] = in[4 * i + 3];
	}
	return RTX_OK;
}

extern "C" int rtx_tile_pack_device(rtx_ctx *c, const void *d_rgb, const void *d_z, uint32_t w, uint32_t h, uint32_t off,
				    uint32_t stride, void *d_out, void *stream)
{
	if (!c || !d_rgb || !d_z || !d_out || !stride || off >= stride)
		return fail(RTX_ERR_ARG, "bad tile pack arguments");
	HIP_TRY(hipSetDevice(c->device));
	hipStream_t s = stream ? (hipStream_t)stream : c->stream;
	HIP_TRY(rtx_launch_tile_pack((const float *)d_rgb, (const float *)d_z, w, h, off, stride, (float4 *)d_out, s));
	HIP_TRY(hipStreamSynchronize(s));
	return RTX_OK;
}

extern "C" int rtx_tile_unpack_device(rtx_ctx *c, const void *d_in, uint32_t w, uint32_t h, uint32_t off, uint32_t stride,
				      void *d_rgb, void *d_z, void *stream)
{
	if (!c || !d_in || !d_rgb || !d_z || !stride || off >= stride)
		return fail(RTX_ERR_ARG, "bad tile unpack arguments");
	HIP_TRY(hipSetDevice(c->device));
	hipStream_t s = stream ? (hipStream_t)stream : c->stream;
	HIP_TRY(rtx_launch_tile_unpack((const float4 *)d_in, w, h, off, stride, (float *)d_rgb, (float *)d_z, s));
	HIP_TRY(hipStreamSynchronize(s));
	return RTX_OK;
}
