/*
 * rtx.h — C-ABI of the MI355X-native trace/intersect/shade path.
 *
 * Drop-in boundary for C-Raytracer's hot path.  The reference
 * enters the path at src/raytracer/main.c:76-79:
 *
 *     accel_init();   // accel.c:266-315   BVH build over objects[]
 *     render_init();  // render.c:61-116   CLI -> render globals
 *     render();       // render.c:345-368  per-pixel cast_ray() recursion
 *     ...
 *     accel_deinit(); // accel.c:100-103
 *
 * with all inputs passed through globals (objects[], emittant_objects[],
 * unbound_objects[], materials[], camera, image, global_ambient_light_intensity)
 * and the outputs image.raster / image.z_buffer.  Here every input crosses the
 * boundary explicitly as plain structs and pointers:
 *
 *     rtx_open()          replaces nothing (device context; owns device memory)
 *     rtx_upload_scene()  replaces accel_init()           accel.c:266
 *     rtx_render()        replaces render_init()+render() render.c:61, 345
 *     rtx_close()         replaces accel_deinit()         accel.c:100
 *
 * Host glue that the reference keeps outside the path (scene.c JSON loader,
 * object.c STL ingest, image.c image-plane setup and TIFF writer, argv.c CLI)
 * lives in librtxscene and is declared in rtx_scene.h.
 *
 * Conventions: every int-returning call returns RTX_OK (0) or a negative
 * RTX_ERR_* code and sets a thread-local message readable with
 * rtx_last_error().  The library never calls exit().  Buffers passed in are
 * caller-owned and copied; the library owns device memory only.
 */
#ifndef RTX_H
#define RTX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RTX_ABI_VERSION 1

enum rtx_status {
	RTX_OK = 0,
	RTX_ERR_ARG = -1,     /* bad argument / shape */
	RTX_ERR_HIP = -2,     /* HIP runtime failure */
	RTX_ERR_NOMEM = -3,   /* host or device allocation failed */
	RTX_ERR_SCENE = -4,   /* scene rejected (reference would error()/exit(1)) */
	RTX_ERR_NODEV = -5,   /* no usable gfx950 device */
	RTX_ERR_STATE = -6,   /* call order (e.g. render before upload) */
	RTX_ERR_IO = -7,      /* file I/O (scene / mesh / TIFF) */
};

/* object.h:17-23 enum ObjectType (UNBOUND_OBJECTS build) */
enum rtx_object_type { RTX_SPHERE = 0, RTX_TRIANGLE = 1, RTX_PLANE = 2 };

/* material.c:27-53 texture kinds, material.h:17-22 enum PeriodicFunction */
enum rtx_texture_type {
	RTX_TEX_UNIFORM = 0,
	RTX_TEX_CHECKERBOARD = 1,
	RTX_TEX_BRICK = 2,
	RTX_TEX_NOISY_PERIODIC = 3,
};
enum rtx_periodic { RTX_PERIODIC_SIN = 0, RTX_PERIODIC_SAW = 1, RTX_PERIODIC_TRIANGLE = 2, RTX_PERIODIC_SQUARE = 3 };

/* struct Material (material.h:30-44) + its texture, flattened. */
typedef struct rtx_material {
	int32_t id;
	float ks[3], ka[3], kr[3], kt[3], ke[3];
	float shininess;
	float refractive_index;
	int32_t texture;        /* enum rtx_texture_type */
	int32_t periodic;       /* enum rtx_periodic (noisy periodic only) */
	/* uniform: color[0]; checkerboard/brick: colors[0], colors[1];
	 * noisy periodic: color[0] = color, color[1] = color gradient */
	float color[2][3];
	float scale;            /* checkerboard, brick */
	float mortar_width;     /* brick */
	float noise_feature_scale, noise_scale, frequency_scale; /* noisy periodic */
	/* material_init (material.c:81-83): ‖k‖ > 1e-6 */
	int32_t emittant, reflective, transparent;
} rtx_material;

/*
 * One object of the reference's objects[] array (object.c:25-44), in load
 * order, with the values its *_postinit / *_scale produced:
 *   sphere   : p0 = position, radius                                (object.c:25-29)
 *   triangle : p0,p1,p2 = vertices, e1 = v1-v0, e2 = v2-v0,
 *              n = norm(e1 x e2)                                    (object.c:31-36, 327-340)
 *   plane    : n = unit normal, d = n . position                    (object.c:39-43, 457-466)
 * epsilon is resolved (per-type default applied), num_lights as loaded.
 */
typedef struct rtx_object {
	int32_t type;           /* enum rtx_object_type */
	int32_t material;       /* index into rtx_scene_desc.materials */
	uint32_t num_lights;
	float epsilon;
	float p0[3], p1[3], p2[3];
	float e1[3], e2[3];
	float n[3];
	float radius;
	float d;
} rtx_object;

/* struct Camera (camera.h:17-22) after camera_init/camera_scale. */
typedef struct rtx_camera {
	float position[3];
	float vectors[3][3];    /* v0, v1 normalised; v2 = v0 x v1 (camera.c:29-32) */
	float fov;
	float focal_length;
} rtx_camera;

/* Everything accel_init() + render() read from globals. */
typedef struct rtx_scene_desc {
	uint32_t num_materials;
	const rtx_material *materials;
	uint32_t num_objects;
	const rtx_object *objects;       /* reference order */
	uint32_t num_emitters;
	const uint32_t *emitters;        /* object indices, emittant_objects[] order */
	float ambient[3];                /* global_ambient_light_intensity */
	rtx_camera camera;
} rtx_scene_desc;

/* struct Image's plane (image.h:17-26) as image_init (image.c:34-56) built it. */
typedef struct rtx_frame {
	uint32_t width, height;
	float corner[3];        /* image.corner */
	float step_x[3];        /* image.vectors[X] */
	float step_y[3];        /* image.vectors[Y] */
	float origin[3];        /* camera.position */
} rtx_frame;

enum rtx_reflection { RTX_PHONG = 0, RTX_BLINN = 1 };                       /* render.c:32-35 */
enum rtx_gi { RTX_GI_AMBIENT = 0, RTX_GI_PATH = 1 };                        /* render.c:37-40 */
enum rtx_attenuation { RTX_ATT_NONE = 0, RTX_ATT_LIN = 1, RTX_ATT_SQR = 2 }; /* render.c:42-46 */
/* rand_flt (system.c:93-96) replacement */
enum rtx_rng {
	RTX_RNG_COUNTER = 0,  /* counter-based hash of (seed, pixel, ray-tree node, draw): i.i.d. draws like
	                       * rand_flt, two per light sample (object.c:298-299, 403-419); the default */
	RTX_RNG_CONST = 1,    /* every draw == 0.5f (the oracle's REF_CONST_RNG) */
	RTX_RNG_STRAT = 2,    /* RTX_RNG_COUNTER with the light samples stratified (opt-in): sample j
	                       * of an emitter's n draws its first number (the sphere's inclination, the
	                       * triangle's p) from [j/n, (j+1)/n) as ((float)j + u) / n; each stratum is
	                       * sampled uniformly, so the estimator keeps render.c:170-229's expectation
	                       * (a different estimator from the reference's i.i.d. one, lower variance) */
};
/* (uint32_t)float in texture_get_color_checkerboard/brick (material.c:164,173)
 * is UB for negatives; its result depends on the host ISA. */
enum rtx_u32conv {
	RTX_U32_SAT = 0,      /* x86 AVX-512 vcvttss2usi: x <= -1 or >= 2^32 or NaN -> 0xFFFFFFFF */
	RTX_U32_WRAP = 1,     /* 64-bit cvttss2si truncated to 32 bits (generic x86-64) */
};

/* render_init() globals (render.c:53-60) + library extensions. */
#define RTX_MAX_BOUNCES 4096 /* the reflection/refraction task stacks are sized for max_bounces up to this */
typedef struct rtx_params {
	uint32_t max_bounces;        /* -b, default 10, at most RTX_MAX_BOUNCES (RTX_ERR_ARG above) */
	float min_intensity_sqr;     /* -a squared, default 1e-4 */
	int32_t reflection;          /* -s, enum rtx_reflection, default phong */
	int32_t gi;                  /* -g, enum rtx_gi, default ambient */
	uint32_t samples;            /* -n, default 1 (path GI samples at the primary hit) */
	int32_t attenuation;         /* -l, enum rtx_attenuation, default sqr */
	float attenuation_offset;    /* -o, default 1.0 */
	int32_t rng;                 /* enum rtx_rng */
	uint64_t seed;
	int32_t u32conv;             /* enum rtx_u32conv */
	/* sharding: render only tiles t with t % tile_stride == tile_offset
	 * (1 tile = 8x8 pixels, row-major over the frame).  Pixels of other tiles are
	 * left untouched in the output.  Defaults 0 / 1 = whole frame. */
	uint32_t tile_offset, tile_stride;
	/* count BVH node visits and primitive tests (slower kernel instance) */
	int32_t count_traversal;
} rtx_params;

/* Defaults of render.c:53-60 (+ counter RNG, seed 1, SAT conversion, whole frame). */
void rtx_params_default(rtx_params *p);

typedef struct rtx_stats {
	uint64_t closest_rays;       /* cast_ray() calls (render.c:136) */
	uint64_t shadow_rays;        /* is_light_blocked() calls (render.c:126) */
	/* only with count_traversal: per-ray work summed over all rays (closest + shadow) */
	uint64_t node_visits;        /* BVH inner nodes fetched (2 child boxes tested) */
	uint64_t tri_tests;
	uint64_t sphere_tests;
	uint64_t plane_tests;
	/* ... of which by shadow rays (node visits in BVH2 units: shadow_box_tests / 2) */
	uint64_t shadow_node_visits;
	uint64_t shadow_tri_tests;
	uint64_t shadow_sphere_tests;
	uint64_t shadow_plane_tests;
	uint64_t shade_points;       /* hits whose direct lighting was evaluated */
	double kernel_ms;            /* device time of the last rtx_render*, HIP events, all kernels */
	double trace_ms;             /* ... closest-hit / shading kernel */
	double shadow_ms;            /* ... shadow-ray kernel */
	double accum_ms;             /* ... per-tile accumulation kernel */
	double sort_ms;              /* ... shade-point ordering (key + radix sort) */
	double build_ms;             /* host wall time of the last rtx_upload_scene's BVH build (incl. its uploads) */
	uint32_t bvh_nodes;
	uint32_t bvh_depth;
	uint32_t bvh_prims;
	uint32_t waves;              /* persistent waves of the closest-hit kernel */
	uint32_t chunks;             /* tile chunks the frame was split into */
	uint32_t builder;            /* RTX_BUILD_* used by the last upload */
	/* only with count_traversal: the shadow walk (k_shadow) */
	uint64_t shadow_box_tests;        /* box tests (threaded-BVH records stepped through), summed over shadow rays */
	uint64_t shadow_global_box_tests; /* ... of which read from the DQNode array (the rest from the LDS top copy) */
	uint64_t shadow_wave_steps;       /* walk-loop iterations summed over waves (a wave steps until its longest ray ends) */
	uint64_t shadow_wave_walks;       /* wave walks (64 lane slots each): steps / walks = the waves' mean walk length */
	uint32_t wide_nodes;              /* 8-wide BVH nodes (0: k_shadow walks the threaded BVH2) */
	uint32_t wide_depth;
	uint64_t shadow_leaf_rounds;      /* only with count_traversal, 8-wide walk: wave iterations of its leaf loops */
	double gather_ms;                 /* rtx_group_render: shard pack + RCCL gather + unpack (0 on one device) */
	uint32_t devices;                 /* devices that rendered the last frame */
	uint32_t pad_;
	uint64_t shadow_uniform_steps;    /* only with count_traversal, 8-wide walk: wave steps whose active lanes were all at one node */
	uint32_t shadow_walk;             /* the BVH k_shadow walks: RTX_WALK_W8 / RTX_WALK_BVH2 / RTX_WALK_LINEAR */
	uint32_t wide_entries;            /* 8-wide walk: 64-byte entries (nodes, primitive records, holes) */
	uint32_t trace_walk;              /* the BVH k_trace walks for closest hits: RTX_WALK_W8 / RTX_WALK_BVH2 */
	uint32_t pad2_;
	uint32_t tree_rotated;            /* the trees are built in a rotated frame (rtx_tree_frame) */
	uint32_t pad3_;
	double frame_cost;                /* its sampled leaf-box surface area over the world frame's (1: world frame) */
	double frame_ms;                  /* host time choosing the frame and taking the leaf boxes in it */
	double upload_copy_ms;            /* device groups: this device's copies of the scene built on device 0
	                                   * (last rtx_group_upload_scene; 0 on device 0 and for single contexts) */
	uint32_t transport;               /* device groups: RTX_TRANSPORT_* of the shard gather */
	uint32_t peer_access;             /* device groups: this device and device 0 have peer access enabled
	                                   * (hipDeviceEnablePeerAccess both ways; 1 on device 0 itself) */
	/* only with count_traversal: rays whose origin lies more than 4 scene radii from the bounded
	 * objects, whose box tests start from a point formed in double near them (any tree frame) */
	uint64_t far_closest_rays;        /* closest-hit rays (the frame origin moved along the ray) */
	uint64_t far_shadow_rays;         /* shadow rays from far shade points (walked from the light end) */
	uint64_t shadow_stack_spills;     /* only with count_traversal, 8-wide walk: lane-stack entries pushed beyond
	                                   * the LDS ones (to HBM, DScene.w8spill) */
	uint64_t shadow_cone_clear;       /* only with count_traversal: shadow rays of packets whose light cone met no
	                                   * box of the 8-wide tree's top levels, so they were not walked
	                                   * (RTX_OPT_SHADOW_CULL) */
} rtx_stats;

typedef struct rtx_ctx rtx_ctx;

/* BVH builders for rtx_upload_scene (replacing accel_init, accel.c:266-315) */
enum {
	RTX_BUILD_SAH_HOST = 0, /* binned SAH on the host (bvh_build.cpp) */
	RTX_BUILD_LBVH_GPU = 1, /* Morton-code linear BVH built on the device (rtx_build.hip) */
	RTX_BUILD_PLOC_GPU = 2, /* locally-ordered clustering (PLOC) on the device (rtx_build.hip) */
	RTX_BUILD_SAH_GPU = 3   /* default: the host's binned SAH run on the device, level by level (rtx_build.hip), the same tree */
};

int rtx_device_count(int *count);
/* Open a context on HIP device `device` (must be gfx950).  Loads the library's device code on
 * that device and primes host-to-device copies once (~0.1 s), so uploads and renders do not. */
int rtx_open(int device, rtx_ctx **out);
/* Flatten + copy the scene to the device, build the BVH (replaces accel_init). */
int rtx_upload_scene(rtx_ctx *ctx, const rtx_scene_desc *scene);
/* Render into caller-owned HOST buffers rgb[W*H*3] (row-major, row 0 = top,
 * overwritten, not accumulated) and z[W*H] (primary-hit distance, 0 on miss);
 * either may be NULL.  Replaces render_init()+render(). */
int rtx_render(rtx_ctx *ctx, const rtx_frame *frame, const rtx_params *params, float *rgb, float *z);
/* Same into DEVICE buffers on the context's device, enqueued on `stream`
 * (hipStream_t, NULL = the context's own stream); synchronises the stream. */
int rtx_render_device(rtx_ctx *ctx, const rtx_frame *frame, const rtx_params *params, void *d_rgb, void *d_z,
		      void *stream);
int rtx_get_stats(const rtx_ctx *ctx, rtx_stats *out);
/* Builder used by subsequent rtx_upload_scene calls on this context (RTX_BUILD_*). */
int rtx_set_builder(rtx_ctx *ctx, int builder);

/* Shadow-walk BVH layouts (rtx_stats.shadow_walk, RTX_OPT_SHADOW_WALK); 1 was the 4-wide walk */
enum {
	RTX_WALK_AUTO = -1, /* the fastest available: LINEAR for tiny scenes, the threaded BVH2 from LDS for
	                     * small ones (<= 1024 bounded objects), else 8-wide */
	RTX_WALK_BVH2 = 0,  /* threaded quantised BVH2 (DQNode), no stack */
	RTX_WALK_W8 = 2,    /* 8-wide compressed BVH (8-bit child boxes in each node's frame) */
	RTX_WALK_LINEAR = 3 /* no tree: every bounded object tested one by one, like the planes (AUTO for
	                     * scenes of at most RTX_SHADOW_LINEAR_MAX bounded objects) */
};
#define RTX_SHADOW_LINEAR_MAX 8
/* The frame the BVHs are built in (RTX_OPT_TREE_FRAME, rtx_tree_frame) */
enum {
	RTX_FRAME_AUTO = 0,  /* default: a rotated frame when it shrinks the leaf boxes (a rotated mesh's own axes) */
	RTX_FRAME_WORLD = 1  /* always the world axes, as accel.c:266-315 */
};
/* Context options: the defaults are the tuned values; the others exist for A/B measurement and
 * tests.  Build options take effect at the next rtx_upload_scene. */
enum rtx_option {
	RTX_OPT_SHADOW_WALK = 1, /* RTX_WALK_* (build; default RTX_WALK_AUTO) */
	RTX_OPT_BVH_LEAF = 2,    /* most primitives per BVH2 leaf, 1..16 (build; default 1) */
	RTX_OPT_SPSORT = 3,      /* 1: shade points in Morton order for k_shadow (default); 0: emission order */
	RTX_OPT_SHADOW_SLOT = 4, /* k_shadow lanes per shade-point slot: 0 = automatic (default), else a power of two <= 64 */
	RTX_OPT_SHADOW_GRAB = 5, /* lane slots per k_shadow work-queue grab, >= 1 (default 4096) */
	RTX_OPT_SHADOW_LDS_STACK = 6, /* 8-wide walk: lane-stack entries kept in LDS, 1..8 (default 8); deeper
	                               * ones spill to HBM (tests use 1 to exercise the spill on any tree) */
	RTX_OPT_TRACE_WALK = 7,       /* closest hits (k_trace): RTX_WALK_AUTO (the 8-wide tree when built,
	                               * default), RTX_WALK_W8 or RTX_WALK_BVH2 (the float BVH2) */
	RTX_OPT_TREE_FRAME = 8,       /* RTX_FRAME_* (build; default RTX_FRAME_AUTO) */
	RTX_OPT_CHUNK_TILES = 9,      /* most 8x8 tiles per chunk of a render (0 = as many as the shade-point budget,
	                               * a third of free HBM, allows; default 0) */
	RTX_OPT_SP_PER_TILE = 10,     /* shade points per tile a chunk is sized for (0 = automatic, default): a
	                               * chunk that overflows is halved and retried, so any value gives the same
	                               * image (tests drive the overflow path with a low one) */
	RTX_OPT_SHADOW_CULL = 11      /* 1 (default): a packet of one shade point's light samples skips the 8-wide
	                               * walk when the cone from the point around the light's bounding sphere
	                               * meets no box of the tree's top two levels (the walk would find nothing,
	                               * so the image is the same); 2: packets of several points (points with
	                               * fewer than 64 samples) too, when every lane's point is clear for its
	                               * emitter (emitters 0..7); 0: every packet walks */
};
int rtx_set_option(rtx_ctx *ctx, int option, int64_t value);
/* The frame rtx_upload_scene builds the scene's BVHs in under RTX_FRAME_AUTO (a diagnostic; no
 * device needed): *rotated = 0 for the world axes, else rot = R (rows, x' = R (x - center)) and
 * *cost_ratio = its sampled leaf-box surface area over the world frame's.  Every primitive is
 * still tested in world space: the frame changes which boxes a ray meets, not any hit. */
int rtx_tree_frame(const rtx_scene_desc *scene, int *rotated, float rot[9], float center[3], double *cost_ratio);
void rtx_close(rtx_ctx *ctx);
const char *rtx_last_error(void);
/* Diagnostics (tests): the uploaded 8-wide tree's 64-byte entries (csrc/rtx_device.h DW8) copied to
 * host memory, at most `capacity` of them; *count = the tree's entry count (0: no 8-wide tree),
 * frame[6] = its 16-bit frame (origin, scale per axis).  entries may be NULL to query the count. */
int rtx_read_wide_tree(rtx_ctx *ctx, void *entries, uint32_t capacity, uint32_t *count, float frame[6]);

/*
 * Several devices rendering one frame (the reference's own parallel point is
 * the OpenMP row loop of render.c:349-352).  The group builds the scene's BVHs once, on its
 * first device (rtx_upload_scene's work: device SAH build, 8-wide collapse), and the other
 * devices copy the built records and trees from it over xGMI (peer access enabled at open, one
 * host thread per device); rtx_group_render deals the frame's 8x8 tiles round-robin (tile t ->
 * device t % n), renders every shard on its own host thread, packs each shard into 16-byte
 * {r, g, b, z} records (64 per tile) and gathers them to the first device over RCCL (grouped
 * ncclSend / ncclRecv on xGMI), which unpacks the frame and copies it to the caller.  Pixels
 * are independent and the RNG is counter-based, so the frame is bit-identical for any n.  One
 * host thread calls the group; it must not be shared.
 */
typedef struct rtx_group rtx_group;
enum { RTX_TRANSPORT_NONE = 0, RTX_TRANSPORT_RCCL = 1, RTX_TRANSPORT_LOOPBACK = 2, RTX_TRANSPORT_RCCL_SELF = 3 };

/* n devices: devices[0..n-1], or 0..n-1 when devices is NULL (each must be gfx950, distinct) */
int rtx_group_open(int n, const int *devices, rtx_group **out);
/* Test transport: a group of n shards as n contexts on ONE device.  Everything is the group's
 * own path (scene built once and copied to every context from one host thread each, one host
 * thread per shard, tile pack, unpack, statistics) except the gather, which is a device-to-device
 * copy in place of RCCL send/recv.  Lets a one-GPU machine check rtx_group_render at any n. */
int rtx_group_open_loopback(int n, int device, rtx_group **out);
/* Test transport: a group of ONE device whose gather still runs the RCCL calls: a one-rank
 * communicator (ncclCommInitAll), shard 0 packed, sent to itself with the grouped ncclSend /
 * ncclRecv of rtx_group_render into a NaN-filled buffer and unpacked over the frame.  Lets a
 * one-GPU machine execute the group's RCCL code; the image must equal rtx_render's. */
int rtx_group_open_rccl_self(int device, rtx_group **out);
int rtx_group_size(const rtx_group *g);
int rtx_group_set_builder(rtx_group *g, int builder);
int rtx_group_set_option(rtx_group *g, int option, int64_t value); /* rtx_set_option on every device */
int rtx_group_upload_scene(rtx_group *g, const rtx_scene_desc *scene);
/* params->tile_offset / tile_stride must be 0 / 1: the group shards the frame itself.
 * rgb / z: HOST buffers as for rtx_render (either may be NULL). */
int rtx_group_render(rtx_group *g, const rtx_frame *frame, const rtx_params *params, float *rgb, float *z);
/* ray and traversal counts summed over the devices, kernel times the slowest device's,
 * gather_ms the pack + RCCL + unpack time */
int rtx_group_get_stats(const rtx_group *g, rtx_stats *out);
/* the statistics of device r (0 <= r < rtx_group_size) for the last frame */
int rtx_group_device_stats(const rtx_group *g, int r, rtx_stats *out);
/* What the runtime reports about member r, read back rather than assumed (a line that claims N
 * devices can show that N communicators of one clique formed on N distinct devices) */
typedef struct rtx_group_member {
	int32_t device;           /* the HIP device ordinal of member r */
	int32_t comm_count;       /* ncclCommCount of its RCCL communicator (0: none, n = 1 or loopback) */
	int32_t comm_rank;        /* ncclCommUserRank (-1: none) */
	int32_t comm_device;      /* ncclCommCuDevice (-1: none) */
	uint32_t can_access_peer0; /* hipDeviceCanAccessPeer(device, device of member 0) */
	uint32_t peer0_can_access; /* hipDeviceCanAccessPeer(device of member 0, device) */
	uint32_t peer_enabled;    /* peer access enabled both ways at rtx_group_open (1 for member 0) */
	uint32_t transport;       /* RTX_TRANSPORT_* */
	char pci_bus_id[32];      /* hipDeviceGetPCIBusId */
} rtx_group_member;
int rtx_group_member_info(const rtx_group *g, int r, rtx_group_member *out);
void rtx_group_close(rtx_group *g);

/* The gather's tile records (rtx_tiles.h): shard `offset` of `stride` of a W x H frame packs
 * to rtx_tile_pack_count() records of 4 floats.  Host reference and device versions. */
size_t rtx_tile_pack_count(uint32_t width, uint32_t height, uint32_t offset, uint32_t stride);
int rtx_tile_pack_host(const float *rgb, const float *z, uint32_t width, uint32_t height, uint32_t offset,
		       uint32_t stride, float *out);
int rtx_tile_unpack_host(const float *in, uint32_t width, uint32_t height, uint32_t offset, uint32_t stride,
			 float *rgb, float *z);
int rtx_tile_pack_device(rtx_ctx *ctx, const void *d_rgb, const void *d_z, uint32_t width, uint32_t height,
			 uint32_t offset, uint32_t stride, void *d_out, void *stream);
int rtx_tile_unpack_device(rtx_ctx *ctx, const void *d_in, uint32_t width, uint32_t height, uint32_t offset,
			   uint32_t stride, void *d_rgb, void *d_z, void *stream);

/*
 * Postprocess: the reference's separate `postprocess` binary
 * (src/postprocess/postproc.c:36-188) applied on the device to an rgb+z frame:
 * brighten (-b), depth of field (--dof scale bias | --dof-camera aperture focal plane),
 * mist (--mist start depth falloff r g b), in that order, with the reference's float
 * arithmetic; the DoF scatter is restated as an ordered gather so every output pixel
 * sums its contributions in the reference's order (bit-identical results).
 */
enum { RTX_DOF_NONE = 0, RTX_DOF_SCALE_BIAS = 1, RTX_DOF_CAMERA = 2 };
enum { RTX_FALLOFF_QUAD = 0, RTX_FALLOFF_LIN = 1, RTX_FALLOFF_INV_QUAD = 2 };

typedef struct rtx_post {
	int32_t brighten;           /* -b given (postproc.c:43-47) */
	float brighten_factor;
	int32_t dof;                /* RTX_DOF_* (postproc.c:49-68) */
	float dof_scale, dof_bias;  /* --dof */
	float aperture, focal_length, plane_in_focus; /* --dof-camera */
	int32_t mist;               /* --mist given (postproc.c:70-90) */
	float mist_start, mist_depth;
	int32_t mist_falloff;       /* RTX_FALLOFF_* */
	float mist_color[3];
} rtx_post;

/* rgb[W*H*3] in/out and z[W*H] in, HOST buffers (replaces postprocess() between
 * image_load() and save_image(), src/postprocess/main.c:66-68). */
int rtx_postprocess(rtx_ctx *ctx, uint32_t width, uint32_t height, const rtx_post *post, float *rgb, const float *z);
/* Same on DEVICE buffers, enqueued on `stream` (NULL = the context's stream); synchronises it. */
int rtx_postprocess_device(rtx_ctx *ctx, uint32_t width, uint32_t height, const rtx_post *post, void *d_rgb,
			   const void *d_z, void *stream);

/*
 * Known-answer entry: evaluates one device function over n inputs on the GPU
 * (used by the -m gpu parity tests against the oracle's KAT fixtures).
 * kind / record layouts are listed in rtx_kat.h.
 */
int rtx_kat(int kind, uint32_t n, const float *in, float *out, const rtx_params *params);

#ifdef __cplusplus
}
#endif

#endif /* RTX_H */
