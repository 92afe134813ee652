/*
 * Device-side scene layout in HBM (shared by the host uploader and the kernels).
 *
 *  DNode  64 B  BVH2 inner node: both children's AABBs + child refs + the
 *               child order per ray-direction octant.  A ref is the byte offset
 *               of the child's 64-byte record from `nodes` (64-aligned), with
 *               RTX_REF_LEAF | RTX_REF_SPH (has a sphere) | (count-1) in its
 *               low bits for a leaf of count
 *               <= 16 primitives contiguous in the record array (primitive i
 *               is record num_nodes + i).
 *               Replaces the pointer-linked struct BVH + malloc'd BoundingCuboid
 *               of accel.c:25-40.  Nodes are stored depth-first (left child
 *               adjacent) so a traversal walks forward through memory.
 *  DPrim  64 B  one bounded object (sphere / triangle) in BVH leaf order:
 *               a = (v0 | centre, epsilon), b = (e1 | (r,0,0), object id bits),
 *               c = (e2, meta bits = material | transparent << 23 | type << 24),
 *               d = (normal, 0).  The primitives follow the nodes in one
 *               allocation (record index nnodes + i), so the shadow walk
 *               addresses both through one base pointer.
 *               Shadow tests read a..c (48 B); d only for the final closest hit.
 *  DPlane 32 B  unbound objects (object.c:168-197), linear scan, never in the BVH.
 *  DMaterial    material + texture parameters (material.c:27-53).
 *  DEmitter     emittant_objects[] entry with ke/num_lights premultiplied
 *               (render.c:175).
 * Hit ids: prim index, or RTX_PLANE_BIT | plane index; RTX_NONE = no object.
 */
#ifndef RTX_DEVICE_H
#define RTX_DEVICE_H

#include <stdint.h>

/* Measurement builds (tools/variants.sh EXTRA=-DRTX_MEASURE=1) read a few RTX_* environment knobs
 * (occupancy, LDS padding); the product library's behaviour never depends on the environment. */
#ifndef RTX_MEASURE
#define RTX_MEASURE 0
#endif

#define RTX_LEAF_BIT 0x80000000u  /* builder-side leaf refs (bvh_build.cpp) */
#define RTX_REF_LEAF 32u          /* device refs: byte offset | leaf flag | sphere flag | count-1 */
#define RTX_REF_SPH 16u           /* leaf holds at least one sphere (else triangles only) */
#define RTX_REF_CNT 15u
#define RTX_REF_OFF (~63u)
#define RTX_PLANE_BIT 0x80000000u
#define RTX_SP_FAR 0x80000000u    /* shade-point record, object word: the point is far from the bounded
                                   * objects (rtx_math.h tf_far), k_shadow walks from the light end */
#define RTX_NONE 0xFFFFFFFFu
#define RTX_EMPTY_REF 0xFFFFFFFFu /* BVH with no bounded objects */
#define RTX_MAX_LEAF 16

/* DPrim meta word (c[3]): material | transparent flag | type << 24 */
#define RTX_META_MAT 0x7FFFFFu
#define RTX_META_TRANSPARENT 0x800000u

#define RTX_MF_EMITTANT 1
#define RTX_MF_REFLECTIVE 2
#define RTX_MF_TRANSPARENT 4

#define RTX_TILE_W 8
#define RTX_TILE_H 8

typedef struct __attribute__((aligned(64))) DNode {
	float lo0x, hi0x, lo0y, hi0y;
	float lo0z, hi0z, lo1x, hi1x;
	float lo1y, hi1y, lo1z, hi1z;
	uint32_t ref0, ref1;
	uint32_t order; /* bit o: left child first for direction octant o (bit a of o: dir[a] >= 0) */
	uint32_t pad;
} DNode;

typedef struct __attribute__((aligned(64))) DPrim {
	float a[4];
	float b[4];
	float c[4];
	float d[4];
} DPrim;

/* threaded (skip-link) copy of the BVH for the ray-by-ray shadow walk: one 16-byte record per
 * BVH node in preorder, so a node is ONE 16-byte vector load.
 *   x, y, z: the node's box (its parent's child slot; the scene bound for the root) quantised
 *            to 16 bits per plane in the frame of the bounded objects' box,
 *            q = (coordinate - qo) * qs, lo rounded down and hi up, then widened by one step
 *            (conservative; lo in the low half, hi in the high half)
 *   link:    inner node: index of the node after its subtree << 6 (where a missed box
 *            continues; a hit continues at the first child, the next record);
 *            leaf: its device ref (record byte offset | RTX_REF_LEAF | RTX_REF_SPH | count-1),
 *            and the walk continues at the next record whether the box is hit or not.
 * Any-hit needs no visit order, so no stack: the walk ends at index num_qnodes. */
typedef struct __attribute__((aligned(16))) DQNode {
	uint32_t x, y, z;
	uint32_t link;
} DQNode;

/* The threaded BVH's top levels, copied to LDS once per k_shadow workgroup (DScene.top):
 * num_top 16-byte records (x, y, z as in DQNode, for every node shallower than the cut depth,
 * in preorder), then num_top 32-bit words.  Record link: a leaf's ref (the walk continues at
 * the next top record); an inner node above the cut: the top index after its top subtree << 6;
 * a cut node (an inner node whose children lie below the cut): its first child's DQNode index
 * << 6 | RTX_QTOP_CUT, and its word = the DQNode index after its subtree.  A hit on a cut
 * node walks that DQNode range, then continues at the next top record. */
#define RTX_QTOP_CUT 1u
#ifndef RTX_TOP_MAX
#define RTX_TOP_MAX 2048 /* top records per workgroup (20 B each in LDS) */
#endif
#ifndef RTX_SH_NW
#define RTX_SH_NW 16 /* waves per k_shadow workgroup (they share the top copy) */
#endif

/* The trees' frame.  Every BVH of a scene (the BVH2 records, the threaded copy, the 8-wide tree)
 * is built over leaf boxes taken in one frame x' = R (x - c): R's rows are the frame's axes in
 * world coordinates, c the centre of the bounded objects' world box.  The uploader picks R from
 * the triangles (rtx_frame.cpp: the frame of least total leaf-box surface area among the identity
 * and the frames of the largest triangles, e.g. a rotated mesh's own axes, where its faces have
 * flat boxes), so R need not be the identity.  A walk transforms its ray once (origin and
 * direction; the parameter t is unchanged, the map is linear) and tests boxes in that frame;
 * primitives are always tested in world space with the reference's arithmetic.  Leaf boxes are
 * padded for the transform's rounding (rtx_frame.cpp), so the culling stays conservative.
 * rotated = 0: R = I, c = 0, and the walks skip the transform (the world-space trees). */
typedef struct DTreeFrame {
	float r[3][3];
	float c[3];
	uint32_t rotated;
	float rad;   /* the largest |x - centre| component over the bounded objects' world box
	              * (rtx_frame_radius), the centre being c + cf: ray origins farther than
	              * RTX_FRAME_FAR * rad from it (in the frame's max-norm, rtx_math.h tf_far) are
	              * handled by tf_shift / tf_point_at, as the boxes' padding covers the slab test's
	              * rounding only for origins near the objects */
	float cf[3]; /* that centre in the frame's coordinates: 0 for a rotated frame (c is the centre),
	              * the world box's centre for the world frame (c = 0) */
} DTreeFrame;

/* 8-wide compressed BVH for the shadow walk (rtx_shadow.hip shadow_walk8), in the style of
 * Ylitie et al.'s compressed wide BVH: an array of 64-byte entries (one 64-byte half line, four
 * global_load_dwordx4; the scalar path reads the DW8S copy below).  A node entry:
 *   w0 = ox | oy << 16, w1 = oz | ex << 16 | ey << 20 | ez << 24
 *        the node's frame on the 16-bit grid of DQNode: origin o (grid units) and a per-axis step
 *        of 2^e grid units (e <= 9)
 *   w2 = base << 8 | imask      children at entries base + c (c = slot 0..7); imask: inner slots
 *   w3 = vmask | tmask << 8     slots holding a child; leaf slots of transparent primitives
 *   w4..w15: 8-bit planes, slot c = byte c & 3 of the word:  lo_x w4,w5  hi_x w6,w7  lo_y w8,w9
 *            hi_y w10,w11  lo_z w12,w13  hi_z w14,w15
 * Child c's box is [o + lo * 2^e, o + hi * 2^e] on the grid, outward-rounded from its 16-bit box
 * (rtx_quant.h), so it contains the float box.  An empty slot has lo = 255, hi = 0 on every axis
 * (never hit by the octant-specialised test; the generic test masks with vmask).  An inner
 * slot's entry is the child node; a leaf slot's entry is a copy of the primitive's 64-byte DPrim
 * record (one primitive per leaf slot) with its material's kt in place of the normal (the
 * shadow walk needs no normal; a transparent hit multiplies by it without a material fetch)
 * and the primitive's record index in the last word (the closest-hit walk's hit id).  A node's eight child entries are contiguous (unused ones are
 * holes), so a lane's pending siblings are one 32-bit group base << 8 | slot mask.
 * Slots follow the children's centroid octant about the node centre (bit a: the + side of
 * axis a), so a ray of direction octant OCT meets them front to back roughly in the order
 * c ^ (~OCT & 7) = 0, 1, ..., 7; the walk visits hit children in that order.
 * Entry 0 is the root node, entry 1 a hole (blocks start on 128-byte lines).  The tree has its own
 * 16-bit frame (DScene.w8qo / w8qs) over its primitives; the emitters are left out of it when the
 * host has the primitive records (DScene.w8noemit): k_shadow tests them linearly, like planes,
 * so a shadow ray no longer walks down to the light it was cast to. */
#ifndef RTX_W8_STACK
#define RTX_W8_STACK 8     /* k_shadow lane-stack entries in LDS; deeper ones spill to HBM (DScene.w8spill) */
#endif
#define RTX_W8_MAX_ENTRIES (1u << 24)
#define RTX_W8_TOP_LEVELS 3 /* levels of the 8-wide tree k_shadow serves from LDS (root, 8, 64 nodes) */
#define RTX_W8_TOP_MAX 80   /* entries of them at most: 2 + 8 + 64 */
typedef struct __attribute__((aligned(64))) DW8 {
	uint32_t w[16];
} DW8;

/* The scalar-path copy of an 8-wide node (DScene.w8s, indexed like the entries; only node
 * entries are filled): when every walking lane of a wave is at one node, the walks read it
 * through the scalar cache (the header with one s_load_dwordx8, each child's planes with one
 * more) and take the 8-bit plane offsets as ready floats, an axis's two planes as one SGPR pair
 * of a v_pk_fma_f32, instead of converting 48 bytes per lane.  The floats are the bytes' exact
 * values, so both paths compute bit-identical box tests.
 *   w = the node's w0..w3;  org = its origin as floats;  q[c] = child c's plane offsets lo_x,
 *   hi_x, lo_y, hi_y, lo_z, hi_z (bytes c & 3 of w4 + (c >> 2) ... as floats), then two zeros */
typedef struct __attribute__((aligned(32))) DW8S {
	uint32_t w[4];
	float org[3];
	uint32_t pad;
	float q[8][8];
} DW8S;

typedef struct DPlane {
	float n[3];
	float d;
	float eps;
	uint32_t obj;
	uint32_t mat;
	uint32_t transparent; /* its material's RTX_MF_TRANSPARENT, copied for the shadow test */
	float kt[3];          /* its material's kt (shadow transmittance), copied likewise */
	uint32_t pad;
} DPlane;

typedef struct DMaterial {
	float ks[3], ka[3], kr[3], kt[3], ke[3];
	float shininess, ior;
	int32_t tex, periodic;
	float color[2][3];
	float scale, mortar, nfs, ns, fs;
	uint32_t flags;
	float pad[2];
} DMaterial;

typedef struct DEmitter {
	uint32_t obj;      /* reference object index (emittant_objects[i]) */
	uint32_t type;     /* RTX_SPHERE / RTX_TRIANGLE */
	uint32_t num_lights;
	float li[3];       /* ke * (1 / num_lights) */
	float p0[3], p1[3], p2[3];
	float radius;
	float e1[3], e2[3]; /* triangle edges (object.c:331-334), for the shadow test of emitters kept */
	float eps;          /* out of the 8-wide shadow tree (DScene.w8noemit) */
	uint32_t transparent;
	float kt[3];
	uint32_t prim;      /* its primitive record index (closest hits of the 8-wide walk) */
	float wlo[3], whi[3]; /* its padded world box (rtx_world_box): tested before the object by rays from
	                       * far origins, whose intersector arithmetic is not to be trusted far off it
	                       * (the reference's own tree culls by this box before object_intersects) */
} DEmitter;

#define RTX_MAX_EMITTERS 64

typedef struct DScene {
	const DNode *nodes;
	const DPrim *prims;
	const DPlane *planes;
	const DMaterial *mats;
	const DEmitter *emitters;
	const DQNode *qnodes;   /* threaded quantised BVH (num_qnodes records), null when the BVH is empty */
	uint32_t num_qnodes;
	float qo[3], qs[3];     /* its quantisation frame: q = (x' - qo) * qs, x' in the trees' frame tf */
	const uint32_t *top;    /* its top levels (num_top records + num_top words, see RTX_QTOP_CUT) */
	uint32_t num_top;
	const DW8 *w8;          /* 8-wide compressed BVH (num_w8 entries), null when not built */
	uint32_t num_w8, w8depth;
	uint32_t w8top;         /* entries [0, w8top): the tree's levels 0..RTX_W8_TOP_LEVELS-1 (the device collapse
	                         * lays levels out breadth-first), which k_shadow copies to LDS; 0: none */
	float w8qo[3], w8qs[3]; /* its 16-bit frame */
	const DW8S *w8s;        /* scalar-path copies of its nodes (num_w8 slots, node entries filled) */
	uint32_t trace_w8;      /* k_trace walks the 8-wide tree for closest hits (else the float BVH2) */
	uint32_t w8noemit;      /* the emitters are not in it (k_shadow tests them linearly) */
	uint32_t w8sph;         /* it holds spheres (else k_shadow's leaf tests are the triangle's alone) */
	const DEmitter *lin;    /* tiny scenes (RTX_WALK_LINEAR): every bounded object as a record k_shadow tests
	                         * one by one like the planes (object order), no walk; null otherwise */
	uint32_t num_lin;
	uint32_t *w8spill;      /* k_shadow lane-stack entries from RTX_W8_STACK on, [entry][grid lane] */
	uint32_t w8spill_lanes; /* grid lanes the spill area was sized for (0: no spill area) */
	uint32_t w8lstk;        /* lane-stack entries k_shadow keeps in LDS (<= RTX_W8_STACK) */
	uint32_t root_ref;
	uint32_t num_nodes;    /* prims == (const DPrim *)(nodes + num_nodes) */
	uint32_t num_prims;
	uint32_t num_planes;
	uint32_t num_emitters;
	uint32_t stack_size;   /* per-lane closest-hit stack entries (>= BVH depth) */
	float ambient[3];
	uint32_t *ostk;        /* k_trace: lane-stack entries from RTX_TRACE_LSTK on, [entry][grid lane] in HBM */
	DTreeFrame tf;         /* the frame every tree's boxes are in (identity unless rotated) */
	const float *cull;     /* k_shadow's cone cull (RTX_OPT_SHADOW_CULL): bounding spheres {world centre,
	                        * radius} (4 floats each) of the 8-wide tree's second level (a root slot's children, or the
	                        * slot's own box when it is a leaf), at most RTX_CULL_MAX; every primitive of
	                        * the tree lies in one.  Null / 0: no cull */
	uint32_t num_cull;
	uint32_t cull_slots;   /* RTX_OPT_SHADOW_CULL 2: the lane-slot path culls too (cone_mask_lane) */
} DScene;
#define RTX_CULL_MAX 64

/* k_trace keeps the first RTX_TRACE_LSTK entries of a lane's closest-hit stack in LDS and the
 * deeper ones (rare) in HBM (DScene.ostk): the LDS per wave, not the tree depth, sets how many
 * waves a CU holds, and the kernel is latency-bound */
#ifndef RTX_TRACE_LSTK
#define RTX_TRACE_LSTK 9
#endif

typedef struct DFrame {
	uint32_t width, height;
	float corner[3], step_x[3], step_y[3], origin[3];
} DFrame;

typedef struct DParams {
	uint32_t max_bounces;
	float min_intensity_sqr;
	int32_t reflection, gi;
	uint32_t samples;
	int32_t attenuation;
	float att_offset;
	int32_t rng;
	uint64_t seed;
	int32_t u32conv;
	uint32_t tile_offset, tile_stride;
	uint32_t ntiles;       /* tiles this launch renders */
	uint32_t tiles_x;
} DParams;

/* secondary (reflection / refraction) ray waiting in a wave's task stack */
typedef struct DTask {
	float o[3];
	float d[3];
	float kr[3];
	uint32_t rb;
	uint32_t inside;
	uint32_t key_lo, key_hi;
	uint32_t slot;
} DTask;

/* counters written by the kernels; all of them are reset at the start of every chunk and read
 * back after it, so a chunk that is retried (staging overflow) never counts twice */
enum {
	RTX_C_TILE = 0,     /* k_trace work queue head */
	RTX_C_SPCOUNT,      /* shade points emitted */
	RTX_C_OVERFLOW,     /* per-tile shade-point staging overflow (host retries with more staging) */
	RTX_C_TASKOVERFLOW, /* reflection/refraction task-stack overflow (host fails: bounded by design) */
	RTX_C_SPOVERFLOW,   /* chunk shade-point array overflow (host retries with fewer tiles) */
	RTX_C_SPQUEUE,      /* k_shadow work queue head */
	RTX_C_CLOSEST,      /* cast_ray() calls */
	RTX_C_SHADOW,       /* is_light_blocked() calls */
	RTX_C_NODES,        /* closest-hit traversal counts (count mode) */
	RTX_C_TRIS,
	RTX_C_SPHERES,
	RTX_C_PLANES,
	RTX_C_SBOXES,       /* shadow walk (count mode): box tests summed over rays */
	RTX_C_SGBOXES,      /* ... of which read from the DQNode array (the rest from the LDS top) */
	RTX_C_STRIS,        /* ... primitive tests */
	RTX_C_SSPHERES,
	RTX_C_SPLANES,
	RTX_C_SSTEPS,       /* ... walk-loop iterations of the waves */
	RTX_C_SWALKS,       /* ... wave walks (64 shadow rays each) */
	RTX_C_SLEAFR,       /* ... 8-wide walk: wave iterations of the leaf loops (rounds of primitive fetches) */
	RTX_C_SUNIF,        /* ... 8-wide walk: wave steps whose active lanes were all at one node */
	RTX_C_FARC,         /* count mode: closest-hit rays whose origin was far (rtx_math.h tf_far: tf_shift) */
	RTX_C_FARS,         /* count mode: shadow rays from far shade points (walked from the light end) */
	RTX_C_SSPILL,       /* count mode, 8-wide walk: lane-stack pushes beyond the LDS entries (HBM) */
	RTX_C_SCLEAR,       /* count mode: shadow rays of packets the cone cull let skip the walk */
	RTX_C_N
};

#endif
