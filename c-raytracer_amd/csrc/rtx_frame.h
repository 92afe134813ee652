/*
 * The trees' frame (rtx_device.h DTreeFrame, rtx_frame.cpp): choosing it for a scene and the
 * leaf boxes in it.  Library-internal (librtx); the public diagnostic is rtx_tree_frame (rtx.h).
 */
#ifndef RTX_FRAME_H
#define RTX_FRAME_H

#include <functional>
#include <vector>

#include "rtx.h"
#include "rtx_device.h"

int rtx_fail(int code, const char *fmt, ...);

/* f(begin, end, chunk) over [0, n) in contiguous chunks of at least `grain` items on host threads
 * (RTX_HOST_THREADS, else OMP_NUM_THREADS, else at most 16; serially when n < 2 grain, and on this
 * thread when no more can start); returns the chunk count */
unsigned rtx_host_parallel(size_t n, const std::function<void(size_t, size_t, unsigned)> &f, size_t grain = 16384);
/* object o's world box (sphere_get_corners / triangle_get_corners, object.c:277-282, 375-388),
 * padded for the walks' FMA slab test */
void rtx_world_box(const rtx_object &o, float lo[3], float hi[3]);
/* the frame for the bounded objects `bounded` of sc (world box lo / hi): F, and its sampled
 * leaf-box cost relative to the identity's (1.0: the identity, F.rotated = 0) */
double rtx_frame_choose(const rtx_scene_desc *sc, const std::vector<uint32_t> &bounded, const float world_lo[3],
			const float world_hi[3], DTreeFrame &F);
/* the largest |x - c| component over the bounded objects' world box world_lo / world_hi (every
 * vertex, every sphere with its radius) */
double rtx_frame_radius(const float world_lo[3], const float world_hi[3], const DTreeFrame &F);
/* F.cf and F.rad for the far-origin test (rtx_math.h tf_far), in either frame */
void rtx_frame_far(const float world_lo[3], const float world_hi[3], DTreeFrame &F);
/* the transform's leaf-box padding for a scene of that radius */
double rtx_frame_pad(double radius);
/* object o's box in frame F (F.rotated), rounded outward and padded by pad plus the relative
 * padding of rtx_world_box */
void rtx_frame_box(const rtx_object &o, const DTreeFrame &F, double pad, float lo[3], float hi[3]);
/* rtx_frame_box of every object in `bounded` (lo / hi: 3 floats each), and their union blo / bhi
 * (host threads; the boxes do not depend on the thread count) */
void rtx_frame_boxes(const rtx_scene_desc *sc, const std::vector<uint32_t> &bounded, const DTreeFrame &F, double pad,
		     float *lo, float *hi, float blo[3], float bhi[3]);
/* rtx_world_box of every object in `bounded`, and their union */
void rtx_world_boxes(const rtx_scene_desc *sc, const std::vector<uint32_t> &bounded, float *lo, float *hi, float blo[3],
		     float bhi[3]);

#endif
