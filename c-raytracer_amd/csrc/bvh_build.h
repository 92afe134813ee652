/*
 * Host BVH builder for the device layout of rtx_device.h.
 *
 * Replaces accel_init (accel.c:266-315).  The reference builds a Morton-code
 * LBVH with one object per leaf; closest-hit and any-hit answers do not depend
 * on the tree (up to exact ties), so this builder is free to optimise traversal
 * cost: binned SAH over all three axes, leaves of up to `max_leaf` objects,
 * depth capped (median splits near the cap) so per-lane LDS stacks are bounded.
 */
#ifndef RTX_BVH_BUILD_H
#define RTX_BVH_BUILD_H

#include <stdint.h>
#include <vector>

#include "rtx_device.h"

struct BvhInput {
	uint32_t n;
	const float *lo; /* n*3 */
	const float *hi; /* n*3 */
};

struct BvhOutput {
	std::vector<DNode> nodes;     /* inner nodes, depth-first; nodes[0] = root when root_ref is inner */
	std::vector<uint32_t> order;  /* leaf order: order[i] = input primitive index */
	uint32_t root_ref = RTX_EMPTY_REF;
	uint32_t depth = 0;           /* max inner-node depth (root = 1) */
	uint32_t leaves = 0;
};

#ifndef RTX_BVH_BINS
#define RTX_BVH_BINS 32
#endif
struct BvhConfig {
	uint32_t max_leaf = 1; /* single-primitive leaves: fewest shadow-walk steps on the bench frame (1078 vs 1239 ms at 4) */
	uint32_t bins = RTX_BVH_BINS;
	uint32_t max_depth = 48;
	float c_trav = 1.0f;
	float c_isect = 1.0f;
};

void bvh_build(const BvhInput &in, const BvhConfig &cfg, BvhOutput &out);

#endif
