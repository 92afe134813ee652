/*
 * Tile sharding and the packed tile records of the multi-device gather (rtx_group_render),
 * shared by the host reference (rtx_api.cpp rtx_tile_pack_host) and the device kernels
 * (rtx_gather.hip), so both index pixels identically.
 *
 * A frame is cut into 8x8-pixel tiles, row-major (render.c:349-352 walks rows; the tiles are
 * this build's unit of work).  Shard `off` of `stride` owns tiles t = off, off + stride, ...
 * (rtx_params.tile_offset / tile_stride).  Its packed form is 64 records of 16 bytes per tile,
 * {r, g, b, z} in the tile's row-major pixel order; pixels outside the frame pack as zeros.
 */
#ifndef RTX_TILES_H
#define RTX_TILES_H

#include <stdint.h>

#if defined(__HIPCC__)
#define RTX_TD __host__ __device__ __forceinline__
#else
#define RTX_TD static inline
#endif

#define RTX_TILE_PX 64u

RTX_TD uint32_t rtx_tiles_x(uint32_t w) { return (w + 7u) / 8u; }
RTX_TD uint64_t rtx_tiles_total(uint32_t w, uint32_t h) { return (uint64_t)rtx_tiles_x(w) * ((h + 7u) / 8u); }

/* tiles of shard off of stride */
RTX_TD uint32_t rtx_shard_tiles(uint32_t w, uint32_t h, uint32_t off, uint32_t stride)
{
	const uint64_t t = rtx_tiles_total(w, h);
	return off < t ? (uint32_t)((t - off + stride - 1) / stride) : 0u;
}

/* pixel of record i (= k * 64 + p: tile k of the shard, pixel p of the tile) */
RTX_TD void rtx_shard_pixel(uint32_t i, uint32_t tiles_x, uint32_t off, uint32_t stride, uint32_t *x, uint32_t *y)
{
	const uint32_t t = off + (i >> 6) * stride, p = i & 63u;
	*x = (t % tiles_x) * 8u + (p & 7u);
	*y = (t / tiles_x) * 8u + (p >> 3);
}

#endif
