"""Tile sharding across ranks and the framebuffer gather.

Tiles are 8x8 pixels, row-major over the frame; rank r of N renders the tiles
t with t % N == r (rtx_params.tile_offset / tile_stride).  Interleaving deals
the expensive centre of the frame to every rank.  After rendering, each rank
packs its tiles (rgb + z = 16 B per pixel) into one contiguous buffer and the
buffers are gathered (torch.distributed.gather: RCCL over xGMI with the "nccl" backend
on GPUs, gloo in the CPU tests) to rank 0, which unpacks: one message of 16 B x max_tiles x 64 per rank
(4.1 MB / N at 1080p).  The only collective is this exchange: pixels are independent, so
there is no reduction.
"""
import numpy as np
import torch

TILE = 8


def tile_grid(width, height):
    return (width + TILE - 1) // TILE, (height + TILE - 1) // TILE


def rank_tiles(width, height, rank, world):
    tx, ty = tile_grid(width, height)
    return np.arange(rank, tx * ty, world, dtype=np.int64)


def tile_pixel_index(width, height, tiles):
    """(len(tiles), 64) flat pixel indices (-1 for pixels outside the frame)."""
    tx, _ = tile_grid(width, height)
    tiles = np.asarray(tiles, np.int64)
    lx = np.arange(64) % TILE
    ly = np.arange(64) // TILE
    x = (tiles % tx)[:, None] * TILE + lx[None, :]
    y = (tiles // tx)[:, None] * TILE + ly[None, :]
    idx = y * width + x
    idx[(x >= width) | (y >= height)] = -1
    return idx


class Gatherer:
    """Packs / gathers (to rank 0) / unpacks one rank's tiles.  Works on any device torch supports."""

    def __init__(self, width, height, rank, world, device, host_staging=False):
        """host_staging: the process group's backend reduces host tensors only (gloo with ranks
        on GPUs, bench.py's RTX_BENCH_REHEARSE): the packed tiles are gathered through host memory"""
        self.w, self.h, self.rank, self.world = width, height, rank, world
        self.device = device
        self.host_staging = host_staging
        counts = [len(rank_tiles(width, height, r, world)) for r in range(world)]
        self.max_tiles = max(counts) if counts else 0
        idx = np.full((self.max_tiles, 64), -1, np.int64)
        mine = tile_pixel_index(width, height, rank_tiles(width, height, rank, world))
        idx[:mine.shape[0]] = mine
        self.mine = torch.from_numpy(idx.reshape(-1)).to(device)
        self.valid = self.mine >= 0
        self.safe = torch.where(self.valid, self.mine, torch.zeros_like(self.mine))
        all_idx = []
        for r in range(world):
            a = np.full((self.max_tiles, 64), -1, np.int64)
            t = tile_pixel_index(width, height, rank_tiles(width, height, r, world))
            a[:t.shape[0]] = t
            all_idx.append(a.reshape(-1))
        self.all_idx = torch.from_numpy(np.concatenate(all_idx)).to(device)
        self.all_valid = self.all_idx >= 0
        self.packed = torch.empty((self.max_tiles * 64, 4), dtype=torch.float32, device=device)
        self.gathered = torch.empty((world * self.max_tiles * 64, 4), dtype=torch.float32, device=device)
        self.parts = list(self.gathered.chunk(world)) if world > 1 else None
        self.message_bytes = self.max_tiles * 64 * 16

    def pack(self, rgb_flat, z_flat):
        """rgb_flat: (W*H, 3), z_flat: (W*H,) tensors on self.device."""
        self.packed[:, :3] = rgb_flat[self.safe]
        self.packed[:, 3] = z_flat[self.safe]
        self.packed[~self.valid] = 0.0
        return self.packed

    def gather(self, rgb_flat, z_flat, group=None):
        """Gather every rank's tiles to rank 0: returns the full (W*H,3), (W*H,) frame on rank 0,
        None elsewhere."""
        packed = self.pack(rgb_flat, z_flat)
        if self.world == 1:
            self.gathered.copy_(packed)
        elif self.host_staging:
            h = packed.cpu()
            parts = [torch.empty_like(h) for _ in range(self.world)] if self.rank == 0 else None
            torch.distributed.gather(h, parts, dst=0, group=group)
            if self.rank != 0:
                return None
            self.gathered.copy_(torch.cat(parts))
        else:
            torch.distributed.gather(packed, self.parts if self.rank == 0 else None, dst=0, group=group)
            if self.rank != 0:
                return None
        return self.unpack(self.gathered)

    def unpack(self, gathered):
        rgb = torch.zeros((self.w * self.h, 3), dtype=torch.float32, device=self.device)
        z = torch.zeros((self.w * self.h,), dtype=torch.float32, device=self.device)
        sel = self.all_valid
        rgb[self.all_idx[sel]] = gathered[sel, :3]
        z[self.all_idx[sel]] = gathered[sel, 3]
        return rgb, z
