"""Multi-rank tile sharding + framebuffer gather to rank 0 (rtxpy.dist, used by bench.py over RCCL),
exercised with the gloo backend on CPU at world_size 2 and 3.  Each rank renders its
tiles with the CPU oracle (test infrastructure standing in for the GPU here); the
gathered frame must be bit-identical to a single-rank render."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir, host_staging=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "c-raytracer_amd"))
    sys.path.insert(0, os.path.join(root, "tests"))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    import conftest as C
    from rtxpy import oracle
    from rtxpy.dist import Gatherer
    scene, frame, params, _ = C.load_config("s3_amb")
    params.tile_offset, params.tile_stride = rank, world
    rgb, z, counts = oracle.render(scene, frame, params, threads=1)
    g = Gatherer(frame.width, frame.height, rank, world, torch.device("cpu"), host_staging=host_staging)
    out = g.gather(torch.from_numpy(rgb.reshape(-1, 3)), torch.from_numpy(z.reshape(-1)))
    assert (out is None) == (rank != 0)  # gathered to rank 0 only
    c = torch.tensor(counts, dtype=torch.int64)
    torch.distributed.all_reduce(c)
    if rank == 0:
        full_rgb, full_z = out
        np.savez(os.path.join(out_dir, "gathered.npz"), rgb=full_rgb.numpy(), z=full_z.numpy(), counts=c.numpy())
    torch.distributed.destroy_process_group()


@pytest.mark.parametrize("world,host_staging", [(2, False), (3, False), (2, True)])
def test_gloo_tile_gather_bit_exact(tmp_path, world, host_staging):
    """host_staging: the gather through host tensors (bench.py RTX_BENCH_REHEARSE=gloo)"""
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path), host_staging), nprocs=world, join=True,
                       start_method="spawn")
    import conftest as C
    from rtxpy import oracle
    scene, frame, params, _ = C.load_config("s3_amb")
    rgb, z, counts = oracle.render(scene, frame, params, threads=1)
    d = np.load(tmp_path / "gathered.npz")
    assert np.array_equal(d["rgb"], rgb.reshape(-1, 3)) and np.array_equal(d["z"], z.reshape(-1))
    assert tuple(d["counts"]) == counts


def test_rank_tiles_partition():
    from rtxpy.dist import rank_tiles, tile_grid
    for w, h, n in [(1920, 1080, 8), (13, 7, 3), (8, 8, 4)]:
        tx, ty = tile_grid(w, h)
        allt = np.sort(np.concatenate([rank_tiles(w, h, r, n) for r in range(n)]))
        assert np.array_equal(allt, np.arange(tx * ty))
