"""The torchrun launch of bench.py (the driver's multi-GPU bench: one rank per GPU, tile shards
gathered to rank 0, the max-over-ranks clock) rehearsed on the one-GPU box: RTX_BENCH_REHEARSE=gloo
runs the same ranks sharing the GPU, gathered over gloo through host memory.  The ranks' rays
together must be exactly the single-rank frame's (every tile rendered once)."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--scene", "scene3", "--width", "256", "--height", "144", "--spp", "4", "--steps", "2", "--warmup", "1",
        "--no-post", "--no-cpu-baseline", "--no-count"]


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _line(out):
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert lines, out[-2000:]
    return json.loads(lines[-1])


@pytest.mark.gpu
@pytest.mark.parametrize("ranks", [2, 3])
def test_gpu_torchrun_ranks_rehearsal(ranks):
    env = dict(os.environ, RTX_BENCH_REHEARSE="gloo", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ranks}",
           "--master-addr", "127.0.0.1", f"--master-port={_port()}", os.path.join(ROOT, "bench.py"),
           "--gpus", str(ranks)] + ARGS
    p = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    multi = _line(p.stdout)
    q = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1"] + ARGS, cwd=ROOT,
                       capture_output=True, text=True, timeout=240)
    assert q.returncode == 0, q.stderr[-3000:]
    one = _line(q.stdout)
    assert multi["ranks"] == ranks and multi["config"]["launch"] == "torchrun" and "rehearsal" in multi
    assert multi["config"]["parallelism"] == f"tiles{ranks}"
    # every tile once: the ranks' rays add up to the single-rank frame's, rank 0 rendered its share
    assert multi["config"]["rays_per_frame"] == one["config"]["rays_per_frame"] == one["config"]["rays_per_frame_rank0"]
    assert 0 < multi["config"]["rays_per_frame_rank0"] < multi["config"]["rays_per_frame"]
    assert multi["value"] > 0 and multi["config"]["gather_message_bytes_per_rank"] > 0
    # the line validates itself: torch.distributed's own world size and backend,
    # every rank reporting, and rank 0's one-GPU frame equal to the gathered one in rays and bits
    v = multi["validation"]
    assert v["ok"] and v["world_size"] == ranks and v["backend"] == "gloo", v["checks"]
    assert [x["rank"] for x in v["ranks"]] == list(range(ranks))
    assert v["rays_per_frame_sum"] == v["one_gpu_frame_rays"] and sum(v["rays_per_frame_sum"]) == one["config"]["rays_per_frame"]
    assert v["gathered_frame_sha256_16"] == v["one_gpu_frame_sha256_16"]
