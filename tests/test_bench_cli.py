"""bench.py's launch contract on a CPU box: `--gpus N` always means N ranks."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(args, env=None):
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=e, capture_output=True,
                          text=True, timeout=300)


def test_gpus_flag_launches_that_many_ranks():
    p = run(["--gpus", "2", "--dry-run"])
    assert p.returncode == 0, p.stderr[-2000:]
    line = [l for l in p.stdout.splitlines() if l.startswith("{")][-1]
    out = json.loads(line)
    assert out["n_gpus"] == 2 and out["ranks_joined"] == 2


def test_gpus_flag_must_match_torchrun_world():
    p = run(["--gpus", "2", "--dry-run"], {"WORLD_SIZE": "3", "RANK": "0"})
    assert p.returncode == 2 and "WORLD_SIZE=3" in p.stderr
