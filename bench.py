#!/usr/bin/env python3
"""Headline benchmark: Mrays/s (primary+secondary) at 1920x1080x64spp on 1..8 MI355X.

Workload (BASELINE.json configs[2]): scenes/scene5.json with its
Mesh pointed at the deterministic dragon stand-in (327,680 triangles; the real
meshes/dragon.stl is missing from the reference snapshot), 1920x1080,
`-g path -n 64`, reference defaults otherwise (-b 10 -a 0.01 -l sqr -o 1 -s phong).
A step = one full frame through the C-ABI (rtx_render_device) with the scene and
BVH already resident in HBM; with N ranks the frame's 8x8 tiles are dealt
round-robin (rank r renders tiles t % N == r) and every step ends with the
RCCL all-gather of the packed tiles (16 B/px), so the image is complete on
every rank.  Rays = cast_ray calls + is_light_blocked calls, exactly as the
reference defines its work; counted by the kernel.

Launch: python bench.py [--gpus N] [--steps K] [--warmup W]
        python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
`--gpus N` always means N ranks: without a torchrun environment, bench.py starts
torch.distributed.run itself (one child process per GPU, before anything touches a GPU)
and exits with its code; under torchrun, WORLD_SIZE must equal N or it exits non-zero.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "c-raytracer_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

METRIC = "Mrays/s (primary+secondary) at 1920×1080×64spp; 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# MI355X_MICROARCH.md: 256 CUs x 4 SIMDs, 2.4 GHz max clock, one wave64 VALU instruction per SIMD
# every 2 cycles -> peak VALU issue in wave-instructions per second
VALU_PEAK_GINST = 256 * 4 * 2.4e9 / 2 / 1e9
VALU_SIMDS, VALU_CLOCK_GHZ = 256 * 4, 2.4
# that peak holds only for the forms gfx950 dual-issues; measured (tools/dev/valu_rates.hip,
# profiles/r05/valu_rates_r05r.log) every other VALU form (min/max, conversions, compares,
# cndmask, perm, fma_mix, any operand in an SGPR) issues at half of it: roofline["issue_slots"]
# useful VALU per operation of k_shadow (the minimal instruction count of the arithmetic the
# reference's algorithm needs, per lane): box_hit_q octant form 17 (6 cvt, 6 fma,
# max/max3/min3/min, cmp), any_tri 39, a plane test 12, and per light sample 100 (counter RNG,
# light point, direction, attenuation, Phong/Blinn incl. powf)
USEFUL_VALU = {"box": 17, "tri": 39, "sphere": 25, "plane": 12, "sample": 100}
# SURVEY 8(d)'s other two bases for the same kernel: FLOPs (~12 per AABB test with a precomputed
# 1/d, ~27 per Moller-Trumbore test) against the FP32 vector peak, and the algorithmic byte model
# B_ray = 64 per node fetch + 48 per triangle + 32 per sphere + 16 per plane test + 48 per ray
FP32_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: FP32 vector
FLOP_MODEL = {"box": 12, "tri": 27}
BYTE_MODEL = {"node": 64, "tri": 48, "sphere": 32, "plane": 16, "ray": 48}
SHADOW_SRCS = ["c-raytracer_amd/csrc/rtx_shadow.hip", "c-raytracer_amd/csrc/rtx_w8.h", "c-raytracer_amd/csrc/rtx_wave.h",
               "c-raytracer_amd/csrc/rtx_math.h", "c-raytracer_amd/csrc/rtx_device.h", "include/rtx_rng.h"]


CPU_AT_N1 = ("cpu_baseline is timed on rank 0 of the N = 1 run only (the same workload on one GPU: "
             "python bench.py --gpus 1); an N > 1 line leaves it null")


def shadow_src_sha():
    """sha1 over k_shadow's sources with comments and blank space stripped: ties a committed PMC
    summary to the kernel code it measured (a comment edit keeps the tie, a code edit breaks it)"""
    import hashlib
    import re
    h = hashlib.sha1()
    for f in SHADOW_SRCS:
        with open(os.path.join(ROOT, f), encoding="utf-8") as fh:
            code = re.sub(r"/\*.*?\*/", " ", fh.read(), flags=re.S)
        code = re.sub(r"//[^\n]*", " ", code)
        h.update(" ".join(code.split()).encode())
    return h.hexdigest()[:16]


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--scene", default="scene5", choices=["scene5", "scene5_l8", "scene6", "scene3", "scene1"])
    ap.add_argument("--launch", default="group", choices=["group", "torchrun"],
                    help="--gpus N > 1 without torchrun: one process driving the C-ABI device group "
                         "(default), or N torchrun ranks")
    ap.add_argument("--walk", default="auto", choices=["auto", "w8", "bvh2", "linear"],
                    help="shadow-walk BVH layout (rtx_set_option RTX_OPT_SHADOW_WALK; auto = the library default)")
    ap.add_argument("--trace-walk", default="auto", choices=["auto", "w8", "bvh2"],
                    help="closest-hit BVH layout (rtx_set_option RTX_OPT_TRACE_WALK)")
    ap.add_argument("--no-cull", action="store_true",
                    help="every shadow packet walks the tree (rtx_set_option RTX_OPT_SHADOW_CULL 0; an A/B of the cone cull)")
    ap.add_argument("--cull-slots", action="store_true",
                    help="the lane-slot packets cull too (rtx_set_option RTX_OPT_SHADOW_CULL 2)")
    ap.add_argument("--frame", default="auto", choices=["auto", "world"],
                    help="the frame the BVHs are built in (rtx_set_option RTX_OPT_TREE_FRAME; auto = the library default)")
    ap.add_argument("--shadow-slot", type=int, default=0,
                    help="k_shadow lanes per shade-point slot (rtx_set_option RTX_OPT_SHADOW_SLOT; 0 = automatic)")
    ap.add_argument("--shadow-grab", type=int, default=0,
                    help="k_shadow lane slots per work-queue grab (RTX_OPT_SHADOW_GRAB; 0 = library default)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-count", action="store_true", help="skip the traversal-counting pass (roofline)")
    ap.add_argument("--no-post", action="store_true", help="skip the postprocess (DoF + mist) side leg")
    ap.add_argument("--cpu-target-s", type=float, default=12.0)
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--loopback", action="store_true",
                    help="--gpus N > 1 as N shards on device 0 (rtx_group_open_loopback: the device group's own path "
                         "with a device-to-device copy for the RCCL gather); a one-GPU rehearsal, never a scaling number")
    ap.add_argument("--dry-run", action="store_true",
                    help="rank bring-up only (gloo, no GPU): print the ranks' world and exit (tests)")
    return ap.parse_args()


def launch_mode(a):
    """How `--gpus N` runs.  Under torchrun (WORLD_SIZE set) this process is one rank of N: it
    must equal --gpus.  Without torchrun: N = 1 renders on one device; N > 1 renders in THIS
    process through the C-ABI device group (rtx_group_*: one host thread per device, the tile
    shards gathered to the first device with RCCL send/recv), the path `engine --gpus N` ships;
    `--launch torchrun` instead starts N ranks through torch.distributed.run as a child process
    (before anything touches a GPU, so no exec of a GPU process).  Returns ("rank", None),
    ("group", None) or ("exit", code)."""
    world = os.environ.get("WORLD_SIZE")
    if world is not None:
        if int(world) != a.gpus:
            print(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world}: refusing to report a different "
                  f"GPU count than asked", file=sys.stderr)
            return "exit", 2
        return "rank", None
    if a.gpus < 1:
        print(f"bench.py: --gpus {a.gpus}: need at least one", file=sys.stderr)
        return "exit", 2
    if a.gpus == 1:
        return "rank", None
    if a.launch == "group":
        return "group", None
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    return "exit", subprocess.run(cmd, env=env).returncode


def dry_run(a, mode):
    """Launch bring-up without a GPU: every torchrun rank joins a gloo group and rank 0 prints the
    world size the JSON line would carry (the device-group mode prints its line's schema: main_group)."""
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    backend, ws, seen = None, 1, [rank]
    if world > 1:
        torch.distributed.init_process_group("gloo")
        t = torch.ones(1)
        torch.distributed.all_reduce(t)
        ranks = int(t.item())
        backend, ws = torch.distributed.get_backend(), torch.distributed.get_world_size()
        seen = [None] * ws
        torch.distributed.all_gather_object(seen, rank)
        torch.distributed.destroy_process_group()
    else:
        ranks = 1
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "ranks_joined": ranks, "gpus_flag": a.gpus,
                          "launch": "torchrun" if world > 1 else "single", "backend": backend, "world_size": ws,
                          "ranks_seen": sorted(seen)}), flush=True)


def scene_path(which):
    import standins
    if which.startswith("scene5") or which == "scene6":
        return standins.ensure_scene(which)
    return os.path.join(ROOT, "tests", "golden", "scenes", which + ".json")


def flags_for(which, spp):
    if which in ("scene1",):
        return []
    return ["-g", "path", "-n", str(spp)]


def _rng_name(mode):
    from rtxpy import abi
    return {abi.RTX_RNG_CONST: "const", abi.RTX_RNG_COUNTER: "counter",
            abi.RTX_RNG_STRAT: "counter, stratified light samples"}.get(mode, str(mode))


def _omp_threads():
    return int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)


def cpu_port(scene, frame, params, target_s, log):
    """Our CPU restatement (oracle/restate.c, 'port') on an evenly spaced sample of the SAME frame's
    tiles, all host threads.  Bit-exact with the reference built -O2, but ~10x faster than the
    reference binary (flat BVH arrays, counter RNG without glibc's rand() lock)."""
    from rtxpy import abi, oracle
    import rtxpy
    threads = _omp_threads()
    tx, ty = (frame.width + 7) // 8, (frame.height + 7) // 8
    total = tx * ty
    p = rtxpy.default_params(**{f: getattr(params, f) for f, _ in abi.Params._fields_})
    stride = max(1, total // 4)
    p.tile_offset, p.tile_stride = 0, stride
    t0 = time.perf_counter()
    oracle.render(scene, frame, p, threads)
    dt = max(time.perf_counter() - t0, 1e-3)
    want = max(4, min(total, int(((total + stride - 1) // stride) / dt * target_s)))
    stride = max(1, total // want)
    p.tile_offset, p.tile_stride = stride // 2 if stride > 1 else 0, stride
    t0 = time.perf_counter()
    _, _, (c, s) = oracle.render(scene, frame, p, threads)
    dt = time.perf_counter() - t0
    n_tiles = len(range(p.tile_offset, total, stride))
    log(f"cpu port: {n_tiles} tiles, {c}+{s} rays in {dt:.2f}s on {threads} threads")
    return {"value": round((c + s) / dt / 1e6, 4), "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": f"{n_tiles} of {total} 8x8 tiles (every {stride}th) of the same {frame.width}x{frame.height} "
                      f"frame and flags, {_rng_name(p.rng)} RNG", "seconds": round(dt, 2), "rays": c + s}


def cpu_reference(scene_file, flags, width, height, target_s, log):
    """The reference itself (oracle/_ref/engine_seed_*: /root/reference's sources built with its own
    Makefile.rt flags + the determinism shim), timed on the host cores at a reduced resolution of the
    same scene and flags (Mrays/s is intensive: scale the resolution, not the spp).
    Both thread modes SURVEY §8(d) asks for are timed, `-m 1` and `-m max` (all host threads), each
    on a frame sized for ~target_s/2 of rendering; the faster is the baseline.  Rays are counted by
    the instrumented build (engine_count_*) on the same config.

    The reference's row loop is OpenMP's static schedule (render.c:349-352: each thread gets a
    contiguous block of ceil(H / threads) rows), so a frame with few rows leaves threads idle.  The
    `-m max` frame (and its calibration frame) therefore has H a multiple of the thread count and at
    least 4 rows per thread, H = 4·threads·k; only its width is fitted to the time target (the
    reference's image plane keeps the horizontal field of view, image.c:41-42)."""
    import subprocess
    import tempfile
    refdir = os.path.join(ROOT, "oracle", "_ref")
    threads = _omp_threads()
    golden = os.path.join(ROOT, "tests", "golden")
    with tempfile.TemporaryDirectory() as wd:
        os.symlink(os.path.join(golden, "meshes"), os.path.join(wd, "meshes"))
        os.symlink(os.path.dirname(scene_file), os.path.join(wd, "scenes"))
        rel = os.path.join("scenes", os.path.basename(scene_file))

        def run(binary, w, h, nthreads):
            env = dict(os.environ, RTX_REF_SEED="1", OMP_NUM_THREADS=str(nthreads))
            cmd = [binary, rel, os.path.join(wd, "o.tif"), str(w), str(h), "-m",
                   "1" if nthreads == 1 else "max"] + flags
            t0 = time.perf_counter()
            p = subprocess.run(cmd, cwd=wd, env=env, capture_output=True, text=True, timeout=600)
            dt = time.perf_counter() - t0
            if p.returncode != 0:
                raise RuntimeError(f"{os.path.basename(binary)} rc={p.returncode}")
            stamps = []
            for line in p.stdout.splitlines():  # reference log: "[sss.mmm] file: func: line: msg"
                if "Commencing raytracing." in line or "Saving image." in line:
                    stamps.append(float(line[1:line.index("]")]))
            t_render = (stamps[-1] - stamps[0]) if len(stamps) == 2 else dt
            t_render = max(t_render, 1e-3)
            counts = None
            for line in p.stderr.splitlines():
                if line.startswith("RTX_REF_COUNT"):
                    kv = dict(x.split("=") for x in line.split()[1:])
                    counts = int(kv["closest"]) + int(kv["shadow"])
            return dt, t_render, counts

        for arch in ("native", "v3"):
            eng = os.path.join(refdir, f"engine_seed_{arch}")
            cnt = os.path.join(refdir, f"engine_count_{arch}")
            if not (os.path.exists(eng) and os.path.exists(cnt)):
                continue
            modes = {}
            try:
                for nthreads in (1, threads):
                    # calibrate (pixels per second), then size the frame for ~target_s/2 of rendering
                    w, h = (16, 9) if nthreads == 1 else (8, 4 * nthreads)
                    _, tr, _ = run(eng, w, h, nthreads)
                    px = w * h / max(tr, 0.05) * target_s / 2
                    if nthreads == 1:
                        scale = min(64.0, max(1.0, px / (w * h)) ** 0.5)
                        w, h = max(16, int(w * scale)), max(9, int(h * scale))
                    else:  # H = 4·threads·k rows (static row schedule), aspect at most 16:9
                        k = max(1, int((px * 9 / 16) ** 0.5 / (4 * nthreads)))
                        h = 4 * nthreads * k
                        w = max(8, min((16 * h) // 9, int(round(px / h))))
                    _, tr, _ = run(eng, w, h, nthreads)
                    _, _, rays = run(cnt, w, h, nthreads)
                    log(f"cpu reference ({arch}, -m {'1' if nthreads == 1 else 'max'}): {w}x{h} "
                        f"{' '.join(flags)}: {rays} rays in {tr:.2f}s on {nthreads} threads")
                    modes[nthreads] = {"value": round(rays / tr / 1e6, 4), "cores": nthreads,
                                       "seconds": round(tr, 2), "rays": rays, "frame": f"{w}x{h}",
                                       "rows_per_thread": h / nthreads}
            except (RuntimeError, subprocess.TimeoutExpired, OSError) as e:
                log(f"reference {arch} unusable here: {e}")
                continue
            best = max(modes.values(), key=lambda m: m["value"])
            return {"value": best["value"], "unit": "Mrays/s", "cores": best["cores"], "kind": "reference",
                    "sample": f"reference engine (Makefile.rt flags, -march={'native' if arch == 'native' else 'x86-64-v3'}"
                              f") on the same scene and flags at a reduced resolution, timed at -m 1 and -m max "
                              f"({threads} host threads; the -m max frame has 4k rows per thread for the static "
                              f"OpenMP row schedule); the faster is the value; render window = its own "
                              f"'Commencing raytracing' -> 'Saving image' log stamps; rays from the instrumented "
                              f"build on the same config",
                    "seconds": best["seconds"], "rays": best["rays"],
                    "m1": modes.get(1), "mmax": modes.get(threads)}
    return None


def frame_hash(rgb, z):
    """sha256 (16 hex digits) of a frame's float32 rgb and z buffers, row-major"""
    import hashlib
    import numpy as np
    h = hashlib.sha256()
    h.update(np.ascontiguousarray(rgb, dtype=np.float32).tobytes())
    h.update(np.ascontiguousarray(z, dtype=np.float32).tobytes())
    return h.hexdigest()[:16]


def _device_ids(dev):
    """what torch reports about a device: name, PCI bus / device / domain ids and UUID where the
    build exposes them"""
    import torch
    p = torch.cuda.get_device_properties(dev)
    out = {"name": p.name}
    for k in ("pci_bus_id", "pci_device_id", "pci_domain_id", "uuid"):
        v = getattr(p, k, None)
        if v is not None:
            out[k] = str(v)
    return out


def rank_validation(a, rank, local, world, dev, rehearse, r, frame, params, d_rgb, d_z, stream, h_rgb, h_z, per_frame):
    """what the N > 1 torchrun line can show about itself.  Every rank reports what
    torch.distributed and the runtime see (world size, backend, rank, device ids) and its shard's rays
    per frame (all_gather_object, one small collective after the timed steps); rank 0 then renders
    the whole frame alone (the N = 1 frame: tile stride 1 on its own device) and checks that the
    shards' rays add up to that frame's exactly and that the gathered image is that frame bit for
    bit (the counter RNG makes the image independent of the sharding).
    Returns the line's `validation` object on rank 0 (None elsewhere)."""
    import numpy as np
    import torch
    import rtxpy
    from rtxpy import abi
    ws = torch.distributed.get_world_size()
    me = {"rank": rank, "local_rank": local, "device": local, "ids": _device_ids(dev),
          "closest_rays": int(per_frame[0]), "shadow_rays": int(per_frame[1])}
    ranks = [None] * ws
    torch.distributed.all_gather_object(ranks, me)
    if rank != 0:
        return None
    p1 = rtxpy.default_params(**{f: getattr(params, f) for f, _ in abi.Params._fields_})
    p1.tile_offset, p1.tile_stride = 0, 1
    r.render_device(frame, p1, d_rgb.data_ptr(), d_z.data_ptr(), stream.cuda_stream)
    torch.cuda.synchronize(dev)
    s1 = r.stats()
    full_hash = frame_hash(d_rgb.cpu().numpy(), d_z.cpu().numpy())
    gathered_hash = frame_hash(h_rgb.numpy(), h_z.numpy())
    sum_c = sum(x["closest_rays"] for x in ranks)
    sum_s = sum(x["shadow_rays"] for x in ranks)
    devs = {(x["ids"].get("pci_domain_id"), x["ids"].get("pci_bus_id"), x["ids"].get("uuid"), x["local_rank"])
            for x in ranks}
    checks = {"world_size_is_gpus": ws == a.gpus,
              "ranks_joined": sorted(x["rank"] for x in ranks) == list(range(ws)),
              "distinct_devices": rehearse or len(devs) == ws,
              "rays_sum_to_one_gpu_frame": (sum_c, sum_s) == (int(s1.closest_rays), int(s1.shadow_rays)),
              "gathered_frame_is_one_gpu_frame": gathered_hash == full_hash}
    return {"backend": torch.distributed.get_backend(), "world_size": ws, "ranks": ranks,
            "rays_per_frame_sum": [sum_c, sum_s],
            "one_gpu_frame_rays": [int(s1.closest_rays), int(s1.shadow_rays)],
            "gathered_frame_sha256_16": gathered_hash, "one_gpu_frame_sha256_16": full_hash,
            "checks": checks, "ok": all(checks.values()),
            "note": "rank 0 rendered the whole frame alone after the timed steps (the N = 1 frame) to check the "
                    "sharded run against it; bench.py exits non-zero after printing when ok is false"}


def shadow_roofline(r, frame, params, d_rgb, d_z, stream, shadow_ms, a, world):
    """the counting pass (count_traversal) of the same frame on renderer r, then shadow_roofline_of"""
    from rtxpy import abi
    import rtxpy
    p2 = rtxpy.default_params(**{f: getattr(params, f) for f, _ in abi.Params._fields_})
    p2.count_traversal = 1
    r.render_device(frame, p2, d_rgb.data_ptr(), d_z.data_ptr(), stream.cuda_stream)
    return shadow_roofline_of(r.stats(), shadow_ms, a, world)


def shadow_roofline_of(c, shadow_ms, a, world):
    """Roofline of the dominant kernel, k_shadow (~97 % of device time).  Its counts come from a
    counting instance of the same kernel over the same frame; its duration is the HIP-event time
    of k_shadow in the timed steps (rocprofv3 agrees: profiles/).
      bound:  VALU issue (the walk is divergent branchy scalar work; its BVH is L2/MALL-resident,
              so HBM is far from saturated).  achieved = useful VALU wave-instructions (USEFUL_VALU
              per box test / triangle / plane / light sample, / 64 lanes) per second; peak = the
              chip's VALU issue rate.  issued = PMC SQ_INSTS_VALU of the same kernel build.
      hbm:    algorithmic bytes = the records k_shadow reads from memory: 16 B per box test whose
              record comes from the DQNode array (LDS top records excluded, reported apart), 48 B
              per primitive test, 96 B per shade-point record + 4 B of its Morton index + 16 B
              written per point; traffic = PMC 2*FETCH_SIZE + WRITE_SIZE (gfx950 correction).
    c: the counting render's rtx_stats (one device's), shadow_ms: that device's k_shadow time in the
    timed steps."""
    dur = shadow_ms * 1e-3
    n_pts = int(c.shade_points)
    prim_tests = int(c.shadow_tri_tests + c.shadow_sphere_tests)
    glob = int(c.shadow_global_box_tests)
    lds_box = int(c.shadow_box_tests) - glob
    algo_bytes = 16 * glob + 48 * prim_tests + (96 + 4 + 16) * n_pts
    useful = (USEFUL_VALU["box"] * c.shadow_box_tests + USEFUL_VALU["tri"] * c.shadow_tri_tests
              + USEFUL_VALU["sphere"] * c.shadow_sphere_tests + USEFUL_VALU["plane"] * c.shadow_plane_tests
              + USEFUL_VALU["sample"] * c.shadow_rays) / 64.0
    achieved = useful / dur / 1e9
    out = {"bound": "valu", "achieved": round(achieved, 1), "peak": VALU_PEAK_GINST, "unit": "Ginst/s",
           "frac": round(achieved / VALU_PEAK_GINST, 4), "traffic": None, "kernel": "k_shadow",
           "kernel_ms": round(shadow_ms, 3), "useful_valu_per_launch": int(useful),
           "useful_valu_model": USEFUL_VALU, "shadow_rays": int(c.shadow_rays), "shade_points": n_pts,
           "box_tests": int(c.shadow_box_tests), "box_tests_global": glob, "box_tests_lds": lds_box,
           "tri_tests": int(c.shadow_tri_tests), "sphere_tests": int(c.shadow_sphere_tests),
           "plane_tests": int(c.shadow_plane_tests), "wave_steps": int(c.shadow_wave_steps),
           "wave_walks": int(c.shadow_wave_walks), "leaf_rounds": int(c.shadow_leaf_rounds),
           "uniform_steps": int(c.shadow_uniform_steps),
           "stack_spills": int(getattr(c, "shadow_stack_spills", 0)),
           "cone_clear_rays": int(getattr(c, "shadow_cone_clear", 0)),
           "shadow_rays_per_s": round(c.shadow_rays / dur / 1e9, 3),
           "shadow_rays_per_s_unit": "G/s (tree-independent: the reference's is_light_blocked calls per second)",
           "k_trace": {"closest_rays": int(c.closest_rays),
                       "node_visits": int(c.node_visits - c.shadow_node_visits),
                       "prim_tests": int(c.tri_tests + c.sphere_tests - c.shadow_tri_tests - c.shadow_sphere_tests),
                       "note": "closest-hit walk counts of the same counting render (8-wide node visits, "
                               "primitive tests)"},
           "wide_nodes": int(c.wide_nodes), "wide_depth": int(c.wide_depth),
           "records": {"bytes_per_launch": int(algo_bytes), "lds_bytes_per_launch": 16 * lds_box,
                       "GBs": round(algo_bytes / dur / 1e9, 1),
                       "note": "bytes of the records the lanes read (served by L1 / L2 / Infinity Cache, so no HBM "
                               "fraction); HBM-side bytes: traffic"}}
    # the same launch on SURVEY 8(d)'s FLOP and byte bases: a node fetch is one 64-byte
    # 8-wide node (8 box tests) on the 8-wide walk, one 16-byte threaded record per box test otherwise
    w8 = int(c.wide_nodes) > 0
    node_bytes = BYTE_MODEL["node"] * c.shadow_box_tests / 8 if w8 else 16 * c.shadow_box_tests
    model_bytes = (node_bytes + BYTE_MODEL["tri"] * c.shadow_tri_tests + BYTE_MODEL["sphere"] * c.shadow_sphere_tests
                   + BYTE_MODEL["plane"] * c.shadow_plane_tests + BYTE_MODEL["ray"] * c.shadow_rays)
    flops = FLOP_MODEL["box"] * c.shadow_box_tests + FLOP_MODEL["tri"] * c.shadow_tri_tests
    out["bases"] = {
        "valu_useful": {"frac": out["frac"], "note": "useful VALU wave-instructions over the all-dual-issue peak (the "
                                                      "line's roofline.frac)"},
        "flop": {"achieved": round(flops / dur / 1e12, 2), "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                 "frac": round(flops / dur / 1e12 / FP32_PEAK_TFLOPS, 4), "flop_per_launch": int(flops),
                 "model": "SURVEY 8(d): 12 FLOP per box test, 27 per triangle test"},
        "bytes_model": {"bytes_per_launch": int(model_bytes), "achieved": round(model_bytes / dur / 1e12, 2),
                        "unit": "TB/s", "peak_hbm": HBM_PEAK_GBS / 1e3,
                        "x_hbm_peak": round(model_bytes / dur / 1e9 / HBM_PEAK_GBS, 3),
                        "model": "SURVEY 8(d) B_ray: 64 B per node fetch (one 64-B 8-wide node per 8 box tests), 48 per "
                                 "triangle, 32 per sphere, 16 per plane test, 48 per ray",
                        "note": "above HBM peak: the tree is served from L2 and the Infinity Cache, so north_star's "
                                "HBM-bound roofline cannot bind this walk; the PMC HBM bytes are hbm.frac"},
        "binding": "VALU issue slots (roofline.issue_slots.frac) with the texture-data path beside it "
                   "(roofline.vmem.td_busy_frac); DESIGN.md section 5"}
    if out["frac"] > 1.0:  # the useful-instruction model overestimates: report, never abort the bench
        print(f"warning: VALU roofline fraction {out['frac']} > 1 (USEFUL_VALU model too high)", file=sys.stderr)
    pmc = os.path.join(ROOT, "profiles", "pmc_k_shadow.json")
    key = f"{a.scene}_{a.width}x{a.height}_n{a.spp}_g{world}"
    try:
        with open(pmc) as fh:
            rec = json.load(fh).get(key)
    except (OSError, ValueError):
        rec = None
    if rec:
        # the counts here (and dur) are the frame's: the PMC summary's per-frame sums (a frame of
        # several chunks launches k_shadow once per chunk), else launches x the per-launch mean
        nl = max(1, int(c.chunks))
        out["pmc"] = {"source": rec.get("source"), "kernel_src_sha": rec.get("kernel_src_sha"),
                      "matches_this_kernel": rec.get("kernel_src_sha") == shadow_src_sha(), "launches_per_frame": nl}
        if "hbm_bytes_per_launch" in rec:
            hbm = rec.get("hbm_bytes_per_frame", nl * rec["hbm_bytes_per_launch"])
            out["bases"]["hbm_pmc"] = {"frac": round(hbm / dur / 1e9 / HBM_PEAK_GBS, 4)}
            out["traffic"] = int(hbm)
            out["hbm"] = {"bytes_per_launch": int(hbm),
                          "achieved": round(hbm / dur / 1e9, 1), "peak": HBM_PEAK_GBS,
                          "unit": "GB/s", "frac": round(hbm / dur / 1e9 / HBM_PEAK_GBS, 4),
                          "source": "PMC 2*FETCH_SIZE + WRITE_SIZE (L2 -> fabric, gfx950 correction)"}
        if "sq_insts_valu" in rec:
            valu = rec.get("sq_insts_valu_frame", nl * rec["sq_insts_valu"])  # per frame when recorded
            issued = valu / dur / 1e9
            out["issued"] = round(issued, 1)
            out["issued_frac"] = round(issued / VALU_PEAK_GINST, 4)
            out["useful_over_issued"] = round(useful / valu, 4)
            out["issued_valu_per_shadow_ray"] = round(valu * 64 / max(1, c.shadow_rays), 1)
            if "sq_active_inst_valu2" in rec:
                # issue slots: gfx950 issues the full-rate VALU forms (f32 add/mul/fma on VGPR or
                # literal operands, mov, and/or/xor, u32 add/sub, lshrrev) two per quad-cycle and
                # every other form one per quad-cycle (tools/dev/valu_rates.hip);
                # SQ_ACTIVE_INST_VALU2 counts the quad-cycles that issued two
                dual = rec.get("sq_active_inst_valu2_frame", nl * rec["sq_active_inst_valu2"])
                used = valu - dual
                avail = dur * VALU_CLOCK_GHZ * 1e9 / 4.0 * VALU_SIMDS
                out["issue_slots"] = {"used_quad_cycles": int(used), "available_quad_cycles": int(avail),
                                      "frac": round(used / avail, 4), "dual_issued_frac": round(2 * dual / valu, 4),
                                      "note": "VALU issue quad-cycles the kernel used (SQ_INSTS_VALU - "
                                              "SQ_ACTIVE_INST_VALU2) over the chip's (1024 SIMDs x 2.4 GHz / 4)"}
                out["bases"]["valu_issue_slots"] = {"frac": out["issue_slots"]["frac"]}
        if "ta_busy_frac" in rec:
            out["vmem"] = {"ta_busy_frac": rec["ta_busy_frac"], "td_busy_frac": rec.get("td_busy_frac"),
                           "note": "PMC TA_TA_BUSY / TD_TD_BUSY per CU cycle: the vector-memory address / data "
                                   "path, the walk's second limit beside VALU issue (DESIGN.md section 5)"}
    return out


POST_FLAGS = ["--dof", "3", "-13", "--mist", "6", "4", "lin", "0.5", "0.5", "0.6"]
# scene6 (configs[4] "Menger sponge + procedural noise + DoF"): focus on the sponge (z ~ 2.4), the
# back plane (z = 8) blurred by a radius-5 disc
POST_FLAGS_SCENE = {"scene6": ["--dof", "2", "-4.8", "--mist", "6", "4", "lin", "0.5", "0.5", "0.6"]}


def post_leg(r, d_rgb, d_z, w, h, dev, log, reps=5, flags=None):
    """§8(f) #1: the postprocess path (rtx_postprocess_device) on the benchmark's own rendered
    frame, next to the reference postprocessor (oracle/_ref/postprocess, single-threaded as it
    ships) on the same raw frame; the 8-bit outputs are compared byte for byte."""
    import subprocess
    import tempfile
    import numpy as np
    import torch
    import rtxpy
    from rtxpy.tiffread import read_tiff
    flags = flags or POST_FLAGS
    post = rtxpy.post_from_args(flags)
    src = d_rgb.clone()
    out = torch.empty_like(d_rgb)
    stream = torch.cuda.current_stream(dev)
    times = []
    for i in range(reps + 1):
        out.copy_(src)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        r.postprocess_device(post, w, h, out.data_ptr(), d_z.data_ptr(), stream.cuda_stream)
        torch.cuda.synchronize(dev)
        if i:
            times.append(time.perf_counter() - t0)
    res = {"flags": " ".join(flags), "gpu_ms": round(1e3 * float(np.median(times)), 3),
           "workload": f"{w}x{h} frame rendered by this bench", "timing": "wall, median of %d, synchronised" % reps}
    ref = os.path.join(ROOT, "oracle", "_ref", "postprocess")
    if not os.path.exists(ref):
        return res
    with tempfile.TemporaryDirectory() as wd:
        raw, o8, g8 = (os.path.join(wd, n) for n in ("in.tif", "ref.tif", "gpu.tif"))
        rgb_h = src.cpu().numpy().reshape(h, w, 3)
        rtxpy.write_tiff(raw, rgb_h, d_z.cpu().numpy().reshape(h, w), raw=True)
        try:
            p = subprocess.run([ref, raw, o8] + flags, capture_output=True, text=True, timeout=600)
        except (subprocess.TimeoutExpired, OSError) as e:
            log(f"reference postprocess unusable: {e}")
            return res
        if p.returncode != 0:
            log(f"reference postprocess rc={p.returncode}")
            return res
        stamps = [float(l[1:l.index("]")]) for l in p.stdout.splitlines()
                  if "Commencing Postprocessing" in l or "Saving image." in l]
        if len(stamps) == 2:
            res["cpu_ref_ms"] = round(1e3 * (stamps[1] - stamps[0]), 1)
            res["cpu_ref_cores"] = 1
        rtxpy.write_tiff(g8, out.cpu().numpy().reshape(h, w, 3))
        res["u8_identical_to_reference"] = bool(np.array_equal(read_tiff(g8)["rgb"], read_tiff(o8)["rgb"]))
    log(f"postprocess: gpu {res['gpu_ms']} ms, reference {res.get('cpu_ref_ms')} ms, "
        f"identical {res.get('u8_identical_to_reference')}")
    return res


CONFIGS = {("scene1", 512, 512): ("configs[0]", None), ("scene3", 1920, 1080): ("configs[1]", 16),
           ("scene5", 1920, 1080): ("configs[2]", 64), ("scene6", 3840, 2160): ("configs[4]", 128)}


def workload(a):
    """the BASELINE.json config this run measures, by name (configs[3] is configs[2]'s scene at
    -n 256 on 8 GPUs), or "custom" """
    name, spp = CONFIGS.get((a.scene, a.width, a.height), (None, None))
    if a.scene == "scene5" and (a.width, a.height, a.spp) == (1920, 1080, 256):
        name, spp = "configs[3]", 256
    label = f"{a.scene} {a.width}x{a.height}" + ("" if a.scene == "scene1" else f" -g path -n {a.spp}")
    if a.scene == "scene5_l8" and (a.width, a.height, a.spp) == (1920, 1080, 64):
        return f"{label} (SURVEY 8(d) level-8 dragon bracket of BASELINE configs[2])"
    return f"{label} (BASELINE {name})" if name and (spp is None or spp == a.spp) else f"{label} (custom)"


def data_label(a):
    if a.scene.startswith("scene5"):
        return ("synthetic: reference scenes/scene5.json with the SURVEY §8(d) deterministic dragon stand-in (level-%d "
                "displaced icosphere; meshes/dragon.stl is missing from the reference)" % (8 if a.scene == "scene5_l8" else 7))
    if a.scene == "scene6":
        return ("synthetic: reference scenes/scene6.json with the SURVEY §8(d) deterministic Menger stand-in (level 4, "
                "672,768 triangles; meshes/menger_sponge.stl is missing from the reference)")
    return f"the reference's own scenes/{a.scene}.json (no mesh)"


WALKS = {"auto": -1, "w8": 2, "bvh2": 0, "linear": 3}
FRAMES = {"auto": 0, "world": 1}


def walk_name(w):
    from rtxpy import abi
    return abi.WALK_NAMES.get(int(w), str(w))


def main():
    a = parse()
    mode, rc = launch_mode(a)
    if mode == "exit":
        sys.exit(rc)
    if mode == "group":
        return main_group(a)
    if a.dry_run:
        dry_run(a, mode)
        return
    import numpy as np
    import torch
    import rtxpy
    from rtxpy import abi
    from rtxpy.dist import Gatherer

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # RTX_BENCH_REHEARSE=gloo: the torchrun ranks' whole path (tile shards, gather to rank 0, the
    # max-over-ranks clock, the JSON line) on however many GPUs the box has, ranks sharing them,
    # over gloo with host staging; a rehearsal of the code, never a scaling number (the driver's
    # launch uses RCCL, one GPU per rank)
    rehearse = world > 1 and os.environ.get("RTX_BENCH_REHEARSE") == "gloo"
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if rehearse:
            local = local % torch.cuda.device_count()
            torch.cuda.set_device(local)
            torch.distributed.init_process_group("gloo")
        else:
            torch.cuda.set_device(local)
            torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # small all-reduces (the clock, the ray counts): gloo reduces host tensors
    red_dev = torch.device("cpu") if rehearse else dev

    def log(msg):
        if a.verbose or rank == 0:
            print(f"[rank {rank}] {msg}", file=sys.stderr, flush=True)

    path = scene_path(a.scene)
    scene = rtxpy.Scene.load(path, base_dir=os.path.join(ROOT, "tests", "golden"))
    frame = scene.frame(a.width, a.height)
    flags = flags_for(a.scene, a.spp)
    params = rtxpy.params_from_args(flags, seed=1)
    params.rng = abi.RTX_RNG_COUNTER  # the reference's i.i.d. light samples (system.c:93-96, object.c:298-299)
    params.tile_offset, params.tile_stride = rank, world

    t_open = time.perf_counter()
    r = rtxpy.Renderer(local)
    open_ms = (time.perf_counter() - t_open) * 1e3  # rtx_open: the device code loaded, copies primed
    r.set_option(abi.RTX_OPT_SHADOW_WALK, WALKS[a.walk])
    r.set_option(abi.RTX_OPT_TRACE_WALK, WALKS[a.trace_walk])
    r.set_option(abi.RTX_OPT_SHADOW_SLOT, a.shadow_slot)
    r.set_option(abi.RTX_OPT_TREE_FRAME, FRAMES[a.frame])
    r.set_option(abi.RTX_OPT_SHADOW_CULL, 0 if a.no_cull else 2 if a.cull_slots else 1)
    if a.shadow_grab:
        r.set_option(abi.RTX_OPT_SHADOW_GRAB, a.shadow_grab)
    t0 = time.perf_counter()
    r.upload(scene)
    upload_ms = (time.perf_counter() - t0) * 1e3
    st = r.stats()
    log(f"scene {os.path.basename(path)}: {scene.num_objects} objects, BVH {st.bvh_nodes} nodes depth {st.bvh_depth}, "
        f"shadow walk {walk_name(st.shadow_walk)}: {st.wide_nodes} wide nodes depth {st.wide_depth}, "
        f"tree frame {'rotated' if st.tree_rotated else 'world'} (leaf-box cost x{st.frame_cost:.3f}) "
        f"({time.perf_counter() - t0:.2f}s build+upload)")

    npx = a.width * a.height
    d_rgb = torch.zeros((npx, 3), dtype=torch.float32, device=dev)
    d_z = torch.zeros((npx,), dtype=torch.float32, device=dev)
    gat = Gatherer(a.width, a.height, rank, world, dev, host_staging=rehearse) if world > 1 else None
    stream = torch.cuda.current_stream(dev)
    # the render window runs up to the framebuffer on the host (rank 0, pinned)
    h_rgb = torch.empty((npx, 3), dtype=torch.float32, pin_memory=True) if rank == 0 else None
    h_z = torch.empty((npx,), dtype=torch.float32, pin_memory=True) if rank == 0 else None

    def step():
        r.render_device(frame, params, d_rgb.data_ptr(), d_z.data_ptr(), stream.cuda_stream)
        s = r.stats()
        if gat is not None:  # shards to rank 0 over RCCL, unpacked there
            out = gat.gather(d_rgb, d_z)
            src = out if rank == 0 else None
        else:
            src = (d_rgb, d_z)
        if src is not None:
            h_rgb.copy_(src[0], non_blocking=True)
            h_z.copy_(src[1], non_blocking=True)
        torch.cuda.synchronize(dev)
        return s

    for i in range(a.warmup):
        s = step()
        log(f"warmup {i}: {s.kernel_ms:.1f} ms, {s.closest_rays}+{s.shadow_rays} rays")

    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    rays = closest = 0
    kms, sms = [], []
    for i in range(a.steps):
        s = step()
        rays += s.closest_rays + s.shadow_rays
        closest += s.closest_rays
        kms.append(s.kernel_ms)
        sms.append(s.shadow_ms)
    torch.cuda.synchronize(dev)
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    stats_closest, stats_shadow = s.closest_rays, s.shadow_rays
    split = {"trace_ms": round(s.trace_ms, 3), "sort_ms": round(s.sort_ms, 3), "shadow_ms": round(s.shadow_ms, 3),
             "accum_ms": round(s.accum_ms, 3),
             "shade_points": int(s.shade_points), "chunks": int(s.chunks)}

    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=red_dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
        rr = torch.tensor([rays, closest], dtype=torch.float64, device=red_dev)
        torch.distributed.all_reduce(rr)
        rays, closest = int(rr[0].item()), int(rr[1].item())

    kernel_ms = float(np.mean(kms))
    shadow_ms = float(np.mean(sms))
    validation = None
    if world > 1:
        validation = rank_validation(a, rank, local, world, dev, rehearse, r, frame, params, d_rgb, d_z, stream,
                                     h_rgb, h_z, (stats_closest, stats_shadow))
    roofline = None
    if not a.no_count:
        roofline = shadow_roofline(r, frame, params, d_rgb, d_z, stream, shadow_ms, a, world)

    strat = None
    if rank == 0 and world == 1 and not a.no_post:
        # side leg: the opt-in stratified light samples (RTX_RNG_STRAT, another estimator of the same
        # expectation; not the reference's sampling), one frame after the timed loop
        p2 = rtxpy.default_params(**{f: getattr(params, f) for f, _ in abi.Params._fields_})
        p2.rng = abi.RTX_RNG_STRAT
        r.render_device(frame, p2, d_rgb.data_ptr(), d_z.data_ptr(), stream.cuda_stream)  # warm its chunk size
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        r.render_device(frame, p2, d_rgb.data_ptr(), d_z.data_ptr(), stream.cuda_stream)
        torch.cuda.synchronize(dev)
        sc_ = r.stats()
        dt = time.perf_counter() - t1
        strat = {"rng": "counter, stratified light samples (RTX_RNG_STRAT, opt-in; not the reference's estimator)",
                 "frame_ms": round(dt * 1e3, 1), "shadow_ms": round(sc_.shadow_ms, 1),
                 "mrays_per_s": round((sc_.closest_rays + sc_.shadow_rays) / dt / 1e6, 1)}
        log(f"stratified-RNG frame: {strat}")

    build = None
    if rank == 0 and world == 1 and not a.no_post:
        # §8(f) #2: every BVH builder on the benchmark scene (build time, then one frame each)
        try:
            names = {abi.RTX_BUILD_SAH_HOST: "sah_host", abi.RTX_BUILD_LBVH_GPU: "lbvh", abi.RTX_BUILD_PLOC_GPU: "ploc",
                     abi.RTX_BUILD_SAH_GPU: "sah_gpu"}
            d = names[int(st.builder)]
            build = {"default": d, "first_upload_wall_ms": round(upload_ms, 1), "open_ms": round(open_ms, 1),
                     "note": f"{d}_ms: the BVH build of this process's first upload (device build + 8-wide collapse); "
                             "first_upload_wall_ms: the whole rtx_upload_scene call; open_ms: rtx_open, which "
                             "loads the library's device code and primes host->device copies once per context",
                     f"{d}_ms": round(st.build_ms, 1), f"{d}_nodes": int(st.bvh_nodes),
                     f"{d}_depth": int(st.bvh_depth), f"{d}_wide_nodes": int(st.wide_nodes),
                     f"{d}_wide_depth": int(st.wide_depth), f"{d}_shadow_walk": walk_name(st.shadow_walk),
                     f"{d}_shadow_ms": round(float(np.mean(sms)), 1)}
            for bid, tag in names.items():
                if bid == int(st.builder):
                    continue
                r.set_builder(bid)
                r.upload(scene)
                sl = r.stats()
                build.update({f"{tag}_ms": round(sl.build_ms, 1), f"{tag}_nodes": int(sl.bvh_nodes),
                              f"{tag}_depth": int(sl.bvh_depth), f"{tag}_wide_nodes": int(sl.wide_nodes),
                              f"{tag}_wide_depth": int(sl.wide_depth),
                              f"{tag}_shadow_walk": walk_name(sl.shadow_walk)})
                r.render_device(frame, params, d_rgb.data_ptr(), d_z.data_ptr(), stream.cuda_stream)
                build[f"{tag}_shadow_ms"] = round(r.stats().shadow_ms, 1)
                build[f"{tag}_trace_ms"] = round(r.stats().trace_ms, 1)
            r.set_builder(int(st.builder))
            r.upload(scene)
            r.render_device(frame, params, d_rgb.data_ptr(), d_z.data_ptr(), stream.cuda_stream)
            log(f"builders: {build}")
        except Exception as e:
            log(f"builder leg failed: {e}")
            build = None

    post = None
    if rank == 0 and world == 1 and not a.no_post:
        try:
            post = post_leg(r, d_rgb, d_z, a.width, a.height, dev, log, flags=POST_FLAGS_SCENE.get(a.scene))
        except Exception as e:  # never let the side leg kill the measurement
            log(f"postprocess leg failed: {e}")

    if world > 1:
        # the GPU work is done: every rank leaves the process group
        r.close()
        r = None
        torch.distributed.destroy_process_group()
    cpu = port = None
    # the CPU baseline is timed on rank 0 at N = 1 only; the N > 1 lines point to that line
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        try:
            cpu = cpu_reference(path, flags, a.width, a.height, a.cpu_target_s, log)
        except Exception as e:  # never let the baseline kill the measurement
            log(f"reference baseline failed: {e}")
        if world == 1:
            port = cpu_port(scene, frame, params, a.cpu_target_s / 2, log)
        if cpu is None:
            cpu = port
            port = None

    if rank == 0:
        value = rays / elapsed / 1e6
        out = {"metric": METRIC, "value": round(value, 2), "unit": "Mrays/s", "n_gpus": world, "steps": a.steps,
               "closest_mrays": round(closest / elapsed / 1e6, 2),
               "warmup": a.warmup, "ms_per_step": round(elapsed / a.steps * 1e3, 3), "higher_is_better": True,
               "scaling": "strong", "vs_baseline": None, "dtype": "f32", "data": data_label(a),
               "config": {"workload": workload(a),
                          "scene": os.path.basename(path), "width": a.width, "height": a.height, "spp": a.spp,
                          "objects": int(scene.num_objects), "rays_per_frame": rays // max(1, a.steps),
                          "rays_per_frame_rank0": stats_closest + stats_shadow,
                          "closest_rays_rank0": stats_closest, "shadow_rays_rank0": stats_shadow,
                          "parallelism": f"tiles{world}", "launch": "torchrun" if world > 1 else "single",
                          "kernel_ms_rank0": round(kernel_ms, 3), "kernels_rank0": split,
                          "shadow_walk": walk_name(st.shadow_walk),
                          "trace_walk": walk_name(s.trace_walk),
                          "tree_frame": {"rotated": bool(st.tree_rotated), "leaf_box_cost_vs_world": round(st.frame_cost, 4),
                                         "choose_ms": round(st.frame_ms, 1)},
                          "step": "render into HBM, tile shards gathered to rank 0 over RCCL (N > 1), frame copied "
                                  "to pinned host memory (SURVEY 8(d): render window up to the framebuffer on the host)",
                          "rng": "counter, i.i.d. light samples (RTX_RNG_COUNTER, the library default; the "
                                 "reference's rand_flt sampling, system.c:93-96, object.c:298-299)"},
               "roofline": roofline, "cpu_baseline": cpu}
        if gat is not None:
            out["config"]["gather_message_bytes_per_rank"] = gat.message_bytes
        if world > 1:
            out["cpu_baseline_note"] = CPU_AT_N1
        if validation is not None:
            out["validation"] = validation
        if rehearse:
            out["n_gpus"] = min(world, torch.cuda.device_count())
            out["ranks"] = world
            out["rehearsal"] = ("RTX_BENCH_REHEARSE=gloo: torchrun ranks sharing the box's GPUs, gathered over gloo "
                                "through host memory; the code path of the RCCL launch, not a scaling number")
        if strat:
            out["rng_strat_frame"] = strat
        if cpu:
            out["config"]["gpu_over_cpu"] = round(value / cpu["value"], 1)
        if port:
            out["cpu_port"] = port
        if post:
            out["postprocess"] = post
        if build:
            out["bvh_build"] = build
        print(json.dumps(out), flush=True)
        if validation is not None and not validation["ok"]:
            print(f"bench.py: the {world}-rank run failed its own checks: {validation['checks']}", file=sys.stderr)
            sys.exit(3)
    if r is not None:
        r.close()


def group_line(a, n, scene_name, objects, elapsed, rays, closest, per_dev, gather_ms, roofline, cpu=None,
               upload=None):
    """the JSON line of a device-group run (also printed by --dry-run, with None for what only a
    GPU measures).  per_dev: one dict per device of its mean kernel / k_trace / k_shadow times
    and rays over the timed steps."""
    steps = a.steps
    kms = [d["kernel_ms"] for d in per_dev if d["kernel_ms"] is not None]
    value = rays / elapsed / 1e6 if elapsed else None
    frame_rays = rays // steps if rays is not None else None
    return {"metric": METRIC, "value": round(value, 2) if value is not None else None, "unit": "Mrays/s",
            "n_gpus": 1 if getattr(a, "loopback", False) else n, "shards": n,
            "steps": steps, "warmup": a.warmup,
            "ms_per_step": round(elapsed / steps * 1e3, 3) if elapsed else None,
            "closest_mrays": round(closest / elapsed / 1e6, 2) if elapsed else None,
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32", "data": data_label(a),
            "config": {"workload": workload(a), "scene": scene_name, "width": a.width, "height": a.height,
                       "spp": a.spp, "objects": objects, "parallelism": f"tiles{n}", "launch": "group",
                       "rays_per_frame": frame_rays,
                       "rng": "counter, i.i.d. light samples (RTX_RNG_COUNTER, the library default)",
                       "step": "rtx_group_render: shards on every device, RCCL send/recv to device 0, unpack, copy to "
                               "pinned host memory (SURVEY 8(d) window)"},
            "group": {"rtx_group_size": n, "rccl_devices": n if n > 1 and not a.loopback else 0,
                      "transport": ("loopback (n shards on device 0, device-to-device copy; a rehearsal of the "
                                    "group path, not a multi-GPU measurement)") if a.loopback else "rccl",
                      "devices": per_dev,
                      "device_kernel_ms_max": max(kms) if kms else None,
                      "device_kernel_ms_min": min(kms) if kms else None,
                      "gather_ms": gather_ms,
                      "gather_message_bytes_per_device": int(16 * 64 * -(-((a.width + 7) // 8) * ((a.height + 7) // 8) // n)),
                      "upload": upload},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "cpu_baseline_note": CPU_AT_N1 if cpu is None else
                                 "the reference's own CPU path on this box's host cores, timed after the GPU steps "
                                 "(the loopback rehearsal runs on one GPU, so it carries the N = 1 baseline)"}


def group_validation(a, g, n, scene, frame, params, h_rgb, h_z, frame_rays, log):
    """VERDICT r05 #5 for the device group: the members as the runtime reports them (every RCCL
    communicator's count, rank and device read back, peer access both ways per pair with device 0,
    PCI bus ids), and the last timed frame against the whole frame rendered by one context on
    device 0 alone (the N = 1 frame): the shards' rays must add up to its rays exactly and the
    gathered image must be it bit for bit."""
    import rtxpy
    from rtxpy import abi
    members = [g.member(r) for r in range(n)]
    single = rtxpy.Renderer(g.devices[0])
    try:
        single.set_option(abi.RTX_OPT_SHADOW_WALK, WALKS[a.walk])
        single.set_option(abi.RTX_OPT_TRACE_WALK, WALKS[a.trace_walk])
        single.set_option(abi.RTX_OPT_SHADOW_SLOT, a.shadow_slot)
        single.set_option(abi.RTX_OPT_TREE_FRAME, FRAMES[a.frame])
        single.set_option(abi.RTX_OPT_SHADOW_CULL, 0 if a.no_cull else 2 if a.cull_slots else 1)
        single.upload(scene)
        rgb1, z1 = single.render(frame, params)
        s1 = single.stats()
    finally:
        single.close()
    one_hash, gathered_hash = frame_hash(rgb1, z1), frame_hash(h_rgb, h_z)
    rccl = n > 1 and not a.loopback
    checks = {"members_are_gpus": len(members) == a.gpus,
              "distinct_devices": a.loopback or len({m["pci_bus_id"] for m in members}) == n,
              "rays_sum_to_one_gpu_frame": (int(frame_rays[0]), int(frame_rays[1])) == (int(s1.closest_rays),
                                                                                        int(s1.shadow_rays)),
              "gathered_frame_is_one_gpu_frame": gathered_hash == one_hash}
    if rccl:
        checks["rccl_comms_count_n"] = all(m["comm_count"] == n for m in members)
        checks["rccl_ranks_distinct"] = sorted(m["comm_rank"] for m in members) == list(range(n))
        checks["rccl_comm_on_member_device"] = all(m["comm_device"] == m["device"] for m in members)
    log(f"validation: {checks}")
    return {"members": members, "rays_per_frame": [int(frame_rays[0]), int(frame_rays[1])],
            "one_gpu_frame_rays": [int(s1.closest_rays), int(s1.shadow_rays)],
            "gathered_frame_sha256_16": gathered_hash, "one_gpu_frame_sha256_16": one_hash,
            "checks": checks, "ok": all(checks.values()),
            "note": "members from rtx_group_member_info (ncclCommCount / ncclCommUserRank / ncclCommCuDevice, "
                    "hipDeviceCanAccessPeer both ways with device 0, hipDeviceGetPCIBusId); the N = 1 frame from one "
                    "context on device 0 after the timed steps; bench.py exits non-zero after printing when ok is false"}


def main_group(a):
    """--gpus N > 1 in one process: the C-ABI device group (rtx_group_*), the path engine --gpus N
    ships.  A step is rtx_group_render: every device renders its tile shard on its own host
    thread, devices 1..N-1 pack their shards and RCCL send/recv moves them to device 0, which
    unpacks and copies the frame to (pinned) host memory.  The line carries every device's
    kernel times (balance) and the roofline of device 0's k_shadow from a counting render."""
    import numpy as np
    import rtxpy
    from rtxpy import abi

    def log(msg):
        print(f"[group] {msg}", file=sys.stderr, flush=True)

    path = scene_path(a.scene)
    scene = rtxpy.Scene.load(path, base_dir=os.path.join(ROOT, "tests", "golden"))
    if a.dry_run:  # the schema of the line, without a GPU
        dev0 = {"device": 0, "kernel_ms": None, "trace_ms": None, "shadow_ms": None, "rays": None}
        out = group_line(a, a.gpus, os.path.basename(path), int(scene.num_objects), None, None, None,
                         [dict(dev0, device=r) for r in range(a.gpus)], None,
                         {"bound": "valu", "achieved": None, "peak": VALU_PEAK_GINST, "unit": "Ginst/s", "frac": None,
                          "traffic": None, "kernel": "k_shadow", "device": 0})
        out["dry_run"] = True
        mkeys = ("device", "comm_count", "comm_rank", "comm_device", "can_access_peer0", "peer0_can_access",
                 "peer_enabled", "transport", "pci_bus_id")
        out["validation"] = {"members": [dict.fromkeys(mkeys) for _ in range(a.gpus)], "rays_per_frame": None,
                             "one_gpu_frame_rays": None, "gathered_frame_sha256_16": None,
                             "one_gpu_frame_sha256_16": None,
                             "checks": dict.fromkeys(("members_are_gpus", "distinct_devices", "rays_sum_to_one_gpu_frame",
                                                      "gathered_frame_is_one_gpu_frame", "rccl_comms_count_n",
                                                      "rccl_ranks_distinct", "rccl_comm_on_member_device")),
                             "ok": None}
        print(json.dumps(out), flush=True)
        return
    import torch
    frame = scene.frame(a.width, a.height)
    flags = flags_for(a.scene, a.spp)
    params = rtxpy.params_from_args(flags, seed=1)
    params.rng = abi.RTX_RNG_COUNTER  # the reference's i.i.d. light samples
    g = rtxpy.Group([0], loopback=a.gpus) if a.loopback else rtxpy.Group(list(range(a.gpus)))
    n = g.size()
    g.set_option(abi.RTX_OPT_SHADOW_WALK, WALKS[a.walk])
    g.set_option(abi.RTX_OPT_TRACE_WALK, WALKS[a.trace_walk])
    g.set_option(abi.RTX_OPT_SHADOW_SLOT, a.shadow_slot)
    g.set_option(abi.RTX_OPT_TREE_FRAME, FRAMES[a.frame])
    g.set_option(abi.RTX_OPT_SHADOW_CULL, 0 if a.no_cull else 2 if a.cull_slots else 1)
    if a.shadow_grab:
        g.set_option(abi.RTX_OPT_SHADOW_GRAB, a.shadow_grab)
    t0 = time.perf_counter()
    g.upload(scene)
    upload_ms = (time.perf_counter() - t0) * 1e3
    s0 = g.device_stats(0)
    log(f"{n} devices, scene {os.path.basename(path)} uploaded in {time.perf_counter() - t0:.2f}s "
        f"(build on device 0 {s0.build_ms:.1f} ms, tree frame {'rotated' if s0.tree_rotated else 'world'})")
    h_rgb = torch.empty((a.height, a.width, 3), dtype=torch.float32, pin_memory=True).numpy()
    h_z = torch.empty((a.height, a.width), dtype=torch.float32, pin_memory=True).numpy()
    for i in range(a.warmup):
        g.render(frame, params, h_rgb, h_z)
        s = g.stats()
        log(f"warmup {i}: {s.kernel_ms:.1f} ms (slowest device), gather {s.gather_ms:.2f} ms")
    t0 = time.perf_counter()
    rays = closest = 0
    dev = [[] for _ in range(n)]
    gms = []
    for i in range(a.steps):
        g.render(frame, params, h_rgb, h_z)
        s = g.stats()
        rays += s.closest_rays + s.shadow_rays
        closest += s.closest_rays
        gms.append(s.gather_ms)
        for r in range(n):
            d = g.device_stats(r)
            dev[r].append((d.kernel_ms, d.trace_ms, d.shadow_ms, d.closest_rays + d.shadow_rays))
    elapsed = time.perf_counter() - t0
    per_dev = []
    for r in range(n):
        m = np.array(dev[r], dtype=np.float64).mean(0)
        per_dev.append({"device": r, "kernel_ms": round(m[0], 3), "trace_ms": round(m[1], 3), "shadow_ms": round(m[2], 3),
                        "rays": int(m[3])})
    validation = group_validation(a, g, n, scene, frame, params, h_rgb, h_z, (s.closest_rays, s.shadow_rays), log)
    roofline = None
    if not a.no_count:
        p2 = rtxpy.default_params(**{f: getattr(params, f) for f, _ in abi.Params._fields_})
        p2.count_traversal = 1
        g.render(frame, p2, h_rgb, h_z)
        roofline = shadow_roofline_of(g.device_stats(0), per_dev[0]["shadow_ms"], a, n)
        roofline["device"] = 0
        roofline["note"] = "device 0's k_shadow over its shard (tiles t % N == 0), counts from a counting render"
    upload = {"wall_ms": round(upload_ms, 1), "build_ms_device0": round(s0.build_ms, 1),
              "peer_copy_ms": [round(g.device_stats(r).upload_copy_ms, 1) for r in range(n)]}
    g.close()
    cpu = None
    if a.loopback and not a.no_cpu_baseline:  # N > 1 devices: the baseline belongs to the N = 1 line
        try:
            cpu = cpu_reference(path, flags, a.width, a.height, a.cpu_target_s, log)
        except Exception as e:  # never let the baseline kill the measurement
            log(f"reference baseline failed: {e}")
    out = group_line(a, n, os.path.basename(path), int(scene.num_objects), elapsed, rays, closest, per_dev,
                     round(float(np.mean(gms)), 3), roofline, cpu, upload)
    out["validation"] = validation
    if cpu and out["value"]:
        out["config"]["gpu_over_cpu"] = round(out["value"] / cpu["value"], 1)
    print(json.dumps(out), flush=True)
    if not validation["ok"]:
        print(f"bench.py: the {n}-device group failed its own checks: {validation['checks']}", file=sys.stderr)
        sys.exit(3)


if __name__ == "__main__":
    main()
