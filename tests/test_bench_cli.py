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
    p = run(["--gpus", "2", "--dry-run", "--launch", "torchrun"])
    assert p.returncode == 0, p.stderr[-2000:]
    line = [l for l in p.stdout.splitlines() if l.startswith("{")][-1]
    out = json.loads(line)
    assert out["n_gpus"] == 2 and out["ranks_joined"] == 2 and out["launch"] == "torchrun"
    assert out["world_size"] == 2 and out["ranks_seen"] == [0, 1] and out["backend"] == "gloo"


def test_gpus_flag_without_torchrun_drives_the_device_group():
    """`--gpus N` run directly: one process drives rtx_group over N devices (the path
    `engine --gpus N` ships), no child ranks are started."""
    p = run(["--gpus", "4", "--dry-run"])
    assert p.returncode == 0, p.stderr[-2000:]
    out = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
    assert out["dry_run"] and out["n_gpus"] == 4 and out["config"]["launch"] == "group"


def test_group_line_schema():
    """the device-group line (--gpus N, one process): the contract's keys, every device's kernel
    times (balance), the gather time and device 0's k_shadow roofline"""
    p = run(["--gpus", "8", "--dry-run", "--scene", "scene3", "--spp", "16"])
    assert p.returncode == 0, p.stderr[-2000:]
    out = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline", "closest_mrays"):
        assert k in out, k
    assert out["metric"].startswith("Mrays/s") and out["n_gpus"] == 8 and out["scaling"] == "strong"
    assert out["config"]["workload"].endswith("(BASELINE configs[1])")
    devs = out["group"]["devices"]
    assert [d["device"] for d in devs] == list(range(8))
    assert all({"kernel_ms", "trace_ms", "shadow_ms", "rays"} <= set(d) for d in devs)
    assert "gather_ms" in out["group"] and out["group"]["rccl_devices"] == 8
    assert "upload" in out["group"]  # per-device copy times of the scene built on device 0
    assert "i.i.d." in out["config"]["rng"]  # the reference's sampling (system.c:93-96)
    assert "cpu_baseline_note" in out  # the same reference CPU leg as the N=1 line, after the GPU steps
    rl = out["roofline"]
    assert rl["kernel"] == "k_shadow" and rl["device"] == 0 and {"bound", "achieved", "peak", "unit", "frac", "traffic"} <= set(rl)
    # the line validates itself (members read back from RCCL / HIP, the N = 1 frame)
    v = out["validation"]
    assert len(v["members"]) == 8 and {"comm_count", "comm_rank", "comm_device", "can_access_peer0",
                                       "peer0_can_access", "pci_bus_id"} <= set(v["members"][0])
    assert {"rays_sum_to_one_gpu_frame", "gathered_frame_is_one_gpu_frame", "rccl_comms_count_n",
            "rccl_ranks_distinct", "distinct_devices"} <= set(v["checks"])
    assert {"one_gpu_frame_rays", "gathered_frame_sha256_16", "one_gpu_frame_sha256_16", "ok"} <= set(v)


def test_workload_labels_name_the_baseline_config():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    A = type("A", (), {})
    for scene, w, h, spp, want in [("scene5", 1920, 1080, 64, "configs[2]"), ("scene3", 1920, 1080, 16, "configs[1]"),
                                   ("scene6", 3840, 2160, 128, "configs[4]"), ("scene5", 1920, 1080, 256, "configs[3]"),
                                   ("scene1", 512, 512, 64, "configs[0]"), ("scene5", 960, 540, 64, "custom"),
                                   ("scene5_l8", 1920, 1080, 64, "level-8 dragon bracket")]:
        a = A()
        a.scene, a.width, a.height, a.spp = scene, w, h, spp
        assert want in b.workload(a), (scene, b.workload(a))
    a = A()
    a.scene = "scene3"
    assert "no mesh" in b.data_label(a)
    a.scene = "scene6"
    assert "Menger" in b.data_label(a)


def test_gpus_flag_must_match_torchrun_world():
    p = run(["--gpus", "2", "--dry-run"], {"WORLD_SIZE": "3", "RANK": "0"})
    assert p.returncode == 2 and "WORLD_SIZE=3" in p.stderr


def test_pmc_summary_sums_a_chunked_frame(tmp_path, monkeypatch):
    """tools/pmc_summary.py: a frame rendered in two chunks launches k_shadow twice with unequal
    work; the per-frame counts the bench's roofline uses are the sum over the launches, not
    twice the mean of one (both agree only for equal chunks)."""
    import importlib.util
    import csv
    spec = importlib.util.spec_from_file_location("pmc_summary", os.path.join(ROOT, "tools", "pmc_summary.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    d = tmp_path / "pmc"
    d.mkdir()
    with open(d / "run_counter_collection.csv", "w", newline="") as fh:
        w = csv.DictWriter(fh, fieldnames=["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for disp, v in ((1, 1631.0), (2, 701.0)):
            w.writerow({"Dispatch_Id": disp, "Kernel_Name": "void k_shadow<false, 8, 2>(KShadow)",
                        "Counter_Name": "SQ_INSTS_VALU", "Counter_Value": v})
        w.writerow({"Dispatch_Id": 3, "Kernel_Name": "k_trace", "Counter_Name": "SQ_INSTS_VALU", "Counter_Value": 5.0})
    mean, n = m.per_launch(str(d), "k_shadow")
    assert n == 2 and mean["SQ_INSTS_VALU"] == 1166.0
    assert m.per_frame(str(d), "k_shadow", 1)["SQ_INSTS_VALU"] == 2332.0
    assert m.per_frame(str(d), "k_shadow", 2)["SQ_INSTS_VALU"] == 1166.0


def test_roofline_issue_slots(tmp_path, monkeypatch):
    """bench.py's roofline: the VALU issue slots the kernel used (SQ_INSTS_VALU minus the
    quad-cycles that issued two, SQ_ACTIVE_INST_VALU2) over the chip's in the kernel's time, from a
    PMC summary whose source hash matches the kernel."""
    import types
    import bench
    (tmp_path / "profiles").mkdir()
    key = "scene5_1920x1080_n64_g1"
    rec = {key: {"kernel_src_sha": bench.shadow_src_sha(), "sq_insts_valu": 4.0e11, "sq_insts_valu_frame": 4.0e11,
                 "sq_active_inst_valu2": 1.0e11, "sq_active_inst_valu2_frame": 1.0e11,
                 "hbm_bytes_per_launch": 1e11, "hbm_bytes_per_frame": 1e11}}
    with open(tmp_path / "profiles" / "pmc_k_shadow.json", "w") as fh:
        json.dump(rec, fh)
    sha = bench.shadow_src_sha()
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    monkeypatch.setattr(bench, "shadow_src_sha", lambda: sha)
    n = dict(shade_points=7e7, shadow_tri_tests=1.8e10, shadow_sphere_tests=0, shadow_global_box_tests=5e11,
             shadow_box_tests=5.2e11, shadow_plane_tests=2.1e10, shadow_rays=2.1e10, shadow_wave_steps=1.6e9,
             shadow_wave_walks=3.5e8, shadow_leaf_rounds=7.6e8, shadow_uniform_steps=6.4e8, closest_rays=1.35e8,
             node_visits=6e9, shadow_node_visits=5e9, tri_tests=2e10, sphere_tests=0, wide_nodes=63578, wide_depth=8,
             chunks=1)
    c = types.SimpleNamespace(**n)
    a = types.SimpleNamespace(scene="scene5", width=1920, height=1080, spp=64)
    out = bench.shadow_roofline_of(c, 500.0, a, 1)
    assert out["pmc"]["matches_this_kernel"]
    s = out["issue_slots"]
    avail = 0.5 * 2.4e9 / 4 * 1024
    assert s["used_quad_cycles"] == int(3.0e11) and abs(s["frac"] - 3.0e11 / avail) < 1e-4
    assert s["dual_issued_frac"] == 0.5
    # the same launch on SURVEY 8(d)'s FLOP and byte-model bases beside the VALU ones
    b = out["bases"]
    flop = 12 * 5.2e11 + 27 * 1.8e10
    assert abs(b["flop"]["frac"] - flop / 0.5 / 1e12 / 157.3) < 1e-4
    model = 64 * 5.2e11 / 8 + 48 * 1.8e10 + 16 * 2.1e10 + 48 * 2.1e10
    assert b["bytes_model"]["bytes_per_launch"] == int(model)
    assert abs(b["bytes_model"]["x_hbm_peak"] - model / 0.5 / 8e12) < 1e-3
    assert b["valu_useful"]["frac"] == out["frac"] and b["valu_issue_slots"]["frac"] == s["frac"]
    assert abs(b["hbm_pmc"]["frac"] - 1e11 / 0.5 / 8e12) < 1e-4 and "binding" in b
