"""bench.py contract pieces that run without a GPU: argument defaults (N = 1, the headline
configuration) and the CPU baseline leg (the oracle library timed on host cores, one core plus the
multi-core leg), on a small sample."""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_defaults_are_the_headline_config():
    import bench

    a = bench.parse([])
    assert (a.map, a.roots, a.sims, a.sampled_times) == ("3m", 256, 50, 1)
    assert not a.strong and not a.no_graph and a.broadcast_every == 0


def test_cpu_baseline_fields(port_lib):
    import bench
    from mazero_amd.synthetic import make_search_inputs

    rng = np.random.default_rng(0)
    B, A, K, S, N = 16, 9, 1, 10, 3
    inputs = [make_search_inputs(rng, B, A, S) for _ in range(N)]
    r = bench.cpu_baseline(inputs, B, A, K, S, N, 0.4, procs=2)
    assert r is not None
    assert r["unit"] == "simulations/s" and r["cores"] == 1 and r["kind"] in ("reference", "port")
    assert r["value"] > 0 and "sims" in r["sample"]
    mc = r["multi_core"]
    assert mc["value"] > 0 and mc["processes"] == 2 and mc["cores"] == 2


def test_gpus_flag_spawns_ranks(port_lib):
    """`bench.py --gpus 2` without torchrun starts two ranks itself (torch.distributed.run), each
    rank reports the job's world size, and rank 0 prints one JSON line.  `value` is the weak leg:
    every rank searches its own --roots roots (one shard of the node's self-play per GPU, the
    "whole node" of the metric); the strong leg (--roots roots split over the ranks) rides beside
    it.  --backend port keeps it on the CPU (gloo): the plumbing, not a measurement."""
    import json
    import subprocess

    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    base = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "port", "--roots", "8",
            "--sims", "6", "--steps", "2", "--warmup", "1", "--no-cpu"]
    r = subprocess.run(base, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["scaling"] == "weak"
    assert line["config"]["roots_total"] == 16 and line["config"]["roots_per_gpu"] == 8
    assert "8 roots" in line["metric"] and "per GPU" in line["metric"]
    st = line["strong_scaling"]
    assert st["roots_total"] == 8 and st["roots_per_gpu"] == 4 and st["value"] > 0
    assert line["value"] > 0
    # the line verifies itself: the collective's world size, every rank's device and own step time
    # in both legs; the headline ms_per_step is the max over ranks
    rk = line["ranks"]
    assert rk["world_size"] == 2 and rk["backend"] == "gloo"
    assert [r["rank"] for r in rk["per_rank"]] == [0, 1]
    assert [r["local_rank"] for r in rk["per_rank"]] == [0, 1]
    for r in rk["per_rank"]:
        assert set(r["ms_per_step"]) == {"strong", "weak"} and min(r["ms_per_step"].values()) > 0
        assert r["device"] == "cpu"
    assert abs(max(r["ms_per_step"]["weak"] for r in rk["per_rank"]) - line["ms_per_step"]) < 1e-3
    assert abs(max(r["ms_per_step"]["strong"] for r in rk["per_rank"]) - st["ms_per_step"]) < 1e-3
    # --strong: the strong leg is the headline (the 8 roots split over the two ranks)
    r = subprocess.run(base + ["--strong"], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][0])
    assert line["scaling"] == "strong" and line["config"]["roots_total"] == 8
    assert "8 roots" in line["metric"] and "per GPU" not in line["metric"]
    assert line["weak_scaling"]["roots_total"] == 16


def test_gpus_flag_eight_ranks(port_lib):
    """The driver's widest job, rehearsed on the CPU: `bench.py --gpus 8` over gloo with the port
    backend, 256 roots on every rank (the strong leg beside it: 32 per rank); rank 0 prints one line
    naming 8 ranks.  With
    --broadcast-every 1 (BASELINE config #5's weight broadcast in the timed loop) the line carries
    every rank's sync count, checkpoint and own time per sync."""
    import json
    import subprocess

    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--backend", "port", "--sims", "4",
           "--steps", "2", "--warmup", "1", "--no-cpu", "--broadcast-every", "1"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 8 and line["scaling"] == "weak"
    assert line["config"]["roots_total"] == 2048 and line["config"]["roots_per_gpu"] == 256
    assert line["metric"].endswith("SMAC 3m, 256 roots×4 sims per GPU")
    assert line["strong_scaling"]["roots_total"] == 256 and line["strong_scaling"]["roots_per_gpu"] == 32
    rk = line["ranks"]
    assert rk["world_size"] == 8 and [x["rank"] for x in rk["per_rank"]] == list(range(8))
    assert abs(max(x["ms_per_step"]["weak"] for x in rk["per_rank"]) - line["ms_per_step"]) < 1e-3
    # config #5's weight broadcast inside the timed loop (--broadcast-every 1): one sync per env step
    # on every rank, each moving the 27m network's weights from rank 0 (warm-up sync + 2 timed)
    wb = line["weight_broadcast"]
    assert wb["every_steps"] == 1 and wb["syncs"] == 2 and wb["src_rank"] == 0 and wb["bytes"] > 1_000_000
    assert wb["checkpoint"] == 3 and wb["transfers"] == 3 and "27m_vs_30m" in wb["network"]
    assert len(wb["per_rank_ms_per_sync"]) == 8 and min(wb["per_rank_ms_per_sync"]) > 0
    for x in rk["per_rank"]:
        for kind in ("weak", "strong"):
            assert x["weight_broadcast"][kind]["syncs"] == 2 and x["weight_broadcast"][kind]["checkpoint"] == 3


def test_strong_leg_is_the_global_batch(port_lib):
    """The strong leg's ranks search slices of ONE global batch: rank r's inputs are rows [lo, hi)
    of the inputs an unsharded run generates (so N > 1 measures the metric's own job)."""
    import bench
    from mazero_amd.shard import shard_bounds, slice_inputs
    from mazero_amd.synthetic import make_search_inputs

    rng = np.random.default_rng(0)
    full = [make_search_inputs(rng, 10, 9, 4) for _ in range(3)]
    lo, hi = shard_bounds(10, 4, 1)
    part = [slice_inputs(x, lo, hi) for x in full]
    assert part[0].B == hi - lo and np.array_equal(part[2].policy, full[2].policy[:, lo:hi])
    assert bench.parse(["--gpus", "4"]).roots == 256


def test_world_size_mismatch_fails(port_lib):
    """Under a launcher whose world size differs from --gpus, bench.py refuses to report."""
    import subprocess

    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "port", "--roots", "4",
           "--sims", "4", "--steps", "1", "--no-cpu"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "--gpus 2" in (r.stderr + r.stdout)


def test_matrix_config_ptree_leg(port_lib):
    """BASELINE config #1 (matrix, N = 2, A = 3, 8 roots x 25 sims): bench.py knows the map and
    its CPU baseline carries the pure-Python ptree timing beside the ctree's."""
    import bench
    from mazero_amd.synthetic import make_search_inputs

    assert bench.CONFIGS["matrix"] == (2, 3)
    rng = np.random.default_rng(1)
    B, A, K, S, N = 8, 3, 1, 25, 2
    inputs = [make_search_inputs(rng, B, A, S) for _ in range(N)]
    r = bench.cpu_baseline(inputs, B, A, K, S, N, 0.4, procs=2, ptree=True)
    pt = r["ptree"]
    assert pt["value"] > 0 and pt["cores"] == 1 and "ptree" in pt["sample"]
