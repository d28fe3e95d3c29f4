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
    assert not a.strong and not a.no_graph


def test_cpu_baseline_fields(port_lib):
    import bench
    from mazero_amd.synthetic import make_search_inputs

    rng = np.random.default_rng(0)
    B, A, K, S, N = 16, 9, 1, 10, 3
    inputs = [make_search_inputs(rng, B, A, S) for _ in range(N)]
    r = bench.cpu_baseline(inputs, B, A, K, S, N, 0.2)
    assert r is not None
    assert r["unit"] == "simulations/s" and r["cores"] == 1 and r["kind"] in ("reference", "port")
    assert r["value"] > 0 and "sims" in r["sample"]
    mc = r["multi_core"]
    assert mc["value"] > 0 and 1 <= mc["threads"] <= 16
