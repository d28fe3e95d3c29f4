"""Where the tree-level drop-in's time goes (bench.py --dropin's loop, one call type at a time).

    python scripts/dropin_split.py [--map 3m] [--sampled-times 1] [--steps 5]

Runs the reference driver's per-search Tree_batch calls (mcts_sampled.py:89-191 minus the network)
on mazero_amd.cytree with host numpy arrays, as bench.py --dropin does, and reports the host wall
time per call of each kind (create, prepare, batch_selection, batch_expansion_and_backup, the two
root readbacks).  batch_selection includes the synchronisation that waits for the GPU; with the
staged host path it also carries the expansion staged by the previous call.  Diagnostics only.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import mazero_amd  # noqa: E402,F401

MAPS = {"3m": (3, 9), "2s3z": (5, 11), "3s5z_vs_3s6z": (8, 15), "27m_vs_30m": (27, 36)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--map", default="3m", choices=sorted(MAPS))
    ap.add_argument("--roots", type=int, default=256)
    ap.add_argument("--sims", type=int, default=50)
    ap.add_argument("--sampled-times", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    import torch  # noqa: F401

    from mazero_amd._lib import load
    from mazero_amd.cytree import Tree_batch
    from mazero_amd.synthetic import DEFAULTS, make_search_inputs

    N, A = MAPS[a.map]
    B, S, K = a.roots, a.sims, a.sampled_times
    d = DEFAULTS
    c2, c1, g = d["pb_c_base"], d["pb_c_init"], d["discount"]
    lib = load()
    rng = np.random.default_rng(0)
    inputs = [make_search_inputs(rng, B, A, S) for _ in range(N)]
    tm = {k: 0.0 for k in ("create", "prepare", "select", "expand", "readback")}
    cnt = {k: 0 for k in tm}

    def clock(k, f, *args):
        t0 = time.perf_counter()
        r = f(*args)
        tm[k] += time.perf_counter() - t0
        cnt[k] += 1
        return r

    def step():
        for inp in inputs:
            tb = clock("create", Tree_batch, B, 1, A, K, S, d["delta_lb"], inp.seed, d["rho"], d["lam"])
            clock("prepare", tb.prepare, inp.root_reward, inp.root_value, inp.root_policy, inp.root_beta, K,
                  inp.noise_eps, inp.root_noise)
            for s in range(S):
                clock("select", tb.batch_selection, c2, c1, g)
                clock("expand", tb.batch_expansion_and_backup, s + 1, g, K, inp.reward[s], inp.value[s],
                      inp.policy[s], inp.beta[s])
            clock("readback", tb.get_roots_values)
            clock("readback", tb.get_roots_marginal_visit_count)

    for _ in range(2):
        step()
    for k in tm:
        tm[k], cnt[k] = 0.0, 0
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    wall = time.perf_counter() - t0
    sims = a.steps * N * B * S
    out = dict(map=a.map, roots=B, sims=S, K=K, steps=a.steps, host_copy=os.environ.get("MZ_HOST_COPY") == "1",
               sims_per_s=round(sims / wall, 1), us_per_sim_call_pair=round(wall / (a.steps * N * S) * 1e6, 2),
               us_per_call={k: round(tm[k] / max(1, cnt[k]) * 1e6, 2) for k in tm},
               us_per_step={k: round(tm[k] / a.steps * 1e6, 1) for k in tm})
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
