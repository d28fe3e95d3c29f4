"""Secondary benchmark: the whole search loop with a network (SURVEY.md §8d "Full-loop").

One step = one environment step of the self-play loop (selfplay_worker.py:187-211): the N agents
of the map are searched one after another with `SampledMCTS.batch_search`, each over B roots x S
simulations, with the network on the GPU. The network is `mazero_amd.nets.MuZeroShapedNet`:
the SMAC MAMuZeroNet's shapes with MLP heads and random weights, run under autocast as the
reference runs it.

Reported, as one JSON line:
- `device`: mazero_amd.mcts_sampled.SampledMCTS. The tree, pool and glue are on the GPU, and
  the search loop is captured in a HIP graph after the first search of each configuration.
- `device_eager`: the same driver without graphs.
- `selfplay_step_host_consumers` / `selfplay_step_device_consumers`: a whole self-play step with
  its per-root decisions (select_action, epsilon-greedy, recorded policy probability,
  selfplay_worker.py:189-293) made by the reference's Python on the host (oracle/consume.py) or
  by the device consumers (mazero_amd.consume); both on the `device` search.
- `reference_loop` (when oracle/_ref is built): the reference driver restated in
  oracle/driver.py, i.e. numpy glue, vstack gathers and the reference C++ ctree on one host
  core, driving the same GPU network. This is what a reference self-play step costs on this
  machine. Its results are checked bit for bit against `device` on the first step.

This is not the headline metric (bench.py is); the network is synthetic and its cost is the
same for both.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
import mazero_amd  # noqa: E402,F401  (HIP runtime settings, before anything initialises HIP)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

MAPS = {"3m": (3, 9), "2s3z": (5, 11), "3s5z_vs_3s6z": (8, 15), "27m_vs_30m": (27, 36)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--map", default="3m", choices=sorted(MAPS))
    ap.add_argument("--roots", type=int, default=256)
    ap.add_argument("--sims", type=int, default=50)
    ap.add_argument("--sampled-times", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--ref-steps", type=int, default=2)
    ap.add_argument("--no-ref", action="store_true")
    ap.add_argument("--device-only", action="store_true",
                    help="only the graph-replayed device loop (profiling runs: with MZ_TRACE_MARKS=1 two one-element "
                         "fills mark its timed region for scripts/search_split.py)")
    args = ap.parse_args()

    import torch

    from mazero_amd.mcts_sampled import SampledMCTS
    from mazero_amd.nets import SearchConfig, make_net, make_root_batch

    N, A = MAPS[args.map]
    B, S, K = args.roots, args.sims, args.sampled_times
    dev = torch.device("cuda", 0)
    cfg = SearchConfig(action_space_size=A, num_simulations=S, sampled_action_times=K)
    net = make_net(N, A, seed=0, device=dev)
    roots = [make_root_batch(net, B, 64, seed=10 + i, device=dev, legal_zero_frac=0.2) for i in range(3)]

    def env_step(mcts, i):
        out, legal = roots[i % len(roots)]
        acts = np.zeros((B, N), np.int32)
        res = None
        for agent in range(N):  # selfplay_worker.py:196-211
            factor = acts[:, :agent].copy() if agent else None
            res = mcts.batch_search(net, out, agent, factor, N, legal, device=dev, add_noise=True)
            acts[:, agent] = [int(a[np.argmax(v), 0]) if len(a) else 0
                              for a, v in zip(res.sampled_actions, res.sampled_visit_count)]
        return res

    def mark(k):  # (MZ_TRACE_MARKS=1: FillFunctor<short> in a rocprofv3 kernel trace, outside the timing)
        if os.environ.get("MZ_TRACE_MARKS") == "1":
            torch.full((1,), k, dtype=torch.int16, device=dev)

    def timed(mcts, steps, warm, marks=False):
        for i in range(warm):
            env_step(mcts, i)
        if marks:
            mark(1)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            env_step(mcts, i)
        torch.cuda.synchronize()
        t = (time.perf_counter() - t0) / steps
        if marks:
            mark(2)
        return t

    sims_per_step = B * S * N
    line = {"metric": f"full search loop simulations/s, SMAC {args.map} ({N} agents x {B} roots x {S} sims, K={K})",
            "unit": "simulations/s", "network": "MuZeroShapedNet (MLP heads, random init, autocast)"}
    t = timed(SampledMCTS(cfg, np.random.RandomState(0), use_graph=True), args.steps, 2, marks=True)
    line["device"] = {"value": round(sims_per_step / t, 1), "ms_per_step": round(t * 1e3, 3)}
    if args.device_only:
        line["steps"] = args.steps
        print(json.dumps(line), flush=True)
        return
    t = timed(SampledMCTS(cfg, np.random.RandomState(0), use_graph=False), max(1, args.steps // 2), 1)
    line["device_eager"] = {"value": round(sims_per_step / t, 1), "ms_per_step": round(t * 1e3, 3)}

    # One whole self-play step (selfplay_worker.py:189-293): the agents' searches plus the per-root
    # decisions (select_action, epsilon-greedy, recorded policy probability), with the decisions
    # made by the reference's Python on the host or by the device consumers (mazero_amd.consume).
    from consume import selfplay_step
    from mazero_amd.consume import selfplay_decisions

    class _DictSearch(SampledMCTS):
        def batch_search(self, *a, **k):
            return super().batch_search(*a, **k)._asdict()

    ur = np.random.default_rng(1)
    u_eps, u_cat = ur.random((N, B)).astype(np.float32), ur.random((N, B))

    def timed_step(fn, steps, warm):
        for i in range(warm):
            fn(i)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            fn(i)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps

    rs_h, rs_d = np.random.default_rng(3), np.random.default_rng(3)
    m_h, m_d = _DictSearch(cfg, rs_h), SampledMCTS(cfg, rs_d)

    def host_decisions(i):
        out, legal = roots[i % len(roots)]
        return selfplay_step(m_h, net, out, N, legal, 1.0, 1.0, 0.1, rs_h, u_eps, u_cat, device=dev)["actions"]

    def device_decisions(i):
        out, legal = roots[i % len(roots)]
        d = selfplay_decisions(m_d, net, out, N, legal, temperature=1.0, greedy_epsilon=0.1,
                               eps_uniforms=(u_eps, u_cat), device=dev)
        return d.actions.cpu().numpy()  # the environment step needs the actions on the host

    same_dec = bool(np.array_equal(host_decisions(0), device_decisions(0)))
    t = timed_step(host_decisions, args.steps, 1)
    line["selfplay_step_host_consumers"] = {"ms_per_step": round(t * 1e3, 3), "value": round(sims_per_step / t, 1)}
    t = timed_step(device_decisions, args.steps, 1)
    line["selfplay_step_device_consumers"] = {"ms_per_step": round(t * 1e3, 3), "value": round(sims_per_step / t, 1),
                                              "actions_equal_host_consumers": same_dec}

    ref_path = os.path.join(ROOT, "oracle", "_ref", "libmzref.so")
    if not args.no_ref and os.path.exists(ref_path):
        import ctypes as C

        from driver import OracleSampledMCTS
        from mazero_amd import _capi

        lib = _capi.bind(C.CDLL(ref_path))

        class _Adapter(OracleSampledMCTS):
            def batch_search(self, *a, **k):
                from mazero_amd.mcts_sampled import SearchOutput

                return SearchOutput(**super().batch_search(*a, **k))

        # parity spot check on one env step
        a = env_step(_Adapter(cfg, np.random.RandomState(7), lib), 0)
        b = env_step(SampledMCTS(cfg, np.random.RandomState(7)), 0)
        same = all(np.array_equal(np.asarray(x), np.asarray(y)) if not isinstance(x, list)
                   else all(np.array_equal(u, v) for u, v in zip(x, y)) for x, y in zip(a, b))
        t = timed(_Adapter(cfg, np.random.RandomState(0), lib), args.ref_steps, 0)
        line["reference_loop"] = {"value": round(sims_per_step / t, 1), "ms_per_step": round(t * 1e3, 3),
                                  "tree": "reference ctree (oracle/_ref), 1 host core", "bit_exact_vs_device": same}
        line["speedup_vs_reference_loop"] = round(line["device"]["value"] / line["reference_loop"]["value"], 2)
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
