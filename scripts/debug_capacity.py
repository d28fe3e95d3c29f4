"""Diagnostic: reproduce the bench_search self-play sequence and, on a search error, re-run the
failing search eagerly and with the oracle driver from the same generator state."""
import copy
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

from mazero_amd.mcts_sampled import SampledMCTS  # noqa: E402
from mazero_amd.nets import SearchConfig, make_net, make_root_batch  # noqa: E402
from mazero_amd._capi import MZError  # noqa: E402
from consume import select_action, eps_greedy_given  # noqa: E402

N, A, B, S, K = 3, 9, 256, 50, 1
dev = torch.device("cuda", 0)
cfg = SearchConfig(action_space_size=A, num_simulations=S, sampled_action_times=K)
net = make_net(N, A, seed=0, device=dev)
roots = [make_root_batch(net, B, 64, seed=10 + i, device=dev, legal_zero_frac=0.2) for i in range(3)]
graph = os.environ.get("GRAPH", "1") == "1"
pre = int(os.environ.get("PRE", "0"))
eager = int(os.environ.get("EAGER", "0"))
for n_runs, use_g in ((pre, True), (eager, False)):  # the bench's earlier runs (graph, then eager)
    m0 = SampledMCTS(cfg, np.random.RandomState(0), use_graph=use_g)
    for i in range(n_runs):
        out, legal = roots[i % 3]
        acts = np.zeros((B, N), np.int32)
        for agent in range(N):
            res = m0.batch_search(net, out, agent, acts[:, :agent].copy() if agent else None, N, legal, device=dev,
                                  add_noise=True)
            acts[:, agent] = [int(a[np.argmax(v), 0]) for a, v in zip(res.sampled_actions, res.sampled_visit_count)]
ur = np.random.default_rng(1)
u_eps, u_cat = ur.random((N, B)).astype(np.float32), ur.random((N, B))
rs = np.random.default_rng(3)
m = SampledMCTS(cfg, rs, use_graph=graph)
for step in range(3):
    out, legal = roots[step % 3]
    acts = np.full((B, N), -1, np.int32)
    for agent in range(N):
        factor = acts[:, :agent].copy() if agent else None
        st = copy.deepcopy(rs.bit_generator.state)
        try:
            so = m.batch_search(net, out, agent, factor, N, legal, device=dev, add_noise=True)
        except MZError as e:
            print(f"step {step} agent {agent}: {e}", flush=True)
            for g in (False, True):
                r2 = np.random.default_rng(0)
                r2.bit_generator.state = copy.deepcopy(st)
                try:
                    SampledMCTS(cfg, r2, use_graph=g).batch_search(net, out, agent, factor, N, legal, device=dev,
                                                                  add_noise=True)
                    print(f"  rerun use_graph={g}: ok", flush=True)
                except MZError as e2:
                    print(f"  rerun use_graph={g}: {e2}", flush=True)
            from driver import OracleSampledMCTS
            import ctypes as C
            from mazero_amd import _capi
            lib = _capi.bind(C.CDLL(os.path.join(ROOT, "oracle", "_build", "libmzport.so")))
            r3 = np.random.default_rng(0)
            r3.bit_generator.state = copy.deepcopy(st)
            try:
                OracleSampledMCTS(cfg, r3, lib).batch_search(net, out, agent, factor, N, legal, device=dev,
                                                             add_noise=True)
                print("  oracle (port): ok", flush=True)
            except Exception as e3:
                print(f"  oracle (port): {e3}", flush=True)
            np.savez(os.path.join(ROOT, "gpurun_out", "cap_fail.npz"), factor=np.asarray(factor) if factor is not None else np.zeros(0),
                     state=np.frombuffer(repr(st).encode(), np.uint8), step=step, agent=agent)
            sys.exit(1)
        for i in range(B):
            pos, _ = select_action(so.sampled_visit_count[i], 1.0, False, rs)
            acts[i, agent] = eps_greedy_given(so.sampled_actions[i][pos, 0], legal[i, agent], 0.1, u_eps[agent, i],
                                              u_cat[agent, i])
    print(f"step {step} ok", flush=True)
