"""Diagnostic (not product): replay a captured search graph many times with thousands of eager
kernel launches (eager searches on another handle, torch ops) between replays, and check every
replay against the first one (same inputs and seed, so bit-identical readbacks are expected).

    MZ_GRAPH_ENV_EXPERIMENT=1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 python scripts/debug_graph_stress.py [rounds] [eager]

Used to decide which HIP runtime settings keep kernel arguments of replayed graphs intact
(mazero_amd/_hipenv.py).
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import mazero_amd  # noqa: E402,F401  (runtime settings before torch initialises HIP)
import torch  # noqa: E402

from mazero_amd.cytree import Tree_batch  # noqa: E402
from mazero_amd.synthetic import DEFAULTS, make_search_inputs  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    eager = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    dev = torch.device("cuda", 0)
    B, A, K, S, H = 256, 9, 1, 50, 384
    d = DEFAULTS
    c2, c1, g = d["pb_c_base"], d["pb_c_init"], d["discount"]
    inp = make_search_inputs(np.random.default_rng(0), B, A, S)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    r, v, p, b = t(inp.reward), t(inp.value), t(inp.policy), t(inp.beta)
    rr, rv, rp, rb, rn = t(inp.root_reward), t(inp.root_value), t(inp.root_policy), t(inp.root_beta), t(inp.root_noise)
    pool = torch.randn(S + 1, B, H, device=dev)
    leaf = torch.empty(B, H, device=dev)
    sel = torch.empty(3, B, dtype=torch.int32, device=dev)
    out = (sel[0], sel[1], sel[2].view(B, 1))
    values = torch.empty(B, device=dev)
    stream = torch.cuda.Stream()

    def search(tb):
        tb.prepare(rr, rv, rp, rb, K, inp.noise_eps, rn)
        tb.batch_selection_device(c2, c1, g, out=out)
        for s in range(S):
            if s + 1 < S:
                tb.expansion_backup_selection_device(s + 1, g, K, r[s], v[s], p[s], b[s], c2, c1, out=out, pool=pool,
                                                     gather_out=leaf)
            else:
                tb.batch_expansion_and_backup(s + 1, g, K, r[s], v[s], p[s], b[s])

    mk = lambda: Tree_batch(B, 1, A, K, S, d["delta_lb"], inp.seed, d["rho"], d["lam"])  # noqa: E731
    tb, other = mk(), mk()
    with torch.cuda.stream(stream):
        search(tb)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=stream):
        search(tb)
    torch.cuda.synchronize()
    ref = None
    bad = 0
    t0 = time.time()
    for k in range(rounds):
        with torch.cuda.stream(stream):
            graph.replay()
        torch.cuda.synchronize()
        tb.state_changed()
        try:
            got = np.asarray(tb.get_roots_values()).copy()
            err = ""
        except RuntimeError as e:
            got, err = None, str(e)
        if ref is None:
            ref = got
        elif err or not np.array_equal(got.view(np.uint32), ref.view(np.uint32)):
            bad += 1
            print(f"round {k}: replay differs ({err or 'values'})", flush=True)
            if err:
                break
        with torch.cuda.stream(stream):  # churn: eager searches (50 launches each) and torch ops
            for _ in range(eager):
                search(other)
                x = torch.randn(512, 512, device=dev)
                (x @ x).sum()
        torch.cuda.synchronize()
    print(f"{rounds} replays, {eager} eager searches between replays: {bad} bad, "
          f"{time.time() - t0:.1f} s, DEBUG_CLR_GRAPH_PACKET_CAPTURE={os.environ.get('DEBUG_CLR_GRAPH_PACKET_CAPTURE')} "
          f"DEBUG_CLR_KERNARG_HDP_FLUSH_WA={os.environ.get('DEBUG_CLR_KERNARG_HDP_FLUSH_WA')}", flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
