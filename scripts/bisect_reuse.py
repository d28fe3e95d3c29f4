"""Diagnostic: test_graph_reuse_keys_on_search_constants's sequence under each driver mode
(device_root on/off, graph on/off), reporting which (step, config) searches differ from the oracle."""
import dataclasses
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]

from driver import OracleSampledMCTS  # noqa: E402
import ctypes as C  # noqa: E402
import mazero_amd  # noqa: E402,F401
from mazero_amd import _capi  # noqa: E402
from mazero_amd import mcts_sampled  # noqa: E402
from mazero_amd.mcts_sampled import SampledMCTS  # noqa: E402
from mazero_amd.nets import SearchConfig, make_net, make_root_batch  # noqa: E402


def diff(got, exp):
    bad = []
    for name in exp:
        g, e = getattr(got, name), exp[name]
        if isinstance(e, list):
            if any(not np.array_equal(np.asarray(a).view(np.uint8), np.asarray(b).view(np.uint8)) for a, b in zip(g, e)):
                bad.append(name)
        elif not np.array_equal(np.asarray(g).view(np.uint8), np.asarray(e).view(np.uint8)):
            bad.append(name)
    return bad


def main():
    port = _capi.bind(C.CDLL(os.path.join(ROOT, "oracle", "_build", "libmzport.so")))
    N, A, B, S, cur = 3, 9, 32, 12, 0
    dev = torch.device("cuda", 0)
    base = SearchConfig(action_space_size=A, num_simulations=S, sampled_action_times=int(os.environ.get("K", 3)))
    cfgs = [base, dataclasses.replace(base, discount=0.9), dataclasses.replace(base, pb_c_init=2.5, pb_c_base=500.0)]
    only = os.environ.get("ONLY")
    if only:
        cfgs = [cfgs[int(c)] for c in only.split(",")]
    for device_root in (True, False):
        for use_graph in (True, False):
            mcts_sampled._LOOPS.clear()
            mcts_sampled._TREES.clear()
            net = make_net(N, A, seed=31, device=dev)
            res = []
            for step in range(3):
                for j, cfg in enumerate(cfgs):
                    out, legal = make_root_batch(net, B, 64, seed=200 + 10 * step + j, device=dev, legal_zero_frac=0.2)
                    rs_o, rs_d = np.random.RandomState(step), np.random.RandomState(step)
                    exp = OracleSampledMCTS(cfg, rs_o, port).batch_search(net, out, cur, None, N, legal, device=dev,
                                                                        add_noise=True)
                    got = SampledMCTS(cfg, rs_d, use_graph=use_graph, device_root=device_root).batch_search(
                        net, out, cur, None, N, legal, device=dev, add_noise=True)
                    b = diff(got, exp)
                    res.append(f"s{step}c{j}:{'ok' if not b else ','.join(b)}")
            print(f"device_root={device_root} graph={use_graph}: {' '.join(res)}", flush=True)


if __name__ == "__main__":
    main()
