"""Debug: the graph-replay driver test with per-step reporting."""
import os, sys, ctypes as C
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import numpy as np, torch
from mazero_amd import _capi
from driver import OracleSampledMCTS
from mazero_amd.mcts_sampled import SampledMCTS
from mazero_amd.nets import SearchConfig, make_net, make_root_batch
port = _capi.bind(C.CDLL("oracle/_build/libmzport.so"))
for K in (1, 5):
    N, A, B, S, cur = 3, 9, 64, 20, 1
    dev = torch.device("cuda", 0)
    cfg = SearchConfig(action_space_size=A, num_simulations=S, sampled_action_times=K)
    net = make_net(N, A, seed=12, device=dev)
    rs_o, rs_d = np.random.RandomState(5), np.random.RandomState(5)
    oracle = OracleSampledMCTS(cfg, rs_o, port)
    drv = SampledMCTS(cfg, rs_d, use_graph=(len(sys.argv) < 2))
    for step in range(4):
        out, legal = make_root_batch(net, B, 64, seed=100 + step, device=dev, legal_zero_frac=0.25)
        factor = np.random.default_rng(step).integers(0, A, size=(B, cur)).astype(np.int32)
        exp = oracle.batch_search(net, out, cur, factor, N, legal, device=dev, add_noise=True)
        try:
            got = drv.batch_search(net, out, cur, factor, N, legal, device=dev, add_noise=True)
            print(f"K={K} step {step}: values equal {np.array_equal(got.value, exp['value'])}", flush=True)
        except Exception as e:
            print(f"K={K} step {step}: {e}", flush=True)
            from mazero_amd.mcts_sampled import _TREES
            for tb in _TREES.values():
                tb.print()
            break
