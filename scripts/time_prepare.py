"""Times mz_prepare / mz_prepare_select alone (HIP events over back-to-back launches) for one
BASELINE configuration; with MZ_LIB_OVERRIDE=<variant .so> for ablation builds."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from mazero_amd.cytree import Tree_batch  # noqa: E402
from mazero_amd.synthetic import DEFAULTS, make_search_inputs  # noqa: E402


def main():
    B, A, K, S = (int(x) for x in (sys.argv[1:5] if len(sys.argv) > 4 else (256, 9, 1, 50)))
    inp = make_search_inputs(np.random.default_rng(0), B, A, S)
    d = DEFAULTS
    dev = torch.device("cuda")
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    rr, rv, rp, rb, rn = (t(x) for x in (inp.root_reward, inp.root_value, inp.root_policy, inp.root_beta, inp.root_noise))
    tb = Tree_batch(B, 1, A, K, S, d["delta_lb"], inp.seed, d["rho"], d["lam"])
    out = (torch.empty(B, dtype=torch.int32, device=dev), torch.empty(B, dtype=torch.int32, device=dev),
           torch.empty(B, 1, dtype=torch.int32, device=dev))
    c2, c1, g = d["pb_c_base"], d["pb_c_init"], d["discount"]
    for _ in range(20):
        tb.prepare_selection_device(rr, rv, rp, rb, K, inp.noise_eps, rn, c2, c1, g, out=out)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        for _ in range(50):
            tb.prepare_selection_device(rr, rv, rp, rb, K, inp.noise_eps, rn, c2, c1, g, out=out)
    res = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        graph.replay()
        e1.record()
        e1.synchronize()
        res.append(e0.elapsed_time(e1) * 1e3 / 50)
    print(f"prepare_select B={B} A={A} K={K} S={S}: {np.median(res):.2f} us per launch")


if __name__ == "__main__":
    main()
