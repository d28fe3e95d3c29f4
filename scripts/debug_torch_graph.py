"""Diagnostic (not product): does a plain torch HIP graph (no mazero_amd kernels) survive thousands
of eager launches between its capture and its replay under the runtime's graph packet capture?

    python scripts/debug_torch_graph.py [rounds] [eager_per_round]

The graph adds i+1 to a buffer for i < 200 (each add a separate kernel with its scalar in the
kernel arguments), so a replay must add exactly 20100 to every element.  Between replays the script
issues `eager_per_round` ordinary launches with varied argument sizes.
"""
import os
import sys

import torch


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    eager = int(sys.argv[2]) if len(sys.argv) > 2 else 5000
    print("env:", {k: v for k, v in os.environ.items() if k.startswith("DEBUG_CLR") or k.startswith("HIP_")},
          flush=True)
    dev = torch.device("cuda", 0)
    n_nodes = 200
    x = torch.zeros(4096, dtype=torch.float64, device=dev)
    y = torch.zeros(4096, dtype=torch.float32, device=dev)
    z = torch.zeros(64, 64, device=dev)
    stream = torch.cuda.Stream()
    with torch.cuda.stream(stream):
        for i in range(n_nodes):  # warm-up
            x.add_(float(i + 1))
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=stream):
        for i in range(n_nodes):
            x.add_(float(i + 1))
    torch.cuda.synchronize()
    expect = n_nodes * (n_nodes + 1) / 2
    bad = 0
    for r in range(rounds):
        x.zero_()
        torch.cuda.synchronize()
        with torch.cuda.stream(stream):
            g.replay()
        torch.cuda.synchronize()
        got = x.cpu()
        ok = bool((got == expect).all())
        if not ok:
            bad += 1
            u = torch.unique(got)
            print(f"round {r}: replay wrong: unique values {u[:8].tolist()} (expect {expect})", flush=True)
        for k in range(eager):  # ordinary launches with different argument blocks
            if k % 3 == 0:
                y.add_(1.0)
            elif k % 3 == 1:
                y.mul_(1.0)
            else:
                z.addmm_(z, z, beta=1.0, alpha=0.0)
        torch.cuda.synchronize()
    print(f"torch-graph: {bad} of {rounds} replays wrong ({eager} eager launches between replays)", flush=True)
    sys.exit(3 if bad else 0)


if __name__ == "__main__":
    main()
