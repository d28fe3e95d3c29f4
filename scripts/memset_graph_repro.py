"""Standalone repro (diagnostics, not product; no mazero_amd code): a hipMemsetAsync node in a torch
CUDA graph replayed after ordinary eager work, under the HIP runtime's default graph packet capture.

The graph holds one 4-byte hipMemsetAsync(word, 0) (called through ctypes on torch's capture
stream, as a library would) between two small torch kernels.  Between replays the process runs
ordinary eager work on the default stream: torch MLP forwards on fresh host batches, D2H reads and
4-byte hipMemsetAsync calls.  Every replay first sets the word to 0xffffffff and then checks that
the replay cleared it.

    python scripts/memset_graph_repro.py [eager iterations per round] [rounds]
"""
import ctypes as C
import os
import sys

import torch


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    print("DEBUG_CLR_GRAPH_PACKET_CAPTURE =", os.environ.get("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "(default)"), flush=True)
    hip = C.CDLL("libamdhip64.so.7")  # the runtime torch loaded (same soname)
    hip.hipMemsetAsync.argtypes = [C.c_void_p, C.c_int, C.c_size_t, C.c_void_p]
    dev = torch.device("cuda", 0)
    word = torch.empty(64, dtype=torch.int32, device=dev)
    scratch = torch.empty(1 << 16, dtype=torch.int32, device=dev)
    net = torch.nn.Sequential(torch.nn.Linear(384, 512), torch.nn.LayerNorm(512), torch.nn.ReLU(),
                              torch.nn.Linear(512, 384)).to(dev)
    x = torch.randn(256, 384, device=dev)
    y = torch.empty_like(x)

    def memset(t, value, n, stream):
        assert hip.hipMemsetAsync(C.c_void_p(t.data_ptr()), value, n, C.c_void_p(stream.cuda_stream)) == 0

    def body():
        y.copy_(x * 2)
        memset(word, 0, 4, torch.cuda.current_stream())
        y.add_(1)

    body()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body()
    torch.cuda.synchronize()
    bad = 0
    for r in range(rounds):
        word.fill_(-1)
        g.replay()
        torch.cuda.synchronize()
        w = int(word[0].item()) & 0xFFFFFFFF
        print(f"replay {r} (after {r * iters} eager iterations): word {w:#010x} (want 0)", flush=True)
        bad += w != 0
        with torch.no_grad():
            for i in range(iters):  # ordinary eager work on the default stream
                h = torch.from_numpy(torch.randn(256, 384).numpy()).to(dev)
                out = net(h)
                memset(scratch[64 * (i % 512):], 0, 4, torch.cuda.current_stream())
                _ = out[0, :4].cpu()
    print("DEFECT: a replayed memset node wrote stale data" if bad else "ok: every replay correct", flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
