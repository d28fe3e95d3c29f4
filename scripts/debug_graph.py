"""Debug: tree-only graph capture of prepare + search vs eager (same seed / inputs)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from mazero_amd.cytree import Tree_batch
from mazero_amd.synthetic import make_search_inputs

B, A, K, S = 64, 9, 1, 20
dev = torch.device("cuda", 0)
rng = np.random.default_rng(0)
inp = make_search_inputs(rng, B, A, S)
T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
rr, rv, rp, rb, rn = T(inp.root_reward), T(inp.root_value), T(inp.root_policy), T(inp.root_beta), T(inp.root_noise)
r, v, p, b = T(inp.reward), T(inp.value), T(inp.policy), T(inp.beta)
tb = Tree_batch(B, 1, A, K, S, 0.01, 7, 0.75, 0.8)
idx = torch.empty(B, dtype=torch.int32, device=dev); idy = torch.empty_like(idx); act = torch.empty(B, 1, dtype=torch.int32, device=dev)

def search():
    tb.prepare(rr, rv, rp, rb, K, inp.noise_eps, rn)
    tb.batch_selection_device(19652.0, 1.25, 0.997, out=(idx, idy, act))
    for s in range(S):
        if s + 1 < S:
            tb.expansion_backup_selection_device(s + 1, 0.997, K, r[s], v[s], p[s], b[s], 19652.0, 1.25, out=(idx, idy, act))
        else:
            tb.batch_expansion_and_backup(s + 1, 0.997, K, r[s], v[s], p[s], b[s])

def vals():
    tb.synchronize()
    return tb.get_roots_values().copy(), tb.get_roots_marginal_visit_count().copy()

search(); e1 = vals()
tb.reseed(9); search(); e9 = vals()
tb.reseed(7)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    search()
g.replay(); tb.state_changed(); g1 = vals()
print("replay seed7 == eager seed7:", np.array_equal(g1[0], e1[0]), np.array_equal(g1[1], e1[1]))
tb.reseed(9); g.replay(); tb.state_changed(); g9 = vals()
print("replay seed9 == eager seed9:", np.array_equal(g9[0], e9[0]), np.array_equal(g9[1], e9[1]))
print("seed7 != seed9:", not np.array_equal(e1[1], e9[1]))

ok = True
for rep in range(8):
    sd = 100 + rep
    tb.reseed(sd); search(); ev = vals()
    tb.reseed(sd); g.replay(); tb.state_changed(); gv = vals()
    same = np.array_equal(ev[0], gv[0]) and np.array_equal(ev[1], gv[1])
    ok &= same
    print("rep", rep, "replay == eager:", same, flush=True)
print("ALL OK" if ok else "MISMATCH")
