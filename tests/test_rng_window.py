"""Engine words past k_tree's LDS window, and the agreement of its three chase copies (needs an
MI355X: `pytest -m gpu`).

A k_tree launch stages kRngWin = 256 words of the tree's mt19937 stream in LDS from the launch's
first word: the expansion takes 2K of them, the selection one per level with a tie list
(`gen() % size`, cnode.cpp:373-377) and the next expansion's 2K <= kNxt words go to the header.
Past the window the kernel reads the stream in HBM (mzmcts.hip `tree_chase`, the level walk, the
header writes).  In the classes with a precomputed chase (B <= the CU count) three waves chase
the same LDS state: wave 0 writes the selection outputs, wave 1 gathers the leaf's row and writes
the path record, wave 2 writes the header.  Round 5 found by reading that wave 1's copy read
words past the window from an unset stream offset; no test reached that branch.

Here `synthetic.make_deep_window_inputs` grows one deep path per tree with a tie at its bottom
(A = 2, K = 64: 128 words per expansion, paths past 130 levels), so that both the tie draws and the
header's words run past the window.  Each configuration asserts:
  * the kernel counted reads past the window of both kinds (MZ_S_RNG_TIE_BEYOND,
    MZ_S_RNG_NXT_BEYOND > 0), so the branches ran;
  * after every fused launch, the three copies agree: the header's leaf (wave 2, or wave 0 in the
    level walk) is the path record's last node (wave 1, or wave 0 with two workgroups per CU), whose
    parent's hidden_state_index_x and edge action are the selection outputs (wave 0), and the
    gathered row (wave 1 where it gathers) is the pool row of that parent;
  * every selection and every final readback bit-exact against the CPU port
    (tests/golden/trace_deep_window_* pin the port to the reference ctree at these shapes).
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import pytest

from conftest import assert_same

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

# (B, S, the fused kernel): one workgroup per CU (wave 1 gathers and writes the path record) and
# two rounds of workgroups (wave 0 does), in a precomputed-chase class and in the level walk
CASES = [
    (64, 190, "k_tree<384>"),
    (512, 190, "k_tree<384>"),
    (64, 300, "k_tree<1024>"),
    (512, 300, "k_tree<1024>"),
]
K, A, H = 64, 2, 24


@pytest.fixture(scope="module")
def gpu_lib():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    from mazero_amd._lib import load

    return load()


def debug_paths(tb, levels):
    B = tb.root_num
    hdr = np.zeros((B, 6), np.int32)
    path = np.zeros((B, levels, 4), np.int32)
    rc = tb._lib.mz_debug_paths(tb._h, hdr.ctypes.data_as(C.c_void_p), path.ctypes.data_as(C.c_void_p), levels)
    assert rc == 0, tb._lib.mz_last_error()
    return hdr, path


@pytest.mark.parametrize("B,S,kernel", CASES, ids=[f"B{b}_S{s}" for b, s, _ in CASES])
def test_beyond_window_chase_copies_agree(gpu_lib, port_lib, B, S, kernel):
    from mazero_amd.cytree import Tree_batch
    from mazero_amd.synthetic import DEFAULTS, make_deep_window_inputs, readbacks, run_search

    inp = make_deep_window_inputs(np.random.default_rng(600 + B + S), B, S, A)
    d = DEFAULTS
    c2, c1, g = d["pb_c_base"], d["pb_c_init"], d["discount"]
    mk = lambda L: Tree_batch(B, 1, A, K, S, d["delta_lb"], inp.seed, d["rho"], d["lam"], lib=L)  # noqa: E731
    expected = run_search(mk(port_lib), inp, K, per_sim=False)

    tb = mk(gpu_lib)
    assert tb.fused_kernel() == kernel
    dev = torch.device("cuda")
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    pool = torch.randn(S + 1, B, H, device=dev)
    leaf = torch.empty(B, H, device=dev)
    idx = torch.empty(S, B, dtype=torch.int32, device=dev)
    idy = torch.empty(S, B, dtype=torch.int32, device=dev)
    act = torch.empty(S, B, 1, dtype=torch.int32, device=dev)
    rows = torch.arange(B, device=dev)
    tb.prepare(t(inp.root_reward), t(inp.root_value), t(inp.root_policy), t(inp.root_beta), K, inp.noise_eps,
               t(inp.root_noise))
    tb.batch_selection_device(c2, c1, g, out=(idx[0], idy[0], act[0]))
    levels = S + 2
    deepest = 0
    for s in range(S):
        if s + 1 == S:
            tb.batch_expansion_and_backup(s + 1, g, K, t(inp.reward[s]), t(inp.value[s]), t(inp.policy[s]),
                                          t(inp.beta[s]))
            break
        tb.expansion_backup_selection_device(s + 1, g, K, t(inp.reward[s]), t(inp.value[s]), t(inp.policy[s]),
                                             t(inp.beta[s]), c2, c1, out=(idx[s + 1], idy[s + 1], act[s + 1]),
                                             pool=pool, gather_out=leaf)
        torch.cuda.synchronize()
        hdr, path = debug_paths(tb, levels)
        assert (hdr[:, 3] == 0).all(), f"launch {s + 1}: error bits {np.unique(hdr[:, 3])}"
        D = hdr[:, 2]
        deepest = max(deepest, int(D.max()))
        r = np.arange(B)
        last, parent = path[r, D], path[r, D - 1]
        where = f"launch {s + 1}"
        assert (last[:, 0] == hdr[:, 4]).all(), f"{where}: the path record's leaf differs from the header's"
        assert (parent[:, 2] == idx[s + 1].cpu().numpy()).all(), f"{where}: idx_x differs from the path record"
        assert (last[:, 3] == act[s + 1, :, 0].cpu().numpy()).all(), f"{where}: action differs from the path record"
        want = pool[idx[s + 1].long(), rows]
        assert torch.equal(leaf, want), f"{where}: the gathered row is not the selected parent's"
    torch.cuda.synchronize()
    st = tb.stats()
    assert deepest > 100, deepest
    assert st["rng_tie_beyond"] > 0 and st["rng_nxt_beyond"] > 0, (st["rng_tie_beyond"], st["rng_nxt_beyond"])
    out = dict(sel_idx=idx.cpu().numpy(), sel_act=act.cpu().numpy()[:, :, 0])
    out.update(readbacks(tb, g))
    assert_same(out, expected, f"gpu deep window B={B} S={S} ")
