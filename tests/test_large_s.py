"""Large simulation counts: the pUCT coefficient table stays O(S) (needs an MI355X: `pytest -m gpu`).

The reference computes pb_c = (logf((n + c2 + 1) / c2) + c1) * sqrt(n) / (v + 1) per score
(cnode.cpp:313-316) and has no bound on simulation_num.  Until round 6 mz_create tabulated it for
every (n, v) with n < S + 2, an O(S^2) table on host and device (8.5 GB at S = 65,000) whose size
was computed in 32-bit ints (it wrapped past S = 32,767).  Now only the kernels that
read the full table get one (k_step's LDS-staged table, k_tree's prior scores: S + 2 <= 342);
every other kernel computes pb_c from the per-n pb / sqrt tables with the same double arithmetic,
and past 512 the table is T[0] alone (mazero_amd/csrc/mzmcts.hip `table_entries`).
"""
from __future__ import annotations

import numpy as np
import pytest

from conftest import assert_same

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def gpu_lib():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    from mazero_amd._lib import load

    return load()


def arena_info(tb):
    import ctypes as C

    out = (C.c_int64 * 5)()
    assert tb._lib.mz_arena_info(tb._h, out, 5) == 0
    return dict(zip(("arena", "tables", "values", "stream", "nodes"), list(out)))


def test_s33000_handle_takes_k_hbm_with_small_tables(gpu_lib):
    """at S >= 32,767 the table size wrapped negative and routed the handle to a
    kernel with a corrupt layout.  A K = 1 chain of 33,002 nodes is past every LDS class: k_hbm,
    with tables of O(S) bytes."""
    from mazero_amd.cytree import Tree_batch

    tb = Tree_batch(1, 1, 9, 1, 33000, 0.01, 3, 0.75, 0.8, lib=gpu_lib)
    assert tb.fused_kernel() == "k_hbm"
    info = arena_info(tb)
    assert info["tables"] < 1 << 20, info  # pb / sq for 33,002 visit counts + T[0]
    assert info["arena"] >= info["values"] + info["stream"] + info["nodes"] + info["tables"]
    del tb


def test_s20000_bit_exact_with_tables_under_64mb(gpu_lib, port_lib):
    """a search of 20,000 simulations (K = 2, A = 9, two roots: 40,003-node pools on
    k_hbm) bit-exact against the CPU port, every selection and readback, with < 64 MB of tables
    (the O(S^2) table alone was 1.6 GB here)."""
    from test_gpu_parity import run_fused, to_device

    from mazero_amd.cytree import Tree_batch
    from mazero_amd.synthetic import DEFAULTS, make_search_inputs, run_search

    B, A, K, S = 2, 9, 2, 20000
    inp = make_search_inputs(np.random.default_rng(20000), B, A, S)
    d = DEFAULTS
    mk = lambda L: Tree_batch(B, 1, A, K, S, d["delta_lb"], inp.seed, d["rho"], d["lam"], lib=L)  # noqa: E731
    expected = run_search(mk(port_lib), inp, K, per_sim=False)
    tb = mk(gpu_lib)
    assert tb.fused_kernel() == "k_hbm"
    info = arena_info(tb)
    assert info["tables"] < 64 << 20, info
    out, _ = run_fused(tb, to_device(inp), K, {}, fused_rb="packed")
    assert_same(out, expected, "gpu S=20000 ")
