"""Parity of the HIP product against the oracle (needs an MI355X: `pytest -m gpu`).

Bar (BASELINE.json north_star): selection indices / actions and visit counts
bit-exact; every float readback bit-exact too (the kernels replay the reference's f32/f64 op
order), which is stronger than the 1e-5 Q tolerance the north star allows.

* every committed golden trace (recorded from the compiled reference) through the host-memory
  path, the device-tensor path and the fused device loop
* BASELINE-size searches (256 roots x 50 sims, 1024 x 50, 512 x 100, 256 x 200) against the CPU
  port, plus size-independent properties
* sharded batches (root_offset) identical to the unsharded batch
* gather kernel, device readbacks, error reporting
"""
from __future__ import annotations

import os

import numpy as np
import pytest

from conftest import assert_same, full_fixtures, golden_traces, load_full, load_trace

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def gpu_lib():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    from mazero_amd._lib import load

    return load()


def make_tb(lib, inp, K, knobs, **kw):
    from mazero_amd.cytree import Tree_batch

    return Tree_batch(inp.B, 1, inp.A, K, inp.S, knobs.get("delta_lb", 0.01), inp.seed, knobs.get("rho", 0.75),
                      knobs.get("lam", 0.8), lib=lib, **kw)


def to_device(inp):
    from dataclasses import replace

    dev = torch.device("cuda")
    f = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    return replace(inp, root_reward=f(inp.root_reward), root_value=f(inp.root_value), root_policy=f(inp.root_policy),
                   root_beta=f(inp.root_beta), root_noise=f(inp.root_noise), reward=f(inp.reward),
                   value=f(inp.value), policy=f(inp.policy), beta=f(inp.beta))


def run_fused(tb, dinp, K, knobs, pool=None, fused_rb=None):
    """The device-resident loop: prepare, select(0), then per simulation one fused
    expand+backup+select(+gather) launch; selections are recorded on the device.  fused_rb: None,
    the last expansion alone (then the host getters); "packed", the last expansion fused with the
    packed readback (mz_expand_backup_readback, out = NULL) before the host getters; a dict of
    get_roots_device output tensors, fused with the readback into them."""
    from mazero_amd.synthetic import DEFAULTS, readbacks

    k = dict(DEFAULTS)
    k.update(knobs)
    c2, c1, g = k["pb_c_base"], k["pb_c_init"], k["discount"]
    B, S = dinp.B, dinp.S
    dev = torch.device("cuda")
    tb.prepare(dinp.root_reward, dinp.root_value, dinp.root_policy, dinp.root_beta, K, dinp.noise_eps,
               dinp.root_noise)
    idx = torch.empty(S, B, dtype=torch.int32, device=dev)
    idy = torch.empty(S, B, dtype=torch.int32, device=dev)
    act = torch.empty(S, B, 1, dtype=torch.int32, device=dev)
    gathered = None
    if pool is not None:
        gathered = torch.empty((S,) + tuple(pool.shape[1:]), dtype=pool.dtype, device=dev)
    tb.batch_selection_device(c2, c1, g, out=(idx[0], idy[0], act[0]))
    if pool is not None:
        tb._lib.mz_gather_rows(tb._h, pool.data_ptr(), pool.stride(0) * pool.element_size(),
                               pool[0, 0].numel() * pool.element_size(), idx[0].data_ptr(), gathered[0].data_ptr())
    for s in range(S):
        if s + 1 < S:
            tb.expansion_backup_selection_device(s + 1, g, K, dinp.reward[s], dinp.value[s], dinp.policy[s],
                                                 dinp.beta[s], c2, c1, out=(idx[s + 1], idy[s + 1], act[s + 1]),
                                                 pool=pool, gather_out=None if pool is None else gathered[s + 1])
        elif fused_rb is not None:
            tb.expansion_backup_readback_device(s + 1, g, K, dinp.reward[s], dinp.value[s], dinp.policy[s],
                                                dinp.beta[s], readback_discount=g,
                                                out=None if fused_rb == "packed" else fused_rb)
        else:
            tb.batch_expansion_and_backup(s + 1, g, K, dinp.reward[s], dinp.value[s], dinp.policy[s], dinp.beta[s])
    torch.cuda.synchronize()
    out = dict(sel_idx=idx.cpu().numpy(), sel_act=act.cpu().numpy()[:, :, 0])
    assert (idy.cpu().numpy() == np.arange(B, dtype=np.int32)[None]).all()
    out.update(readbacks(tb, g))
    return out, gathered


TRACES = golden_traces()
IDS = [os.path.basename(p)[6:-4] for p in TRACES]


@pytest.mark.parametrize("path", TRACES, ids=IDS)
def test_golden_host_path(gpu_lib, path):
    from mazero_amd.synthetic import run_search

    inp, knobs, K, expected = load_trace(path)
    tb = make_tb(gpu_lib, inp, K, knobs)
    assert_same(run_search(tb, inp, K, knobs), expected, "gpu(host) ")


@pytest.mark.parametrize("copy", [False, True], ids=["zero_copy", "dma_copy"])
@pytest.mark.parametrize("path", TRACES, ids=IDS)
def test_golden_host_path_fused(gpu_lib, path, copy, monkeypatch):
    """The host-memory path as the reference driver calls it (batch_selection, then
    batch_expansion_and_backup, no readback in between): each staged expansion is launched fused
    with the next selection.  Zero-copy (default): the kernel reads the pinned stage and writes the
    selection into it; MZ_HOST_COPY=1: one host->device and one device->host copy per simulation."""
    from mazero_amd.synthetic import run_search

    inp, knobs, K, expected = load_trace(path)
    if copy:
        monkeypatch.setenv("MZ_HOST_COPY", "1")
    tb = make_tb(gpu_lib, inp, K, knobs)
    monkeypatch.delenv("MZ_HOST_COPY", raising=False)
    expected = {k: v for k, v in expected.items() if k not in ("root_values_per_sim", "marginal_per_sim")}
    assert_same(run_search(tb, inp, K, knobs, per_sim=False), expected, "gpu(host, fused) ")


@pytest.mark.parametrize("path", TRACES, ids=IDS)
def test_golden_device_tensors(gpu_lib, path):
    from mazero_amd.synthetic import run_search

    inp, knobs, K, expected = load_trace(path)
    tb = make_tb(gpu_lib, inp, K, knobs)
    assert_same(run_search(tb, to_device(inp), K, knobs), expected, "gpu(device) ")


@pytest.mark.parametrize("path", TRACES, ids=IDS)
def test_golden_fused_loop(gpu_lib, path):
    inp, knobs, K, expected = load_trace(path)
    tb = make_tb(gpu_lib, inp, K, knobs)
    out, _ = run_fused(tb, to_device(inp), K, knobs)
    expected = {k: v for k, v in expected.items() if k not in ("root_values_per_sim", "marginal_per_sim")}
    assert_same(out, expected, "gpu(fused) ")


FULL = full_fixtures()


@pytest.mark.parametrize("path", FULL, ids=[os.path.basename(p)[5:-4] for p in FULL])
def test_baseline_sizes_vs_reference(gpu_lib, path):
    """The fused device loop against the reference ctree's own outputs at every BASELINE size
    (oracle/gen_golden.py --full: 3m 256 x 50 K in {1, 5, 10}, 2s3z 1024 x 50 K in {1, 5}, 3s5z
    512 x 100 K in {5, 10}, 27m 256 x 200 K in {1, 5}, a tie variant and a 30 %-masked variant):
    selections of every simulation and all final readbacks, bit for bit.  The inputs are
    regenerated on the box and checked against the recorded SHA-256 first."""
    inp, K, expected = load_full(path)
    out, _ = run_fused(make_tb(gpu_lib, inp, K, {}), to_device(inp), K, {})
    assert_same(out, expected, f"gpu {os.path.basename(path)} ")


HBM_FULL = [p for p in FULL if os.path.basename(p) in (
    "full_3m_k1.npz", "full_3m_k5.npz", "full_3m_k5_ties.npz", "full_3s5z_k10.npz", "full_27m_k5.npz",
    "full_3s5z_k5_legal30.npz")]


@pytest.mark.parametrize("path", HBM_FULL, ids=[os.path.basename(p)[5:-4] for p in HBM_FULL])
def test_hbm_kernel_vs_reference(gpu_lib, path, monkeypatch):
    """The HBM-resident kernel (k_hbm, forced with MZ_HBM=1 at mz_create) on BASELINE-size fixtures
    recorded from the reference ctree: every selection and readback bit for bit, through the fused
    loop and the fused readback."""
    inp, K, expected = load_full(path)
    monkeypatch.setenv("MZ_HBM", "1")
    tb = make_tb(gpu_lib, inp, K, {})
    monkeypatch.delenv("MZ_HBM")
    assert tb.fused_kernel() == "k_hbm"
    out, _ = run_fused(tb, to_device(inp), K, {}, fused_rb="packed")
    assert_same(out, expected, f"gpu k_hbm {os.path.basename(path)} ")


@pytest.mark.parametrize("path", TRACES, ids=IDS)
def test_hbm_kernel_golden_traces(gpu_lib, path, monkeypatch):
    """k_hbm (MZ_HBM=1) on every golden trace: the host path (per-call selection, its
    per-simulation readbacks) and the fused device loop."""
    from mazero_amd.synthetic import run_search

    inp, knobs, K, expected = load_trace(path)
    monkeypatch.setenv("MZ_HBM", "1")
    tb, tb2 = make_tb(gpu_lib, inp, K, knobs), make_tb(gpu_lib, inp, K, knobs)
    monkeypatch.delenv("MZ_HBM")
    assert tb.fused_kernel() == "k_hbm"
    assert_same(run_search(tb, inp, K, knobs), expected, "gpu k_hbm (host) ")
    out, _ = run_fused(tb2, to_device(inp), K, knobs)
    expected = {k: v for k, v in expected.items() if k not in ("root_values_per_sim", "marginal_per_sim")}
    assert_same(out, expected, "gpu k_hbm (fused) ")


BIG = [
    ("3m_k1", 256, 9, 1, 50, 0.0),
    ("3m_k5", 256, 9, 5, 50, 0.3),
    ("3m_k10", 256, 9, 10, 50, 0.0),
    ("2s3z_k5", 1024, 11, 5, 50, 0.0),
    ("3s5z_k5", 512, 15, 5, 100, 0.3),
    ("27m_k1", 256, 36, 1, 200, 0.0),
    ("27m_k5", 256, 36, 5, 200, 0.0),
    ("27m_k8_general_layout", 64, 36, 8, 200, 0.0),  # 1616-node pool: LDS layout from Geo (class 0)
    # K = 2 trees grow deep paths: k_tree's back-propagation waves handle more than their two
    # pre-staged levels (later levels staged after the first barrier)
    ("deep_k2", 64, 9, 2, 200, 0.0),
    # value sets longer than a k_tree staging slot (E = 401 > kBkCap): the handle falls back to k_step
    ("k2_long_value_sets", 32, 9, 2, 400, 0.0),
    # deep K = 2 paths inside the 256-node class (seven back-propagation waves): levels past a
    # wave's two pre-staged ones (i + 14, ...) are staged after the first barrier
    ("deep_k2_tree", 64, 9, 2, 120, 0.0),
    # the 512-node class keeps 128-entry staging slots (two workgroups per CU): E = 151 takes k_step,
    # E = 101 k_tree
    ("k3_512_class_kstep", 64, 9, 3, 150, 0.0),
    ("k4_512_class_tree", 64, 9, 4, 100, 0.0),
    # K = 1 pools above k_chain3's 256 nodes: k_chain<512> (S + 2 <= 512), k_chain<1024>, and the
    # run-time layout k_chain<0> (S >= 1023)
    ("k1_chain512", 64, 9, 1, 300, 0.3),
    ("k1_chain1024", 32, 11, 1, 700, 0.0),
    ("k1_chain_general", 16, 9, 1, 1100, 0.0),
    # pools past 1,024 nodes whose LDS image fits only without the staged pUCT table and with
    # 512-entry value chunks (mz_create's second layout): K = 10 at S = 200
    ("k10_s200_general", 16, 9, 10, 200, 0.3),
    ("27m_k10_s200", 8, 36, 10, 200, 0.0),
    # pools whose LDS image exceeds one CU's 160 KB: the HBM-resident kernel (refused before round 5;
    # the reference allocates K * (S + 2) nodes for any K and S, cnode.cpp:553-577)
    ("hbm_a64_k70_s60", 32, 64, 70, 60, 0.3),      # 3,905 reachable nodes
    ("hbm_27m_k16_s200", 64, 36, 16, 200, 0.0),    # 3,217
    ("hbm_k1_s2300", 2, 9, 1, 2300, 0.0),          # a K = 1 chain of 2,302 nodes (path records past 64 levels)
    # action spaces past one lane per action (round 5: expand_wide + k_hbm; the reference has no bound)
    ("wide_a100_k10", 64, 100, 10, 50, 0.3),
    ("wide_a255_k300", 8, 255, 300, 20, 0.0),      # roots with > 64 children: chunked walk and readback
]


# the fused kernel each row exists for (mz_fused_kernel)
BIG_KERNEL = {"3m_k1": "k_chain3<64>", "27m_k1": "k_chain3<256>", "k1_chain512": "k_chain<512>",
              "k1_chain1024": "k_chain<1024>", "k1_chain_general": "k_chain<0>",
              "27m_k8_general_layout": "k_step<0>", "k2_long_value_sets": "k_step<1024>",
              "k10_s200_general": "k_step<0>", "27m_k10_s200": "k_step<0>", "hbm_a64_k70_s60": "k_hbm",
              "hbm_27m_k16_s200": "k_hbm", "hbm_k1_s2300": "k_hbm", "wide_a100_k10": "k_hbm",
              "wide_a255_k300": "k_hbm"}


@pytest.mark.parametrize("name,B,A,K,S,lz", BIG, ids=[b[0] for b in BIG])
def test_baseline_sizes_vs_port(gpu_lib, port_lib, name, B, A, K, S, lz):
    from mazero_amd.synthetic import make_search_inputs, run_search

    rng = np.random.default_rng(sum(map(ord, name)) * 7919 + B)
    inp = make_search_inputs(rng, B, A, S, legal_zero_frac=lz)
    knobs = {}
    exp = run_search(make_tb(port_lib, inp, K, knobs), inp, K, knobs)
    tb = make_tb(gpu_lib, inp, K, knobs)
    if name in BIG_KERNEL:
        assert tb.fused_kernel() == BIG_KERNEL[name]
    out, _ = run_fused(tb, to_device(inp), K, knobs)
    exp = {k: v for k, v in exp.items() if k not in ("root_values_per_sim", "marginal_per_sim")}
    assert_same(out, exp, f"gpu {name} ")
    # size-independent properties (hold for the reference by construction)
    vc = out["sampled_visit_count"].sum(axis=1)
    assert (vc == S).all()  # every simulation passes through exactly one root child
    assert (out["marginal_visit_count"].sum(axis=(1, 2)) == S).all()
    deg = out["degree"]
    assert (deg >= 1).all() and (deg <= min(K, A)).all()
    if name == "wide_a255_k300":
        assert deg.max() > 64  # (the chunked paths ran)
    bh = out["sampled_beta_hat"].sum(axis=1)
    assert np.allclose(bh, 1.0, atol=1e-5)  # beta_hat = counts / K over the K root draws


def test_trim_caches_releases_destroyed_arenas(gpu_lib):
    """A destroyed handle's device arena goes to the library's process-wide cache (reused by the next
    handle of a fitting size); mz_trim_caches (mazero_amd._lib.trim_caches, called by
    mcts_sampled.release) frees what the cache holds."""
    import gc

    from mazero_amd._lib import trim_caches
    from mazero_amd.synthetic import make_search_inputs

    trim_caches()
    inp = make_search_inputs(np.random.default_rng(7), 64, 9, 20)
    tb = make_tb(gpu_lib, inp, 5, {})
    torch.cuda.synchronize()
    del tb
    gc.collect()
    assert trim_caches() > 0
    assert trim_caches() == 0


@pytest.mark.parametrize(
    "K,S,ties",
    [(5, 200, True), (5, 200, False), (3, 250, True), (7, 120, True), (7, 120, False), (8, 120, True)],
    ids=["k5_s200_ties", "k5_s200", "k3_s250_ties", "k7_s120_ties", "k7_s120", "k8_s120_ties"],
)
def test_level_walk_two_levels_per_pass(gpu_lib, port_lib, K, S, ties):
    """The level walk's two-level passes (round 6, k_tree's 1,024-node classes, K <= 7): lanes 0..7
    score a node's children and lanes 8 + 8g + i child g's children, one segmented max and two
    ballots resolve both levels.  Uniform policies (`ties`) put a tie list at every level, so both
    levels read engine words in the pass; K = 8 takes the one-level walk.  Against the port."""
    from mazero_amd.synthetic import make_search_inputs, run_search

    B, A = 32, 36
    rng = np.random.default_rng(8080 + 31 * K + S + ties)
    inp = make_search_inputs(rng, B, A, S, ties=ties)
    knobs = {}
    exp = run_search(make_tb(port_lib, inp, K, knobs), inp, K, knobs)
    tb = make_tb(gpu_lib, inp, K, knobs)
    assert tb.fused_kernel().startswith("k_tree<1024"), tb.fused_kernel()
    out, _ = run_fused(tb, to_device(inp), K, knobs)
    exp = {k: v for k, v in exp.items() if k not in ("root_values_per_sim", "marginal_per_sim")}
    assert_same(out, exp, f"gpu level walk K={K} S={S} ties={ties} ")
    assert (out["sampled_visit_count"].sum(axis=1) == S).all()


@pytest.mark.parametrize("K,S", [(3, 700), (2, 40)], ids=["k3_s700", "k2_s40"])
def test_hbm_wave_per_node_backup(gpu_lib, port_lib, K, S, monkeypatch):
    """k_hbm's back-propagation (hbm_node_wave, round 5): one wave per path node, dealt over three
    waves.  S = 700 puts more than 512 entries in the root's value set (the batched two-pass count
    and tail move instead of the registers); S = 40 keeps every node in registers.  Forced with
    MZ_HBM=1, against the port."""
    from mazero_amd.synthetic import make_search_inputs, run_search

    B, A = 8, 9
    rng = np.random.default_rng(4242 + S)
    inp = make_search_inputs(rng, B, A, S)
    knobs = {}
    exp = run_search(make_tb(port_lib, inp, K, knobs), inp, K, knobs)
    monkeypatch.setenv("MZ_HBM", "1")
    tb = make_tb(gpu_lib, inp, K, knobs)
    monkeypatch.delenv("MZ_HBM")
    assert tb.fused_kernel() == "k_hbm"
    out, _ = run_fused(tb, to_device(inp), K, knobs)
    exp = {k: v for k, v in exp.items() if k not in ("root_values_per_sim", "marginal_per_sim")}
    assert_same(out, exp, f"gpu k_hbm K={K} S={S} ")
    assert (out["sampled_visit_count"].sum(axis=1) == S).all()


@pytest.mark.parametrize("seeding", ["table", "chain", "beyond_table"])
@pytest.mark.parametrize("K", [1, 5])
def test_seeding_paths_vs_port(gpu_lib, port_lib, seeding, K, monkeypatch):
    """k_prepare seeds each tree's mt19937 (cnode.cpp:574) from the per-device checkpoint table
    (seed values below its size), by the sequential chain with MZ_NO_SEED_TABLE=1 (read at
    mz_create), and by the chain for a seed value beyond the table (random_seed 100000: v =
    233,300,000 + i).  Every selection and readback against the CPU port; 2 x 624 + 102 words of
    engine stream are consumed at S = 50, so the twist's block boundaries are crossed too."""
    from dataclasses import replace

    from mazero_amd.synthetic import make_search_inputs, run_search

    rng = np.random.default_rng(4242 + K)
    inp = make_search_inputs(rng, 128, 9, 50, legal_zero_frac=0.2)
    if seeding == "beyond_table":
        inp = replace(inp, seed=100000)
    exp = run_search(make_tb(port_lib, inp, K, {}), inp, K, {})
    if seeding == "chain":
        monkeypatch.setenv("MZ_NO_SEED_TABLE", "1")
    tb = make_tb(gpu_lib, inp, K, {})
    monkeypatch.delenv("MZ_NO_SEED_TABLE", raising=False)
    out, _ = run_fused(tb, to_device(inp), K, {})
    exp = {k: v for k, v in exp.items() if k not in ("root_values_per_sim", "marginal_per_sim")}
    assert_same(out, exp, f"gpu seeding={seeding} K={K} ")


FUSED_RB = [
    # (name, B, A, K, S, env): which kernel ends the search -- k_chain3 / k_tree write the readback
    # themselves, the others are followed by k_readback; S = 1: the last leaf is a root child
    ("chain3", 64, 9, 1, 30, None), ("chain3_s1", 64, 9, 1, 1, None), ("tree", 64, 9, 5, 30, None),
    ("tree_s1", 64, 9, 5, 1, None), ("tree_k10", 32, 15, 10, 40, None), ("chain_v2", 64, 9, 1, 30, "MZ_CHAIN_V2"),
    ("kstep_k70", 16, 64, 70, 12, None), ("chain512", 16, 9, 1, 300, None),
    ("unfused_env", 64, 9, 5, 30, "MZ_NO_FUSED_READBACK"), ("hbm", 16, 64, 70, 12, "MZ_HBM"),
]


@pytest.mark.parametrize("name,B,A,K,S,env", FUSED_RB, ids=[f[0] for f in FUSED_RB])
def test_fused_readback(gpu_lib, port_lib, name, B, A, K, S, env, monkeypatch):
    """mz_expand_backup_readback: the search's last expansion with every root output, into the
    packed buffer (then the host getters, against the CPU port) and into caller tensors (against
    mz_get_roots_device on the same final state), for every kernel that can end a search."""
    from mazero_amd.synthetic import make_search_inputs, run_search

    rng = np.random.default_rng(sum(map(ord, name)) + 31 * S)
    inp = make_search_inputs(rng, B, A, S, legal_zero_frac=0.2)
    exp = run_search(make_tb(port_lib, inp, K, {}), inp, K, {})
    exp = {k: v for k, v in exp.items() if k not in ("root_values_per_sim", "marginal_per_sim")}
    if env:
        monkeypatch.setenv(env, "1")
    tb = make_tb(gpu_lib, inp, K, {})
    tb2 = make_tb(gpu_lib, inp, K, {})
    if env:
        monkeypatch.delenv(env)
    out, _ = run_fused(tb, to_device(inp), K, {}, fused_rb="packed")
    assert_same(out, exp, f"gpu fused packed readback {name} ")
    # into caller tensors: every field, against a separate readback of the same final state
    dev = torch.device("cuda")
    NA = A
    W = min(K, A)
    from mazero_amd._capi import FIELDS, INT_FIELDS

    def outs():
        return dict(values=torch.full((B,), -7.0, device=dev),
                    marginal_visit_count=torch.full((B, 1, NA), -7, dtype=torch.int32, device=dev),
                    marginal_priors=torch.full((B, 1, NA), -7.0, device=dev),
                    degrees=torch.full((B,), -7, dtype=torch.int32, device=dev),
                    sampled={f: torch.full((B, W), -7, dtype=torch.int32 if f in INT_FIELDS else torch.float32,
                                           device=dev) for f in FIELDS})
    got = outs()
    run_fused(tb2, to_device(inp), K, {}, fused_rb=got)
    ref = outs()
    from mazero_amd.synthetic import DEFAULTS

    tb2.get_roots_device(DEFAULTS["discount"], **ref)
    torch.cuda.synchronize()
    for k in ("values", "marginal_visit_count", "marginal_priors", "degrees"):
        assert torch.equal(got[k].view(torch.int32) if got[k].is_floating_point() else got[k],
                           ref[k].view(torch.int32) if ref[k].is_floating_point() else ref[k]), (name, k)
    for f in FIELDS:
        a, b = got["sampled"][f], ref["sampled"][f]
        assert torch.equal(a.view(torch.int32) if a.is_floating_point() else a,
                           b.view(torch.int32) if b.is_floating_point() else b), (name, f)


def test_chain_v2_on_reference_fixture(gpu_lib, monkeypatch):
    """MZ_CHAIN_V2=1 (read at mz_create) sends K = 1 pools of <= 256 nodes to the round-2 k_chain
    instead of k_chain3: the 3m K = 1 BASELINE fixture through it, against the reference."""
    path = [p for p in FULL if os.path.basename(p) == "full_3m_k1.npz"][0]
    inp, K, expected = load_full(path)
    monkeypatch.setenv("MZ_CHAIN_V2", "1")
    tb = make_tb(gpu_lib, inp, K, {})
    monkeypatch.delenv("MZ_CHAIN_V2")
    assert tb.fused_kernel() == "k_chain<64>"
    assert make_tb(gpu_lib, inp, K, {}).fused_kernel() == "k_chain3<64>"
    out, _ = run_fused(tb, to_device(inp), K, {})
    assert_same(out, expected, "gpu k_chain (MZ_CHAIN_V2) ")


@pytest.mark.parametrize("B,A,K,S", [(256, 9, 5, 50), (128, 15, 10, 100), (64, 3, 10, 60)])
def test_ties_vs_port(gpu_lib, port_lib, B, A, K, S):
    """Uniform policies and zero rewards/values: children with equal priors tie in select_child
    (cnode.cpp:355-370), so the walk breaks ties with engine words (gen() % list size) on many
    levels -- the exact record path of select_walk, at full batch sizes."""
    from mazero_amd.synthetic import make_search_inputs, run_search

    inp = make_search_inputs(np.random.default_rng(B * 1000 + K), B, A, S, ties=True)
    exp = run_search(make_tb(port_lib, inp, K, {}), inp, K, {})
    out, _ = run_fused(make_tb(gpu_lib, inp, K, {}), to_device(inp), K, {})
    exp = {k: v for k, v in exp.items() if k not in ("root_values_per_sim", "marginal_per_sim")}
    assert_same(out, exp, f"gpu ties B={B} A={A} K={K} ")


@pytest.mark.parametrize("K,H", [
    (5, 384),    # 1.5 KiB rows (3m): register chunks
    (1, 384),    # K = 1: the row prefetched in round 1
    (1, 3456),   # 13.5 KiB rows (27m): LDS-DMA staging, prefetched in round 1
    (5, 3456),   # 13.5 KiB rows, staged after the selection
    (1, 1025),   # 4100-byte rows: not 16-byte aligned (dword loop)
    (5, 5000),   # 20,000-byte rows: above the staging area (plain loop)
])
def test_gather_pool(gpu_lib, K, H):
    """Fused leaf hidden-state gather == pool[idx_x[i], i] (mcts_sampled.py:130-134), over the
    kernel's row-size classes."""
    from mazero_amd.synthetic import make_search_inputs

    B, A, S = 64, 9, 20
    inp = make_search_inputs(np.random.default_rng(3), B, A, S)
    pool = torch.randn(S + 1, B, H, device="cuda")
    out, gathered = run_fused(make_tb(gpu_lib, inp, K, {}), to_device(inp), K, {}, pool=pool)
    idx = torch.from_numpy(out["sel_idx"]).long().cuda()
    ref = pool[idx, torch.arange(B, device="cuda")[None, :]]
    assert torch.equal(gathered, ref)
    # fp16 pools (autocast) gather the same bytes
    pool16 = pool.half()
    g16 = torch.empty(B, H, dtype=torch.float16, device="cuda")
    tb = make_tb(gpu_lib, inp, K, {})
    rc = gpu_lib.mz_gather_rows(tb._h, pool16.data_ptr(), pool16.stride(0) * 2, H * 2,
                                idx[3].int().contiguous().data_ptr(), g16.data_ptr())
    torch.cuda.synchronize()
    if (H * 2) % 4:  # the standalone gather copies whole dwords: other row sizes are refused
        assert rc != 0 and b"multiple of 4" in gpu_lib.mz_last_error()
        return
    assert rc == 0
    assert torch.equal(g16, pool16[idx[3], torch.arange(B, device="cuda")])


def test_sharded_equals_unsharded(gpu_lib):
    """Roots split over two handles with root_offset (one per rank in a multi-GPU job) give the
    bit-identical trees of one unsharded batch (seed_i = random_seed*2333 + global index)."""
    from dataclasses import replace

    from mazero_amd.synthetic import make_search_inputs, run_search

    B, A, K, S = 96, 9, 5, 30
    inp = make_search_inputs(np.random.default_rng(11), B, A, S)
    full = run_search(make_tb(gpu_lib, inp, K, {}), inp, K)
    h = B // 3
    parts = []
    for lo, hi in ((0, h), (h, B)):
        sub = replace(inp, B=hi - lo, root_reward=inp.root_reward[lo:hi], root_value=inp.root_value[lo:hi],
                      root_policy=inp.root_policy[lo:hi], root_beta=inp.root_beta[lo:hi],
                      root_noise=inp.root_noise[lo:hi], reward=inp.reward[:, lo:hi], value=inp.value[:, lo:hi],
                      policy=inp.policy[:, lo:hi], beta=inp.beta[:, lo:hi])
        parts.append(run_search(make_tb(gpu_lib, sub, K, {}, root_offset=lo), sub, K))
    for k in ("sel_idx", "sel_act", "root_values_per_sim"):
        assert np.array_equal(np.concatenate([parts[0][k], parts[1][k]], axis=1), full[k]), k
    for k in ("root_values", "marginal_visit_count", "sampled_visit_count", "sampled_qvalues"):
        a, b = parts[0][k], parts[1][k]
        w = max(a.shape[1], b.shape[1]) if a.ndim > 1 else None
        if w is not None and a.ndim == 2:
            a = np.pad(a, ((0, 0), (0, full[k].shape[1] - a.shape[1])))
            b = np.pad(b, ((0, 0), (0, full[k].shape[1] - b.shape[1])))
        assert np.array_equal(np.concatenate([a, b], axis=0), full[k]), k


def test_device_readbacks(gpu_lib):
    from mazero_amd._capi import MZ_MEM_DEVICE
    from mazero_amd.synthetic import make_search_inputs, run_search

    B, A, K, S = 32, 9, 5, 20
    inp = make_search_inputs(np.random.default_rng(5), B, A, S)
    tb = make_tb(gpu_lib, inp, K, {})
    ref = run_search(tb, inp, K)
    v = torch.empty(B, device="cuda")
    mv = torch.empty(B, 1, A, dtype=torch.int32, device="cuda")
    assert gpu_lib.mz_get_roots_values(tb._h, v.data_ptr(), MZ_MEM_DEVICE) == 0
    assert gpu_lib.mz_get_roots_marginal_visit_count(tb._h, mv.data_ptr(), MZ_MEM_DEVICE) == 0
    torch.cuda.synchronize()
    assert np.array_equal(v.cpu().numpy(), ref["root_values"])
    assert np.array_equal(mv.cpu().numpy(), ref["marginal_visit_count"])


def test_rebind_after_bound_stream_destroyed(gpu_lib, port_lib):
    """mz_set_stream never queries the stream it leaves (the caller may have destroyed it): half a
    search runs on a raw HIP stream, the stream is destroyed with that work possibly in flight, the
    handle is rebound to torch's stream and the search finishes -- bit-exact against the port."""
    import ctypes as C

    from mazero_amd.synthetic import DEFAULTS, make_search_inputs, readbacks, run_search

    B, A, K, S = 64, 9, 5, 30
    inp = make_search_inputs(np.random.default_rng(77), B, A, S)
    exp = run_search(make_tb(port_lib, inp, K, {}), inp, K, {}, per_sim=False)
    hip = C.CDLL("libamdhip64.so.7")
    raw = C.c_void_p()
    assert hip.hipStreamCreate(C.byref(raw)) == 0
    d = DEFAULTS
    c2, c1, g = d["pb_c_base"], d["pb_c_init"], d["discount"]
    dinp = to_device(inp)
    torch.cuda.synchronize()
    tb = make_tb(gpu_lib, inp, K, {})
    idx = torch.empty(S, B, dtype=torch.int32, device="cuda")  # (nothing is allocated on the raw stream)
    idy = torch.empty(B, dtype=torch.int32, device="cuda")
    act = torch.empty(B, 1, dtype=torch.int32, device="cuda")
    with torch.cuda.stream(torch.cuda.ExternalStream(raw.value)):
        tb.prepare(dinp.root_reward, dinp.root_value, dinp.root_policy, dinp.root_beta, K, dinp.noise_eps,
                   dinp.root_noise)
        for s in range(S // 2):
            tb.batch_selection_device(c2, c1, g, out=(idx[s], idy, act))
            tb.batch_expansion_and_backup(s + 1, g, K, dinp.reward[s], dinp.value[s], dinp.policy[s], dinp.beta[s])
    assert hip.hipStreamDestroy(raw) == 0
    for s in range(S // 2, S):  # torch's current stream: the handle rebinds (mz_set_stream)
        tb.batch_selection_device(c2, c1, g, out=(idx[s], idy, act))
        tb.batch_expansion_and_backup(s + 1, g, K, dinp.reward[s], dinp.value[s], dinp.policy[s], dinp.beta[s])
    torch.cuda.synchronize()
    out = dict(sel_idx=idx.cpu().numpy())
    out.update(readbacks(tb, g))
    exp.pop("sel_act")
    assert_same(out, exp, "gpu rebind ")


def test_rebind_with_staged_expansion_after_stream_destroyed(gpu_lib, port_lib):
    """A host-memory batch_expansion_and_backup is only staged (launched by the handle's next
    call).  Staged while the handle is bound to a raw HIP stream that is then destroyed, it must be
    launched on the stream the handle is rebound to, never on the destroyed one: the
    search finishes on torch's stream, bit-exact against the port."""
    import ctypes as C

    from mazero_amd.synthetic import DEFAULTS, make_search_inputs, readbacks, run_search

    B, A, K, S = 32, 9, 5, 16
    inp = make_search_inputs(np.random.default_rng(78), B, A, S)
    exp = run_search(make_tb(port_lib, inp, K, {}), inp, K, {}, per_sim=False)
    hip = C.CDLL("libamdhip64.so.7")
    raw = C.c_void_p()
    assert hip.hipStreamCreate(C.byref(raw)) == 0
    c2, c1, g = DEFAULTS["pb_c_base"], DEFAULTS["pb_c_init"], DEFAULTS["discount"]
    torch.cuda.synchronize()
    tb = make_tb(gpu_lib, inp, K, {})
    sels = []
    with torch.cuda.stream(torch.cuda.ExternalStream(raw.value)):
        tb.prepare(inp.root_reward, inp.root_value, inp.root_policy, inp.root_beta, K, inp.noise_eps, inp.root_noise)
        for s in range(S // 2):
            sels.append(tb.batch_selection(c2, c1, g)[0])
            tb.batch_expansion_and_backup(s + 1, g, K, inp.reward[s], inp.value[s], inp.policy[s], inp.beta[s])
    assert hip.hipStreamDestroy(raw) == 0  # the last expansion is still staged
    for s in range(S // 2, S):
        sels.append(tb.batch_selection(c2, c1, g)[0])
        tb.batch_expansion_and_backup(s + 1, g, K, inp.reward[s], inp.value[s], inp.policy[s], inp.beta[s])
    out = dict(sel_idx=np.asarray(sels, np.int32))
    out.update(readbacks(tb, g))
    exp.pop("sel_act")
    assert_same(out, exp, "gpu rebind (staged) ")


def test_wide_action_space_limits(gpu_lib):
    """Past 64 actions the tree takes up to 255 (Bn packs the action in 8 bits); the device driver
    glue, one lane per action, refuses them with an error instead of computing garbage."""
    import ctypes as C

    from mazero_amd._capi import MZError
    from mazero_amd.cytree import Tree_batch

    with pytest.raises(MZError, match="255"):
        Tree_batch(4, 1, 256, 5, 10, 0.01, 1, 0.75, 0.8, lib=gpu_lib)
    with pytest.raises(MZError, match="joint"):
        Tree_batch(4, 2, 65, 5, 10, 0.01, 1, 0.75, 0.8, lib=gpu_lib)
    tb = Tree_batch(4, 1, 100, 5, 10, 0.01, 1, 0.75, 0.8, lib=gpu_lib)
    assert tb.fused_kernel() == "k_hbm"
    logits = torch.zeros(4, 1, 100, device="cuda")
    probs = torch.empty(4, 100, device="cuda")
    tb._sync_stream()
    rc = gpu_lib.mz_policy_glue(tb._h, C.c_void_p(logits.data_ptr()), 0, 100, 0, 1.0, C.c_void_p(probs.data_ptr()),
                                C.c_void_p(probs.data_ptr()))
    assert rc != 0 and b"action_space_size > 64" in gpu_lib.mz_last_error()


def test_too_many_simulations_raise(gpu_lib):
    """The reference's pools are sized for simulation_num; overrunning them is reported as a
    RuntimeError at the call that overflows (host path is synchronous like the reference)."""
    from mazero_amd.cytree import Tree_batch

    B, A, K, S = 4, 3, 1, 2
    tb = Tree_batch(B, 1, A, K, S, 0.01, 5, 0.75, 0.8, lib=gpu_lib)
    p = np.full((B, 1, A), 1.0 / A, np.float32)
    z = np.zeros(B, np.float32)
    tb.prepare(z, z, p, p, K, 0.0, p)
    with pytest.raises(RuntimeError):
        for s in range(10):
            tb.batch_selection(19652.0, 1.25, 0.997)
            tb.batch_expansion_and_backup(s + 1, 0.997, K, z, z, p, p)


def test_graph_of_one_step_replayed(gpu_lib, port_lib):
    """A HIP graph holding ONE fused simulation step, replayed for every simulation.  The host's
    staging bounds baked into the graph are stale from the second replay on, so the kernel must
    detect it from the tree header and stage the rest (slow path) -- results stay bit-exact."""
    from mazero_amd.synthetic import DEFAULTS, make_search_inputs, readbacks

    B, A, K, S = 48, 9, 5, 24
    inp = make_search_inputs(np.random.default_rng(21), B, A, S)
    c2, c1, g = DEFAULTS["pb_c_base"], DEFAULTS["pb_c_init"], DEFAULTS["discount"]
    # CPU port with the same call sequence (hidden_state_index_x frozen at 1 like the graph)
    ref = make_tb(port_lib, inp, K, {})
    ref.prepare(inp.root_reward, inp.root_value, inp.root_policy, inp.root_beta, K, inp.noise_eps, inp.root_noise)
    ref_sel = [ref.batch_selection(c2, c1, g)[0]]
    for s in range(S - 1):
        ref.batch_expansion_and_backup(1, g, K, inp.reward[s], inp.value[s], inp.policy[s], inp.beta[s])
        ref_sel.append(ref.batch_selection(c2, c1, g)[0])
    dinp = to_device(inp)
    tb = make_tb(gpu_lib, inp, K, {})
    dev = torch.device("cuda")
    out = (torch.empty(B, dtype=torch.int32, device=dev), torch.empty(B, dtype=torch.int32, device=dev),
           torch.empty(B, 1, dtype=torch.int32, device=dev))
    stat = [torch.empty_like(dinp.reward[0]), torch.empty_like(dinp.value[0]), torch.empty_like(dinp.policy[0]),
            torch.empty_like(dinp.beta[0])]
    stream = torch.cuda.Stream()
    with torch.cuda.stream(stream):
        tb.prepare(dinp.root_reward, dinp.root_value, dinp.root_policy, dinp.root_beta, K, dinp.noise_eps,
                   dinp.root_noise)
        tb.batch_selection_device(c2, c1, g, out=out)
    torch.cuda.synchronize()
    got = [out[0].cpu().tolist()]
    graph = torch.cuda.CUDAGraph()
    for st_, src in zip(stat, (dinp.reward[0], dinp.value[0], dinp.policy[0], dinp.beta[0])):
        st_.copy_(src)
    torch.cuda.synchronize()
    with torch.cuda.graph(graph, stream=stream):
        tb.expansion_backup_selection_device(1, g, K, *stat, c2, c1, out=out)
    # capture does not execute: replay the step for every simulation with fresh inputs
    for s in range(S - 1):
        for st_, src in zip(stat, (dinp.reward[s], dinp.value[s], dinp.policy[s], dinp.beta[s])):
            st_.copy_(src)
        graph.replay()
        torch.cuda.synchronize()
        got.append(out[0].cpu().tolist())
    assert got == ref_sel
    a, b = readbacks(tb, g), readbacks(ref, g)
    for k in ("root_values", "marginal_visit_count", "sampled_qvalues"):
        assert np.array_equal(a[k], b[k]), k


# ---- agent_num > 1: joint-action trees (upstream MAZero semantics) ----------
JOINT = [
    # (name, B, N, A, K, S)
    ("matrix_n2_k5", 8, 2, 3, 5, 25),
    ("3m_n3_k5", 32, 3, 9, 5, 30),
    ("n2_k1_chain", 16, 2, 9, 1, 30),
    ("n5_k10_keywrap", 16, 5, 11, 10, 20),  # 23333^5 overflows int64: two's-complement key order
    ("n6_a4_k16", 8, 6, 4, 16, 15),
    ("n2_a1", 4, 2, 1, 3, 10),               # single-action agents draw no engine words
    ("n2_k64_s60_hbm", 8, 2, 9, 64, 60),     # 3,905-node pools: k_hbm<joint>
]


def _joint_run(lib, B, N, A, K, S, seed):
    from mazero_amd.cytree import Tree_batch

    rng = np.random.default_rng(seed)
    pol = lambda: rng.dirichlet([1.0] * A, (B, N)).astype(np.float32) if A > 1 else np.ones((B, N, A), np.float32)  # noqa: E731
    p0, b0 = pol(), pol()
    noise = rng.dirichlet([0.3] * A, (B, N)).astype(np.float32) if A > 1 else np.ones((B, N, A), np.float32)
    r0 = (0.1 * rng.standard_normal(B)).astype(np.float32)
    v0 = rng.standard_normal(B).astype(np.float32)
    tb = Tree_batch(B, N, A, K, S, 0.01, 17, 0.75, 0.8, lib=lib)
    tb.prepare(r0, v0, p0, b0, K, 0.25, noise)
    rec = []
    for s in range(S):
        ix, iy, act = tb.batch_selection(19652.0, 1.25, 0.997)
        rec.append((np.asarray(ix), np.asarray(act).copy()))
        r = (0.1 * rng.standard_normal(B)).astype(np.float32)
        v = rng.standard_normal(B).astype(np.float32)
        p, b = pol(), pol()
        tb.batch_expansion_and_backup(s + 1, 0.997, K, r, v, p, b)
    out = dict(values=tb.get_roots_values(), mv=tb.get_roots_marginal_visit_count(),
               mp=tb.get_roots_marginal_priors(), q=tb.get_roots_sampled_qvalues(0.997),
               acts=tb.get_roots_sampled_actions(), vc=tb.get_roots_sampled_visit_count(),
               pr=tb.get_roots_sampled_priors(), bh=tb.get_roots_sampled_beta_hat())
    return rec, out


@pytest.mark.gpu
@pytest.mark.parametrize("name,B,N,A,K,S", JOINT, ids=[j[0] for j in JOINT])
@pytest.mark.parametrize("hbm", [False, True], ids=["lds", "hbm"])
def test_joint_action_trees_vs_port(gpu_lib, port_lib, name, B, N, A, K, S, hbm, monkeypatch):
    if hbm:
        monkeypatch.setenv("MZ_HBM", "1")
    rec_g, out_g = _joint_run(gpu_lib, B, N, A, K, S, 3)
    monkeypatch.delenv("MZ_HBM", raising=False)
    rec_c, out_c = _joint_run(port_lib, B, N, A, K, S, 3)
    for s, ((ig, ag), (ic, ac)) in enumerate(zip(rec_g, rec_c)):
        np.testing.assert_array_equal(ig, ic, err_msg=f"idx sim {s}")
        np.testing.assert_array_equal(ag, ac, err_msg=f"actions sim {s}")
        assert ag.shape == (B, N)
    for k in ("values", "mv", "mp"):
        g, c = out_g[k], out_c[k]
        assert g.shape == c.shape and g.dtype == c.dtype, k
        np.testing.assert_array_equal(g.view(np.int32), c.view(np.int32), err_msg=k)
    for k in ("q", "acts", "vc", "pr", "bh"):
        for i, (g, c) in enumerate(zip(out_g[k], out_c[k])):
            assert g.shape == c.shape, (k, i)
            np.testing.assert_array_equal(g.view(np.int32), c.view(np.int32), err_msg=f"{k}[{i}]")
    assert (out_g["mv"].sum(axis=2) == S).all()  # every agent's marginal sums to the simulations


@pytest.mark.parametrize("K", [1, 5])
def test_prepare_select_and_one_launch_readback(gpu_lib, port_lib, K):
    """mz_prepare_select (prepare + the first selection in one launch) and mz_get_roots_device (every
    readback in one launch) against the separate calls of the CPU port, at a BASELINE-like size."""
    from mazero_amd.synthetic import DEFAULTS, make_search_inputs, readbacks

    B, A, S = 128, 9, 30
    inp = make_search_inputs(np.random.default_rng(40 + K), B, A, S)
    c2, c1, g = DEFAULTS["pb_c_base"], DEFAULTS["pb_c_init"], DEFAULTS["discount"]
    ref = make_tb(port_lib, inp, K, {})
    ref.prepare(inp.root_reward, inp.root_value, inp.root_policy, inp.root_beta, K, inp.noise_eps, inp.root_noise)
    ref_sel = [ref.batch_selection(c2, c1, g)]
    for s in range(S - 1):
        ref.batch_expansion_and_backup(s + 1, g, K, inp.reward[s], inp.value[s], inp.policy[s], inp.beta[s])
        ref_sel.append(ref.batch_selection(c2, c1, g))
    dinp = to_device(inp)
    tb = make_tb(gpu_lib, inp, K, {})
    dev = torch.device("cuda")
    out = (torch.empty(B, dtype=torch.int32, device=dev), torch.empty(B, dtype=torch.int32, device=dev),
           torch.empty(B, 1, dtype=torch.int32, device=dev))
    tb.prepare_selection_device(dinp.root_reward, dinp.root_value, dinp.root_policy, dinp.root_beta, K,
                                dinp.noise_eps, dinp.root_noise, c2, c1, g, out=out)
    got = [(out[0].cpu().tolist(), out[1].cpu().tolist(), out[2].cpu().numpy())]
    for s in range(S - 1):
        tb.expansion_backup_selection_device(s + 1, g, K, dinp.reward[s], dinp.value[s], dinp.policy[s],
                                             dinp.beta[s], c2, c1, out=out)
        got.append((out[0].cpu().tolist(), out[1].cpu().tolist(), out[2].cpu().numpy()))
    for s, ((gi, gy, ga), (ri, ry, ra)) in enumerate(zip(got, ref_sel)):
        assert gi == list(ri) and gy == list(ry), f"selection {s}"
        assert np.array_equal(ga.reshape(B, -1), np.asarray(ra).reshape(B, -1)), f"actions {s}"
    # every field of one mz_get_roots_device launch == the per-field readbacks of the port
    from mazero_amd._capi import FIELDS, INT_FIELDS

    exp = readbacks(ref, g)
    W = tb.max_children()
    vals = torch.empty(B, device=dev)
    mv = torch.empty(B, 1, A, dtype=torch.int32, device=dev)
    mp = torch.empty(B, 1, A, device=dev)
    deg = torch.empty(B, dtype=torch.int32, device=dev)
    sampled = {f: torch.zeros(B, W, dtype=torch.int32 if f in INT_FIELDS else torch.float32, device=dev) for f in FIELDS}
    tb.get_roots_device(g, values=vals, marginal_visit_count=mv, marginal_priors=mp, degrees=deg, sampled=sampled)
    torch.cuda.synchronize()
    assert np.array_equal(vals.cpu().numpy().view(np.int32), exp["root_values"].view(np.int32))
    assert np.array_equal(mv.cpu().numpy(), exp["marginal_visit_count"])
    assert np.array_equal(mp.cpu().numpy().view(np.int32), np.asarray(exp["marginal_priors"], np.float32).view(np.int32))
    assert np.array_equal(deg.cpu().numpy(), exp["degree"])
    for f, t_ in sampled.items():
        e = exp["sampled_" + f]
        gg = t_.cpu().numpy()[:, : e.shape[1]]
        assert np.array_equal(gg.view(np.int32), e.astype(gg.dtype).view(np.int32)), f


@pytest.mark.parametrize("path", FULL, ids=[os.path.basename(p)[5:-4] for p in FULL])
def test_bench_sequence_vs_reference(gpu_lib, path):
    """bench.py's timed launch sequence, exactly as HipLeg.one_search issues it --
    mz_prepare_select, (S-1) x mz_expand_backup_select with the leaf-row gather from a pool,
    mz_expand_backup, one mz_get_roots_device launch -- on every BASELINE-size fixture against the
    reference ctree's own outputs (oracle/gen_golden.py --full): the selection of every simulation,
    every field of the one-launch readback, and every gathered row."""
    from mazero_amd._capi import FIELDS, INT_FIELDS
    from mazero_amd.synthetic import DEFAULTS

    inp, K, expected = load_full(path)
    d = to_device(inp)
    B, A, S = inp.B, inp.A, inp.S
    c2, c1, g = DEFAULTS["pb_c_base"], DEFAULTS["pb_c_init"], DEFAULTS["discount"]
    dev = torch.device("cuda")
    tb = make_tb(gpu_lib, inp, K, {})
    idx = torch.empty(S, B, dtype=torch.int32, device=dev)
    idy = torch.empty(S, B, dtype=torch.int32, device=dev)
    act = torch.empty(S, B, 1, dtype=torch.int32, device=dev)
    pool = torch.randn(S + 1, B, 96, device=dev)
    leaf = torch.full((S, B, 96), float("nan"), device=dev)
    tb.prepare_selection_device(d.root_reward, d.root_value, d.root_policy, d.root_beta, K, d.noise_eps, d.root_noise,
                                c2, c1, g, out=(idx[0], idy[0], act[0]))
    for s in range(S):
        if s + 1 < S:
            tb.expansion_backup_selection_device(s + 1, g, K, d.reward[s], d.value[s], d.policy[s], d.beta[s], c2, c1,
                                                 out=(idx[s + 1], idy[s + 1], act[s + 1]), pool=pool,
                                                 gather_out=leaf[s + 1])
        else:
            tb.batch_expansion_and_backup(s + 1, g, K, d.reward[s], d.value[s], d.policy[s], d.beta[s])
    W = tb.max_children()
    vals = torch.empty(B, device=dev)
    mv = torch.empty(B, 1, A, dtype=torch.int32, device=dev)
    mp = torch.empty(B, 1, A, device=dev)
    deg = torch.empty(B, dtype=torch.int32, device=dev)
    sampled = {f: torch.full((B, W), -7, dtype=torch.int32 if f in INT_FIELDS else torch.float32, device=dev)
               for f in FIELDS}
    tb.get_roots_device(g, values=vals, marginal_visit_count=mv, marginal_priors=mp, degrees=deg, sampled=sampled)
    torch.cuda.synchronize()
    name = os.path.basename(path)
    assert (idy.cpu().numpy() == np.arange(B, dtype=np.int32)[None]).all()
    got = dict(sel_idx=idx.cpu().numpy(), sel_act=act.cpu().numpy()[:, :, 0], root_values=vals.cpu().numpy(),
               marginal_visit_count=mv.cpu().numpy(), marginal_priors=mp.cpu().numpy(), degree=deg.cpu().numpy())
    assert_same(got, {k: expected[k] for k in got}, f"bench sequence {name} ")
    dg = got["degree"]
    for f, t_ in sampled.items():
        e = expected["sampled_" + f]
        gg = t_.cpu().numpy()[:, : e.shape[1]].copy()
        for i in range(B):  # entries past a root's degree are padding (zeros in the fixture)
            gg[i, dg[i]:] = 0
        assert_same({f: gg}, {f: e}, f"bench sequence {name} ")
    # the leaf rows each fused launch gathered: pool[idx_x[i]][i] (mcts_sampled.py:130-134)
    ix = idx[1:].long()
    exp_rows = pool[ix, torch.arange(B, device=dev)[None, :]]
    assert torch.equal(leaf[1:], exp_rows), f"{name}: gathered rows"


def test_get_roots_device_checks_outputs(gpu_lib):
    """get_roots_device refuses caller tensors the readback launch would overrun or misread
    (ADVICE r2): wrong dtype, too few elements, non-contiguous, host tensors."""
    from mazero_amd.synthetic import make_search_inputs, run_search

    inp = make_search_inputs(np.random.default_rng(3), 8, 9, 6)
    tb = make_tb(gpu_lib, inp, 3, {})
    run_search(tb, inp, 3, {}, record=False)
    dev = torch.device("cuda")
    W = tb.max_children()
    bad = [
        dict(values=torch.empty(8, dtype=torch.float64, device=dev)),
        dict(values=torch.empty(7, device=dev)),
        dict(marginal_visit_count=torch.empty(8, 1, 9, device=dev)),
        dict(marginal_priors=torch.empty(8, 9, 2, device=dev)[:, :, 0]),
        dict(degrees=torch.empty(8, dtype=torch.int32)),
        dict(sampled={"visit_count": torch.empty(8, W - 1, dtype=torch.int32, device=dev)}),
        dict(sampled={"priors": torch.empty(8, W, dtype=torch.int32, device=dev)}),
    ]
    for kw in bad:
        with pytest.raises(ValueError):
            tb.get_roots_device(0.997, **kw)
    v = torch.empty(8, device=dev)
    tb.get_roots_device(0.997, values=v, sampled={"visit_count": torch.empty(8, W, dtype=torch.int32, device=dev)})
    torch.cuda.synchronize()
    assert np.array_equal(v.cpu().numpy().view(np.int32), tb.get_roots_values().view(np.int32))


# MZ_FUZZ_CHUNKS=N widens the fuzz to N chunks of ten configurations (a one-off deeper run)
@pytest.mark.parametrize("chunk", range(int(os.environ.get("MZ_FUZZ_CHUNKS", "4"))))
def test_fuzz_small_configs_vs_port(gpu_lib, port_lib, chunk):
    """Forty seeded random configurations (A from 1 to 64, K from 1 to 70 -- chains, trees, the
    general kernel --, S from 1 to 60, B from 1 to 48, every search knob varied, masks, ties, noise
    on and off): the device loop (fused launches) against the CPU port, every selection and readback,
    and every fourth one through the host path too."""
    from dataclasses import replace

    from mazero_amd.synthetic import make_search_inputs, run_search

    from fuzz_configs import fuzz_configs

    for i, (B, A, K, S, knobs, lz, ties, eps, s) in enumerate(fuzz_configs(1234 + chunk, 10)):
        rng = np.random.default_rng(s)
        inp = replace(make_search_inputs(rng, B, A, S, legal_zero_frac=lz, ties=ties), noise_eps=eps)
        where = f"B={B} A={A} K={K} S={S} knobs={knobs} lz={lz} ties={ties} eps={eps}: "
        # every configuration is accepted (pools past the LDS image take k_hbm); every third one is
        # also forced onto k_hbm
        if i % 3 == 1:
            os.environ["MZ_HBM"] = "1"
        try:
            tb = make_tb(gpu_lib, inp, K, knobs)
        finally:
            os.environ.pop("MZ_HBM", None)
        big = 1 + min(K, A) * (S + 1) > 2300
        assert tb.fused_kernel() == "k_hbm" or not big, where + tb.fused_kernel()
        exp = run_search(make_tb(port_lib, inp, K, knobs), inp, K, knobs)
        exp = {k: v for k, v in exp.items() if k not in ("root_values_per_sim", "marginal_per_sim")}
        out, _ = run_fused(tb, to_device(inp), K, knobs)
        assert_same(out, exp, "gpu fused " + where)
        if i % 4 == 0:
            host = run_search(make_tb(gpu_lib, inp, K, knobs), inp, K, knobs)
            host = {k: v for k, v in host.items() if k not in ("root_values_per_sim", "marginal_per_sim")}
            assert_same(host, exp, "gpu host path " + where)


@pytest.mark.parametrize("chunk", range(int(os.environ.get("MZ_FUZZ_CHUNKS", "2"))))
def test_fuzz_large_configs_vs_port(gpu_lib, port_lib, chunk):
    """Four seeded random configurations at SMAC-like sizes (A 5-64, K 1-16, S 60-300, B 64-512):
    the fused device loop against the CPU port, every selection and readback; none is refused
    (pools over the per-tree LDS limit take k_hbm)."""
    from dataclasses import replace

    from mazero_amd.synthetic import make_search_inputs, run_search

    from fuzz_configs import fuzz_configs_large

    for B, A, K, S, knobs, lz, ties, eps, s in fuzz_configs_large(777 + chunk, 4):
        rng = np.random.default_rng(s)
        inp = replace(make_search_inputs(rng, B, A, S, legal_zero_frac=lz, ties=ties), noise_eps=eps)
        where = f"B={B} A={A} K={K} S={S} knobs={knobs} lz={lz} eps={eps}: "
        tb = make_tb(gpu_lib, inp, K, knobs)
        exp = run_search(make_tb(port_lib, inp, K, knobs), inp, K, knobs)
        exp = {k: v for k, v in exp.items() if k not in ("root_values_per_sim", "marginal_per_sim")}
        out, _ = run_fused(tb, to_device(inp), K, knobs)
        assert_same(out, exp, "gpu fused " + where)
