"""On-device consumers of the search output (mazero_amd.consume, include/mzconsume.h) against the
restated reference consumers (oracle/consume.py: core/utils.py:289-334,
core/selfplay_worker.py:189-293, core/reanalyze_worker.py:266-366).

CPU tests pin what the kernels rely on:
- numpy's `choice(n, p)` draws exactly one double per call, so one `random(B)` per agent
  replaces the per-root draws (Generator and RandomState);
- the kernels' arithmetic (repeated products, sequential sums, cdf / last > u) picks the same
  child as numpy's `choice`;
- torch compares the epsilon-greedy draw with eps in float32;
- the inverse-cdf categorical has Categorical(mask)'s distribution.
GPU tests compare the kernels bit for bit (entropies to 1e-12), then whole self-play steps and
reanalyze targets against the oracle driver + oracle consumers on the same network.
"""
from __future__ import annotations

import math

import numpy as np
import pytest
import torch

from consume import categorical_given, eps_greedy_given, reanalyze_policy, select_action, selfplay_step


def kernel_select(row, temperature, deterministic, u):
    """The arithmetic of k_select_actions (mzconsume.hip), in Python floats."""
    e = 1.0 / temperature
    ipow = int(e) if (e == math.floor(e) and 1.0 <= e <= 8.0) else 0

    def vp(v):
        if ipow == 0:
            return float(v) ** e
        r = float(v)
        for _ in range(ipow - 1):
            r *= float(v)
        return r

    n = len(row)
    total = 0.0
    for v in row:
        total += vp(v)
    if deterministic:
        pos = 0
        for j in range(1, n):
            if row[j] > row[pos]:
                pos = j
        return pos
    last = 0.0
    for v in row:
        last += vp(v) / total
    c = 0.0
    for j, v in enumerate(row):
        c += vp(v) / total
        if c / last > u:
            return j
    return n - 1


def _rows(rng, n_rows, kmax, vmax=60):
    out = []
    for _ in range(n_rows):
        n = int(rng.integers(1, kmax + 1))
        r = rng.integers(0, vmax, size=n).astype(np.int32)
        if r.sum() == 0:
            r[rng.integers(0, n)] = 1
        out.append(r)
    return out


@pytest.mark.parametrize("gen", ["generator", "randomstate"])
@pytest.mark.parametrize("temperature", [1.0, 0.5, 0.25])
def test_choice_is_one_double_per_root(gen, temperature):
    """select_action's np_random.choice (core/utils.py:311-314) == inverse cdf of one
    np_random.random() per root, drawn as one batch in root order; same generator state after."""
    rows = _rows(np.random.default_rng(1), 400, 10)
    make = (lambda: np.random.Generator(np.random.PCG64(7))) if gen == "generator" else \
        (lambda: np.random.RandomState(7))
    ra, rb = make(), make()
    exp = [select_action(r, temperature=temperature, deterministic=False, np_random=ra)[0] for r in rows]
    u = rb.random(len(rows))
    got = [kernel_select(list(r), temperature, False, u[i]) for i, r in enumerate(rows)]
    assert got == [int(x) for x in exp]
    assert ra.random() == rb.random()


def test_kernel_arithmetic_deterministic_and_ties():
    rows = _rows(np.random.default_rng(2), 300, 8, vmax=4)  # many ties
    for r in rows:
        assert kernel_select(list(r), 1.0, True, 0.0) == int(select_action(r, 1.0, True)[0])


def test_eps_threshold_is_float32_like_torch():
    """torch compares a float32 draw with a Python float in float32 (core/utils.py:327-328)."""
    for eps in (0.7, 0.3, 0.1, 0.05, 1e-7):
        e32 = np.float32(eps)
        for u in (e32, np.nextafter(e32, np.float32(0)), np.nextafter(e32, np.float32(1))):
            t = bool((torch.tensor([u], dtype=torch.float32) < eps).item())
            assert t == bool(np.float32(u) < e32), (eps, u)
            picked = eps_greedy_given(-7, np.ones(5, np.int64), eps, u, 0.5) != -7
            assert picked == t


def test_categorical_given_matches_torch_categorical_distribution():
    rng = np.random.default_rng(3)
    torch.manual_seed(0)
    for _ in range(6):
        w = (rng.random(9) > 0.4).astype(np.int64)
        w[rng.integers(0, 9)] = 1
        grid = (np.arange(20000) + 0.5) / 20000
        ours = np.bincount([categorical_given(w, u) for u in grid], minlength=9) / grid.size
        np.testing.assert_allclose(ours, w / w.sum(), atol=1e-4)
        ts = torch.distributions.Categorical(torch.from_numpy(w)).sample((20000,)).numpy()
        theirs = np.bincount(ts, minlength=9) / ts.size
        assert (theirs[w == 0] == 0).all()
        np.testing.assert_allclose(theirs, w / w.sum(), atol=0.02)


# ------------------------------------------------------------------------------------------------
# GPU
# ------------------------------------------------------------------------------------------------
def _synthetic_output(B, A, width, rng, dev, N=1):
    """A DeviceSearchOutput with synthetic per-root lists, bound to a fresh handle (for the stream
    and geometry only)."""
    from mazero_amd.cytree import Tree_batch
    from mazero_amd.mcts_sampled import DeviceSearchOutput

    tb = Tree_batch(B, N, A, width, 4, 0.01, 0, 0.75, 0.8)
    deg = rng.integers(1, width + 1, size=B).astype(np.int32)
    visits = np.zeros((B, width), np.int32)
    actions = np.zeros((B, width * N), np.int32)
    for i in range(B):
        r = rng.integers(0, 40, size=deg[i]).astype(np.int32)
        if r.sum() == 0:
            r[0] = 3
        visits[i, : deg[i]] = r
        actions[i, : deg[i] * N] = rng.integers(0, A, size=deg[i] * N)
    marg = rng.integers(0, 30, size=(B, N, A)).astype(np.int32)
    marg[rng.random(B) < 0.05] = 0  # roots without visits
    t = lambda a: torch.from_numpy(a).to(dev)  # noqa: E731
    out = DeviceSearchOutput(t(np.zeros(B, np.float32)), t(marg), t(np.zeros((B, N, A), np.float32)), t(deg),
                             {"visit_count": t(visits), "actions": t(actions)}, tb)
    return out, deg, visits, actions, marg


def _eps_fixture():
    import os

    return np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "eps_greedy_torch.npz"))


def test_torch_eps_draws_replay_reference_eps_greedy():
    """mazero_amd.consume.torch_eps_uniforms turns torch's CPU stream into the kernel's uniforms:
    with the same torch seed, eps_greedy_given (the kernel's arithmetic) reproduces the actions
    core/utils.py's eps_greedy_action itself produced root after root (tests/golden/
    eps_greedy_torch.npz, recorded by oracle/gen_driver_golden.py), for eps 0.1, 0.5, 1.0."""
    from mazero_amd.consume import torch_eps_uniforms

    z = _eps_fixture()
    masks, greedy = z["masks"], z["greedy"]
    for j, (eps, seed) in enumerate(zip(z["eps"], z["seeds"])):
        torch.manual_seed(int(seed))
        u_eps, u_cat = torch_eps_uniforms(masks)
        got = [eps_greedy_given(greedy[i], masks[i], float(eps), u_eps[i], u_cat[i]) for i in range(len(greedy))]
        np.testing.assert_array_equal(np.asarray(got, np.int64), z[f"actions_eps{j}"], err_msg=f"eps={eps}")


@pytest.mark.gpu
def test_eps_greedy_kernel_torch_stream():
    """The device kernel fed torch_eps_uniforms reproduces the reference's eps_greedy_action."""
    from mazero_amd.consume import eps_greedy, torch_eps_uniforms

    dev = torch.device("cuda", 0)
    z = _eps_fixture()
    masks, greedy = z["masks"], z["greedy"]
    B, A = masks.shape
    out, *_ = _synthetic_output(B, A, 4, np.random.default_rng(3), dev)
    legal_d = torch.from_numpy(masks.astype(np.int32)).to(dev)
    for j, (eps, seed) in enumerate(zip(z["eps"], z["seeds"])):
        torch.manual_seed(int(seed))
        u_eps, u_cat = torch_eps_uniforms(masks)
        act = torch.from_numpy(greedy.copy()).to(dev)
        eps_greedy(out, act, legal_d, float(eps), torch.from_numpy(u_eps).to(dev), torch.from_numpy(u_cat).to(dev))
        np.testing.assert_array_equal(act.cpu().numpy().astype(np.int64), z[f"actions_eps{j}"], err_msg=f"eps={eps}")


@pytest.mark.gpu
@pytest.mark.parametrize("temperature", [1.0, 0.5, 0.25, 0.3])
@pytest.mark.parametrize("deterministic", [False, True])
def test_select_actions_kernel(temperature, deterministic):
    from mazero_amd.consume import select_actions

    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(int(temperature * 100) + deterministic)
    B, A, W = 300, 9, 10
    out, deg, visits, actions, _ = _synthetic_output(B, A, W, rng, dev)
    gen = np.random.Generator(np.random.PCG64(5))
    u = np.random.Generator(np.random.PCG64(5)).random(B)
    pos, act, ent = select_actions(out, torch.from_numpy(u).to(dev), temperature, deterministic)
    pos, act, ent = pos.cpu().numpy(), act.cpu().numpy(), ent.cpu().numpy()
    for i in range(B):
        row = visits[i, : deg[i]]
        p, h = select_action(row, temperature=temperature, deterministic=deterministic, np_random=gen)
        assert pos[i] == p, i
        assert act[i] == actions[i, p]
        np.testing.assert_allclose(ent[i], h, rtol=1e-12, atol=1e-15)


@pytest.mark.gpu
def test_eps_greedy_kernel():
    from mazero_amd.consume import eps_greedy

    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(9)
    B, A = 257, 11
    out, *_ = _synthetic_output(B, A, 4, rng, dev)
    legal = (rng.random((B, 3, A)) > 0.35).astype(np.int32)
    legal[5] = 0  # no legal action: greedy kept
    greedy = rng.integers(0, A, size=B).astype(np.int32)
    u_eps = rng.random(B).astype(np.float32)
    u_eps[:4] = np.float32(0.7)
    u_cat = rng.random(B)
    act = torch.from_numpy(greedy.copy()).to(dev)
    legal_d = torch.from_numpy(legal).to(dev)
    eps_greedy(out, act, legal_d[:, 1, :], 0.7, torch.from_numpy(u_eps).to(dev), torch.from_numpy(u_cat).to(dev))
    exp = [eps_greedy_given(greedy[i], legal[i, 1], 0.7, u_eps[i], u_cat[i]) for i in range(B)]
    np.testing.assert_array_equal(act.cpu().numpy(), np.asarray(exp, np.int32))


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["given", "argmax"])
def test_marginal_policy_kernel(mode):
    from mazero_amd._capi import MZ_MARGINAL_ARGMAX, MZ_MARGINAL_GIVEN
    from mazero_amd.consume import marginal_policy

    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(11)
    B, A = 200, 15
    out, _, _, _, marg = _synthetic_output(B, A, 5, rng, dev)
    legal = (rng.random((B, A)) > 0.3).astype(np.int32)
    prob0 = rng.random(B) + 0.5
    prob = torch.from_numpy(prob0.copy()).to(dev)
    ent = torch.full((B,), -5.0, dtype=torch.float64, device=dev)
    if mode == "given":
        action = rng.integers(0, A, size=B).astype(np.int32)
        act = torch.from_numpy(action.copy()).to(dev)
        marginal_policy(out, MZ_MARGINAL_GIVEN, act, prob, entropy=ent)
    else:
        act = torch.full((B,), 99, dtype=torch.int32, device=dev)
        marginal_policy(out, MZ_MARGINAL_ARGMAX, act, prob, legal=torch.from_numpy(legal).to(dev), entropy=ent)
    act, prob, ent = act.cpu().numpy(), prob.cpu().numpy(), ent.cpu().numpy()
    for i in range(B):
        m = marg[i, 0]
        if mode == "argmax":
            if m.sum() == 0:
                assert act[i] == -1 and prob[i] == prob0[i] and ent[i] == -5.0
                continue
            assert act[i] == np.argmax(m * legal[i].astype(np.int64)), i
        a = act[i]
        if m.sum() > 0:
            d = m / np.sum(m)
            assert prob[i] == prob0[i] * d[a], i  # bit-exact float64
            np.testing.assert_allclose(ent[i], -np.sum(d * np.log(d + 1e-9)), rtol=1e-12, atol=1e-15)
        else:
            assert prob[i] == prob0[i] * (1.0 / A) and ent[i] == 0.0


@pytest.mark.gpu
@pytest.mark.parametrize("K,temperature,eps", [(1, 1.0, 0.0), (5, 0.5, 0.3), (3, 0.25, 1.0)])
def test_selfplay_decisions_match_oracle(K, temperature, eps, port_lib):
    """One self-play environment step (selfplay_worker.py:189-293): the device agent loop with
    device consumers == the oracle driver with the restated Python consumers."""
    from driver import OracleSampledMCTS
    from mazero_amd.consume import selfplay_decisions
    from mazero_amd.mcts_sampled import SampledMCTS
    from mazero_amd.nets import SearchConfig, make_net, make_root_batch

    N, A, B, S = 3, 9, 48, 12
    dev = torch.device("cuda", 0)
    cfg = SearchConfig(action_space_size=A, num_simulations=S, sampled_action_times=K)
    net = make_net(N, A, seed=21, device=dev)
    out, legal = make_root_batch(net, B, 64, seed=22, device=dev, legal_zero_frac=0.3)
    ur = np.random.default_rng(23)
    u_eps = ur.random((N, B)).astype(np.float32)
    u_cat = ur.random((N, B))
    rs_o = np.random.Generator(np.random.PCG64(31))
    rs_d = np.random.Generator(np.random.PCG64(31))
    exp = selfplay_step(OracleSampledMCTS(cfg, rs_o, port_lib), net, out, N, legal, temperature, 1.0, eps, rs_o,
                        u_eps, u_cat, device=dev)
    got = selfplay_decisions(SampledMCTS(cfg, rs_d), net, out, N, legal, temperature=temperature,
                             greedy_epsilon=eps, eps_uniforms=(u_eps, u_cat), device=dev)
    np.testing.assert_array_equal(got.actions.cpu().numpy(), exp["actions"])
    np.testing.assert_array_equal(got.prob_action.cpu().numpy(), exp["prob_action"])
    np.testing.assert_array_equal(got.root_value.cpu().numpy().view(np.uint32), exp["root_value"].view(np.uint32))
    np.testing.assert_allclose(got.count_entropy.cpu().numpy(), exp["count_entropy"], rtol=1e-12, atol=1e-15)
    np.testing.assert_allclose(got.visit_entropy.cpu().numpy(), exp["visit_entropy"], rtol=1e-12, atol=1e-15)
    assert rs_o.random() == rs_d.random()  # np_random consumed identically


@pytest.mark.gpu
@pytest.mark.parametrize("K", [1, 5])
def test_reanalyze_policy_targets_match_oracle(K, port_lib):
    from driver import OracleSampledMCTS
    from mazero_amd.consume import reanalyze_policy_targets
    from mazero_amd.mcts_sampled import SampledMCTS
    from mazero_amd.nets import SearchConfig, make_net, make_root_batch

    N, A, B, S = 3, 9, 40, 10
    dev = torch.device("cuda", 0)
    cfg = SearchConfig(action_space_size=A, num_simulations=S, sampled_action_times=K)
    net = make_net(N, A, seed=41, device=dev)
    out, legal = make_root_batch(net, B, 64, seed=42, device=dev, legal_zero_frac=0.25)
    mask = np.random.default_rng(43).random(B) > 0.2
    rs_o = np.random.Generator(np.random.PCG64(44))
    rs_d = np.random.Generator(np.random.PCG64(44))
    exp = reanalyze_policy(OracleSampledMCTS(cfg, rs_o, port_lib), net, out, legal, mask, rs_o, device=dev)
    got = reanalyze_policy_targets(SampledMCTS(cfg, rs_d), net, out, legal, mask, device=dev)
    for name in exp:
        g = getattr(got, name).cpu().numpy()
        e = np.asarray(exp[name])
        assert g.shape == e.shape, name
        if e.dtype == np.float32:
            np.testing.assert_array_equal(g.astype(np.float32).view(np.uint32), e.view(np.uint32), err_msg=name)
        else:
            np.testing.assert_array_equal(g, e, err_msg=name)
    assert rs_o.random() == rs_d.random()
