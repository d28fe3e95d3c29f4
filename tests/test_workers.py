"""Process-per-GPU self-play / reanalyze harness (mazero_amd.workers) on the
CPU: gloo, world size 2, the oracle search driver over the CPU port and the restated host
consumers injected in place of the MI355X search and the device consumers.

Checked:
- every rank's decisions in every step are rows [lo, hi) of an unsharded run of the same loop
  (actions, recorded policy probability, visit entropies, root values), bit for bit;
- the weights come from the learner's rank by the reference's checkpoint-interval rule
  (selfplay_worker.py:371-375): rank 1 starts from different weights, pulls checkpoint 0 before its
  first step, and later checkpoints arrive only when the trained-steps counter crosses a multiple
  of checkpoint_interval;
- reanalyze policy targets of a sharded batch equal the unsharded targets.
"""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import PORT_LIB, ROOT

N, A, OBS, TOTAL, STEPS, CI = 3, 9, 16, 10, 5, 20


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _env(t, lo, hi):
    rng = np.random.default_rng(1000 + t)
    obs = rng.standard_normal((TOTAL, N, OBS)).astype(np.float32)
    legal = (rng.random((TOTAL, N, A)) > 0.3).astype(np.int64)
    legal[..., 1] = 1
    return torch.from_numpy(obs[lo:hi]), legal[lo:hi]


def _eps_uniforms(t):
    rng = np.random.default_rng(2000 + t)
    return rng.random((N, TOTAL)).astype(np.float32), rng.random((N, TOTAL))


class _Learner:
    """Stands in for the training loop: after every env step it has trained 10 more steps and
    offers new weights (a deterministic perturbation of its own copy)."""

    def __init__(self, model):
        self.sd = {k: v.detach().clone() for k, v in model.state_dict().items()}

    def __call__(self, model, t):
        g = torch.Generator().manual_seed(t)
        for k, v in self.sd.items():
            if v.is_floating_point():
                v.mul_(0.9).add_(0.05 * torch.randn(v.shape, generator=g))
        return 10 * (t + 1), self.sd


def _run(rank, group, port_lib, make_net, SearchConfig, wb_cls, shard_cls, oracle_driver, oracle_consume, seed_w):
    net = make_net(N, A, obs_size=OBS, seed=seed_w)
    wb = wb_cls(net, src=0, group=group, checkpoint_interval=CI)
    cfg = SearchConfig(action_space_size=A, num_simulations=8, sampled_action_times=3)

    def make_mcts(config, rs, shard):
        return oracle_driver.OracleSampledMCTS(config, rs, port_lib, root_shard=shard)

    def decide(mcts, model, net_out, n, legal, *, temperature, sampled_tau, greedy_epsilon, eps_uniforms, device):
        u_eps, u_cat = eps_uniforms
        return oracle_consume.selfplay_step(mcts, model, net_out, n, legal, temperature, sampled_tau, greedy_epsilon,
                                            mcts.np_random, u_eps, u_cat, device, root_shard=mcts.root_shard)

    sp = shard_cls(net, cfg, TOTAL, N, seed=11, broadcaster=wb, group=group, make_mcts=make_mcts, decide=decide)
    learner = _Learner(make_net(N, A, obs_size=OBS, seed=7)) if rank == 0 else None
    recs = sp.run(_env, STEPS, learner=learner, eps_uniforms=_eps_uniforms, greedy_epsilon=0.25)
    return recs, wb.syncs


def _reanalyze(group, port_lib, make_net, SearchConfig, wb_cls, re_cls, oracle_driver, oracle_consume, seed_w):
    net = make_net(N, A, obs_size=OBS, seed=seed_w)
    wb = wb_cls(net, src=0, group=group, checkpoint_interval=CI)
    cfg = SearchConfig(action_space_size=A, num_simulations=6, sampled_action_times=2)

    def make_mcts(config, rs, shard):
        return oracle_driver.OracleSampledMCTS(config, rs, port_lib, root_shard=shard)

    def decide(mcts, model, net_out, legal, policy_mask, device):
        return oracle_consume.reanalyze_policy(mcts, model, net_out, legal, policy_mask, mcts.np_random, device)

    rs = re_cls(net, cfg, TOTAL, seed=5, broadcaster=wb, group=group, make_mcts=make_mcts, decide=decide)
    obs, legal = _env(99, rs.lo, rs.hi)
    return rs.targets(obs, legal, np.ones(rs.hi - rs.lo))


def _worker(rank, world, port, q):
    import ctypes as C
    import sys

    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
    import torch.distributed as dist

    import consume as oracle_consume
    import driver as oracle_driver
    from mazero_amd import _capi
    from mazero_amd.nets import SearchConfig, make_net
    from mazero_amd.weights import WeightBroadcaster
    from mazero_amd.workers import ReanalyzeShard, SelfPlayShard

    torch.set_num_threads(1)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    solo = dist.new_group([0])  # rank 0 alone: the unsharded run
    port_lib = _capi.bind(C.CDLL(PORT_LIB))
    common = (port_lib, make_net, SearchConfig, WeightBroadcaster)
    # every rank starts from its own weights: checkpoint 0 comes from rank 0
    recs, syncs = _run(rank, None, *common, SelfPlayShard, oracle_driver, oracle_consume, seed_w=7 + 100 * rank)
    re_t = _reanalyze(None, *common, ReanalyzeShard, oracle_driver, oracle_consume, seed_w=7 + 100 * rank)
    got = [None] * world
    dist.all_gather_object(got, (recs, syncs, re_t))
    if rank == 0:
        ref_recs, ref_syncs = _run(0, solo, *common, SelfPlayShard, oracle_driver, oracle_consume, seed_w=7)
        ref_re = _reanalyze(solo, *common, ReanalyzeShard, oracle_driver, oracle_consume, seed_w=7)
        q.put((got, ref_recs, ref_syncs, ref_re))
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_selfplay_matches_unsharded(port_lib):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world = 2
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got, ref, ref_syncs, ref_re = q.get(timeout=600)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # the checkpoint each step searched with: 0 first, then every crossing of a multiple of CI
    # by the counter (10 per step): 0, 0 (10), 20, 20 (30), 40
    want_idx = [0, 0, 20, 20, 40]
    assert [r.model_index for r in ref] == want_idx
    for rank in range(world):
        recs, syncs, _ = got[rank]
        assert [r.model_index for r in recs] == want_idx
        assert syncs == 3  # checkpoints 0, 20, 40 moved; 10 and 30 did not
    assert ref_syncs == 3
    for t in range(STEPS):
        for f in ("actions", "prob_action", "root_value", "count_entropy", "visit_entropy"):
            cat = np.concatenate([getattr(got[r][0][t], f) for r in range(world)])
            exp = getattr(ref[t], f)
            assert cat.shape == exp.shape, (t, f)
            assert np.array_equal(cat, exp), f"step {t} field {f}: sharded != unsharded"
        assert [got[r][0][t].lo for r in range(world)] == [0, TOTAL // 2]
    # reanalyze targets
    for k in ("sampled_actions", "sampled_policies", "sampled_qvalues", "root_mcts_values"):
        cat = np.concatenate([np.asarray(got[r][2][k]) for r in range(world)])
        assert np.array_equal(cat, np.asarray(ref_re[k])), k


@pytest.mark.gpu
def test_sharded_selfplay_on_device_matches_unsharded():
    """The default harness on one MI355X: SampledMCTS(root_shard=...) and the device consumers.
    Two shards (ranks 0 and 1 of 2, run one after the other in this process) decide exactly the
    rows of the unsharded step."""
    from mazero_amd.nets import SearchConfig, make_net
    from mazero_amd.workers import SelfPlayShard

    dev = torch.device("cuda", 0)
    total = 64
    net = make_net(N, A, obs_size=OBS, seed=3, device=dev)
    cfg = SearchConfig(action_space_size=A, num_simulations=12, sampled_action_times=2)

    def env(t, lo, hi):
        rng = np.random.default_rng(500 + t)
        obs = rng.standard_normal((total, N, OBS)).astype(np.float32)
        legal = (rng.random((total, N, A)) > 0.3).astype(np.int64)
        legal[..., 1] = 1
        return torch.from_numpy(obs[lo:hi]).to(dev), legal[lo:hi]

    def eps_u(t):
        rng = np.random.default_rng(600 + t)
        return rng.random((N, total)).astype(np.float32), rng.random((N, total))

    def run(rank, world):
        sp = SelfPlayShard(net, cfg, total, N, seed=21, rank=rank, world=world, device=dev)
        return sp.run(env, 3, eps_uniforms=eps_u, greedy_epsilon=0.25)

    ref = run(0, 1)
    parts = [run(r, 2) for r in range(2)]
    for t in range(3):
        for f in ("actions", "prob_action", "root_value", "count_entropy", "visit_entropy"):
            cat = np.concatenate([getattr(parts[r][t], f) for r in range(2)])
            assert np.array_equal(cat, getattr(ref[t], f)), f"step {t} field {f}"
