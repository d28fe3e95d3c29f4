"""Process-per-GPU self-play and reanalyze.

The reference runs its workers as Ray actors (`RemoteDataWorker`, core/selfplay_worker.py:344-407;
`RemoteReanalyzeWorker`, core/reanalyze_worker.py:614-722).  Each one pulls fresh weights from the
`SharedStorage` actor through the object store (core/storage.py:68-80) when the learner's trained-steps
counter has crossed into a new checkpoint interval (`_update_model_before_step`,
selfplay_worker.py:371-375; reanalyze: `target_model_interval`, reanalyze_worker.py:663-669).

Here there is one process per GPU and one rank per process:
- the environments (self-play) or the batch's roots (reanalyze) are sharded over the ranks,
  contiguously (`shard.shard_bounds`);
- every rank holds the same `np_random` state and its search is `SampledMCTS(..., root_shard=...)`:
  the per-root random draws are made for the whole batch and sliced, and tree i is seeded with its
  global index, so rank r's decisions are rows [lo, hi) of the unsharded step, bit for bit;
- the weights travel by one collective from the learner's rank (`weights.WeightBroadcaster`, RCCL
  over xGMI on MI355X; gloo on the CPU), with the reference's checkpoint-interval rule;
- nothing crosses ranks during a search.

The environment, the replay buffer and the learner stay out of scope: `env` is a
callable that yields a shard's observations and legal-action masks, and `learner` is an optional
callable run on the source rank after each step, returning the trained-steps counter it publishes.
`make_mcts` and `decide` default to the MI355X search and the on-device consumers
(mazero_amd.consume); tests inject the oracle driver and the restated host consumers to run the
same harness on the CPU.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, List, Optional

import numpy as np
import torch
import torch.distributed as dist

from .shard import shard_bounds


def _rank_world(group=None):
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(group), dist.get_world_size(group)
    return 0, 1


def _to_np(x):
    if isinstance(x, torch.Tensor):
        return x.detach().cpu().numpy()
    return np.asarray(x)


def _device_selfplay_decide(mcts, model, network_output, N, legal, *, temperature, sampled_tau, greedy_epsilon,
                            eps_uniforms, device):
    from .consume import selfplay_decisions

    d = selfplay_decisions(mcts, model, network_output, N, legal, temperature=temperature, sampled_tau=sampled_tau,
                           greedy_epsilon=greedy_epsilon, eps_uniforms=eps_uniforms, device=device)
    return dict(actions=d.actions, count_entropy=d.count_entropy, prob_action=d.prob_action,
                visit_entropy=d.visit_entropy, root_value=d.root_value)


def _device_reanalyze_decide(mcts, model, network_output, legal, policy_mask, device):
    from .consume import reanalyze_policy_targets

    return reanalyze_policy_targets(mcts, model, network_output, legal, policy_mask, device)._asdict()


def _default_mcts(config, np_random, root_shard):
    from .mcts_sampled import SampledMCTS

    return SampledMCTS(config, np_random, root_shard=root_shard)


@dataclass
class StepRecord:
    """What one rank decided in one environment step (selfplay_worker.py:189-293)."""

    step: int
    model_index: int          # the checkpoint the rank searched with
    lo: int                   # the rank's first global environment
    actions: np.ndarray       # int32 [hi - lo, N]
    prob_action: np.ndarray   # float64 [hi - lo]
    root_value: np.ndarray    # float32 [hi - lo]
    count_entropy: np.ndarray  # float64 [hi - lo, N]
    visit_entropy: np.ndarray  # float64 [hi - lo, N]


class _Shard:
    def __init__(self, model, config, total: int, *, seed: int, broadcaster=None, group=None, src: int = 0,
                 make_mcts: Optional[Callable] = None, device=None, rank: Optional[int] = None,
                 world: Optional[int] = None):
        self.model, self.config, self.total = model, config, int(total)
        self.rank, self.world = _rank_world(group)
        if rank is not None or world is not None:  # a shard without a process group (single-GPU tests)
            if broadcaster is not None:
                raise ValueError("an explicit rank / world needs broadcaster=None")
            self.rank, self.world = int(rank or 0), int(world or 1)
        self.lo, self.hi = shard_bounds(self.total, self.world, self.rank)
        if self.hi <= self.lo:
            raise ValueError(f"rank {self.rank} of {self.world} owns no roots of {self.total}")
        # the same generator state on every rank: sharded draws are sliced from whole-batch draws
        self.np_random = np.random.RandomState(seed)
        self.broadcaster, self.src, self.group = broadcaster, src, group
        self.make_mcts = make_mcts or _default_mcts
        self.device = device
        self.model_index = -1
        if broadcaster is not None and self.rank == src and broadcaster.model_index < 0:
            # the source's weights are checkpoint 0, pulled by every rank before its first step
            # (last_model_index starts at -1: -1 // interval < 0 // interval)
            broadcaster.publish(0)

    @property
    def root_shard(self):
        return (self.lo, self.hi, self.total)

    def _sync(self) -> int:
        if self.broadcaster is not None:
            self.model_index = self.broadcaster.sync()
        return self.model_index

    def _publish(self, learner, t) -> None:
        """The learner's hook on the source rank: learner(model, t) -> trained-steps counter, or
        (counter, state_dict) with the learner's new weights, or None."""
        if learner is None or self.rank != self.src:
            return
        r = learner(self.model, t)
        if r is None or self.broadcaster is None:
            return
        trained, sd = (r if isinstance(r, tuple) else (r, None))
        self.broadcaster.publish(int(trained), sd)

    def _initial_inference(self, obs):
        with torch.no_grad(), torch.autocast("cuda", enabled=isinstance(obs, torch.Tensor) and obs.is_cuda):
            return self.model.initial_inference(obs)  # selfplay_worker.py:181-185


class SelfPlayShard(_Shard):
    """One rank of process-per-GPU self-play over `total_envs` environments: the rank-local
    replacement of DataWorker.run + RemoteDataWorker._update_model_before_step."""

    def __init__(self, model, config, total_envs: int, num_agents: int, *, decide: Optional[Callable] = None,
                 **kw):
        super().__init__(model, config, total_envs, **kw)
        self.num_agents = int(num_agents)
        self.decide = decide or _device_selfplay_decide

    def step(self, t: int, obs, legal, *, temperature: float = 1.0, sampled_tau: float = 1.0,
             greedy_epsilon: float = 0.0, eps_uniforms=None) -> StepRecord:
        """One environment step of this rank's environments.  `obs` / `legal` are the shard's rows;
        `eps_uniforms` (u_eps [N, total], u_cat [N, total]) are whole-batch draws, sliced here."""
        idx = self._sync()  # _update_model_before_step, selfplay_worker.py:176-177
        net_out = self._initial_inference(obs)
        mcts = self.make_mcts(self.config, self.np_random, self.root_shard)  # :187
        if eps_uniforms is not None:
            eps_uniforms = tuple(np.asarray(u)[:, self.lo:self.hi] for u in eps_uniforms)
        d = self.decide(mcts, self.model, net_out, self.num_agents, legal, temperature=temperature,
                        sampled_tau=sampled_tau, greedy_epsilon=greedy_epsilon, eps_uniforms=eps_uniforms,
                        device=self.device)
        return StepRecord(t, idx, self.lo, _to_np(d["actions"]).astype(np.int32), _to_np(d["prob_action"]),
                          _to_np(d["root_value"]).reshape(-1), _to_np(d["count_entropy"]),
                          _to_np(d["visit_entropy"]))

    def run(self, env: Callable, steps: int, *, learner: Optional[Callable] = None, eps_uniforms: Callable = None,
            **step_kw) -> List[StepRecord]:
        """`steps` environment steps.  env(t, lo, hi) -> (obs, legal) for environments [lo, hi);
        learner(model, t) on the source rank after step t -> the trained-steps counter to publish
        (or None); eps_uniforms(t) -> whole-batch (u_eps, u_cat) or None."""
        out = []
        for t in range(steps):
            obs, legal = env(t, self.lo, self.hi)
            out.append(self.step(t, obs, legal, eps_uniforms=None if eps_uniforms is None else eps_uniforms(t),
                                 **step_kw))
            self._publish(learner, t)
        return out


class ReanalyzeShard(_Shard):
    """One rank of process-per-GPU reanalysis: the policy targets of `_prepare_policy_re`
    (reanalyze_worker.py:212-366) for this rank's share of a batch's B·(K+1) roots, with the target
    weights refreshed by the target-model-interval rule (reanalyze_worker.py:663-669; build the
    broadcaster with checkpoint_interval = config.target_model_interval)."""

    def __init__(self, model, config, total_roots: int, *, decide: Optional[Callable] = None, **kw):
        super().__init__(model, config, total_roots, **kw)
        self.decide = decide or _device_reanalyze_decide

    def targets(self, obs, legal, policy_mask) -> dict:
        """obs / legal / policy_mask: this rank's rows [lo, hi) of the batch."""
        idx = self._sync()
        net_out = self._initial_inference(obs)
        mcts = self.make_mcts(self.config, self.np_random, self.root_shard)
        out = self.decide(mcts, self.model, net_out, legal, policy_mask, self.device)
        out = {k: _to_np(v) for k, v in out.items()}
        out["model_index"] = idx
        out["lo"] = self.lo
        return out
