"""On-device consumers of the search output (C-ABI include/mzconsume.h).

After every agent's search the reference workers copy each root's result lists to the host and
decide per root in Python:
- self-play (core/selfplay_worker.py:189-293): `select_action` over the root children's visit
  counts with `np_random` (core/utils.py:289-316), `eps_greedy_action` with torch's generator
  (core/utils.py:319-334), then the stored policy probability and visit entropy;
- reanalyze (core/reanalyze_worker.py:275-366, `_prepare_policy_re`): the action
  argmax(marginal visits * legal), and the product of the agents' marginal visit distributions.

Here the same decisions are made on the device from `DeviceSearchOutput`, in the tree handle's
stream; the next agent's search takes the actions as a device tensor, so an environment step
needs no device-to-host copy of the search lists.

Random draws keep the reference's host generator and order where it has one: each root's
`np_random.choice(n, p=probs)` draws one double (`np_random.random()`), so one
`np_random.random(B)` per agent, in root order, reproduces them (tests/test_consume.py checks this
against numpy's own `choice`).  The epsilon-greedy draws come from torch's global generator in the
reference, one root at a time on the CPU; here they are device uniforms (the same distribution,
not the same stream), or caller-supplied ones.
"""
from __future__ import annotations

import ctypes as C
from typing import List, NamedTuple, Optional, Tuple

import numpy as np
import torch

from ._capi import MZ_MARGINAL_ARGMAX, MZ_MARGINAL_GIVEN, check
from .mcts_sampled import DeviceSearchOutput


def _p(t: Optional[torch.Tensor]):
    return None if t is None else C.c_void_p(t.data_ptr())


def _dev_i32(x, dev) -> torch.Tensor:
    if isinstance(x, torch.Tensor):
        return x.to(device=dev, dtype=torch.int32).contiguous()
    a = np.asarray(x)
    if a.dtype.kind == "f" and not np.array_equal(a, np.round(a)):
        raise ValueError("legal-action masks must hold integer weights")
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.int32)).to(dev)


def _root_uniforms(mcts, B: int) -> np.ndarray:
    """select_action's np_random.choice doubles for B roots (a sharded driver draws the whole
    batch's and keeps its own, mcts_sampled.SampledMCTS.draw_root_uniforms)."""
    fn = getattr(mcts, "draw_root_uniforms", None)
    if fn is not None:
        return fn(B)
    return np.asarray(mcts.np_random.random(B), dtype=np.float64)


def _tree(out: DeviceSearchOutput):
    if out.tree is None:
        raise ValueError("DeviceSearchOutput without its tree handle (use SampledMCTS.batch_search_device)")
    tb = out.tree
    tb._sync_stream()
    return tb


def select_actions(out: DeviceSearchOutput, uniforms: Optional[torch.Tensor], temperature: float = 1.0,
                   deterministic: bool = False) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """select_action (core/utils.py:289-316) at every root -> (pos, agent-0 action, count
    entropy), int32 / int32 / float64 [B] device tensors.  `uniforms`: float64 [B], the doubles
    `np_random.choice` would draw, in root order (unused when deterministic)."""
    tb = _tree(out)
    visits = out.sampled["visit_count"].contiguous()
    actions = out.sampled["actions"].contiguous()
    B, width = visits.shape
    dev = visits.device
    if not deterministic:
        uniforms = torch.as_tensor(uniforms, dtype=torch.float64).to(dev).contiguous()
        if uniforms.shape != (B,):
            raise ValueError(f"uniforms must have shape ({B},)")
    pos = torch.empty(B, dtype=torch.int32, device=dev)
    act = torch.empty(B, dtype=torch.int32, device=dev)
    ent = torch.empty(B, dtype=torch.float64, device=dev)
    lib = tb._lib
    check(lib, lib.mz_select_actions(tb._h, _p(out.degrees), _p(visits), _p(actions), int(width), float(temperature),
                                     int(bool(deterministic)), None if deterministic else _p(uniforms), _p(pos),
                                     _p(act), _p(ent)), "select_actions")
    return pos, act, ent


def eps_greedy(out: DeviceSearchOutput, action: torch.Tensor, legal: torch.Tensor, eps: float,
               u_eps: torch.Tensor, u_cat: torch.Tensor) -> torch.Tensor:
    """eps_greedy_action (core/utils.py:319-334) at every root, in place on `action` (int32 [B]).
    legal: int32 [B, A] (a view with unit column stride); u_eps float32 [B]; u_cat float64 [B]."""
    tb = _tree(out)
    if legal.stride(-1) != 1:
        legal = legal.contiguous()
    lib = tb._lib
    check(lib, lib.mz_eps_greedy(tb._h, _p(legal), int(legal.stride(0)), float(eps), _p(u_eps.contiguous()),
                                 _p(u_cat.contiguous()), _p(action)), "eps_greedy")
    return action


def marginal_policy(out: DeviceSearchOutput, mode: int, action: torch.Tensor, prob: torch.Tensor,
                    legal: Optional[torch.Tensor] = None, entropy: Optional[torch.Tensor] = None):
    """One agent's marginal visit distribution at each root (include/mzconsume.h
    mz_marginal_policy): ARGMAX picks `action`, both modes multiply `prob` (float64 [B]) by the
    distribution at the action and write the visit entropy."""
    tb = _tree(out)
    marginal = out.marginal_visit_count[:, 0, :]
    if marginal.stride(-1) != 1:
        marginal = marginal.contiguous()
    if legal is not None and legal.stride(-1) != 1:
        legal = legal.contiguous()
    lib = tb._lib
    check(lib, lib.mz_marginal_policy(tb._h, _p(marginal), int(marginal.stride(0)), _p(legal),
                                      int(legal.stride(0)) if legal is not None else 0, int(mode), _p(action),
                                      _p(prob), _p(entropy)), "marginal_policy")


class SelfPlayDecisions(NamedTuple):
    """One environment step's decisions for every active env (selfplay_worker.py:189-293)."""

    actions: torch.Tensor          # int32 [B, N]: agent_actions
    count_entropy: torch.Tensor    # float64 [B, N]: select_action's entropy (temp_entropies)
    prob_action: torch.Tensor      # float64 [B]: sampled_policy, prod_k marginal_k[action_k]
    visit_entropy: torch.Tensor    # float64 [B, N]: agent_entropies
    root_value: torch.Tensor       # float32 [B]: agent 0's search value
    outputs: List[DeviceSearchOutput]


def torch_eps_uniforms(legal_rows) -> Tuple[np.ndarray, np.ndarray]:
    """The epsilon-greedy draws of eps_greedy_action (core/utils.py:319-334) from torch's global CPU
    generator, exactly as the reference's worker loop makes them: root after root, one
    `torch.rand_like` (float32) then one `Categorical(mask).sample()`.  Returned as the uniforms the
    device kernel (mz_eps_greedy) takes: u_eps is the float32 draw itself; u_cat is the lower edge of
    the sampled action's interval of the mask's cumulative weights, c[a-1] / total in float64, which
    the kernel's inverse cdf maps back to exactly that action (a positive-weight action: the sample's
    own).  legal_rows: [B, A] (the agent's rows, the reference's array dtype).  A host loop over the
    roots, as the reference's: for replaying the reference's torch stream bit for bit."""
    rows = np.asarray(legal_rows)
    B = rows.shape[0]
    u_eps = np.empty(B, np.float32)
    u_cat = np.empty(B, np.float64)
    for i in range(B):
        mask = torch.from_numpy(np.ascontiguousarray(rows[i]))
        u_eps[i] = float(torch.rand_like(mask[..., 0].float()))
        a = int(torch.distributions.Categorical(mask).sample())
        c = np.cumsum(rows[i].astype(np.int64))
        u_cat[i] = 0.0 if a == 0 else float(c[a - 1]) / float(c[-1])
    return u_eps, u_cat


def selfplay_decisions(mcts, model, network_output, true_num_agents: int, legal_actions_lst, *,
                       temperature: float, sampled_tau: float = 1.0, greedy_epsilon: float = 0.0,
                       eps_uniforms: Optional[Tuple] = None, device=None) -> SelfPlayDecisions:
    """The self-play agent loop of selfplay_worker.py:189-293 on the device: one search per
    agent (`mcts.batch_search_device`, later agents conditioned on the earlier agents' device
    actions), select_action + epsilon-greedy per root, then the recorded policy probability.

    `mcts.np_random` is consumed exactly as the reference consumes `self.np_random`.
    eps_uniforms: optional (u_eps float32 [N, B], u_cat float64 [N, B]); drawn with torch.rand on
    the device when omitted (same distribution, not the reference's stream); "torch": drawn per agent
    from torch's global CPU generator as the reference draws them (torch_eps_uniforms), so the
    actions replay the reference's bit for bit (a host loop over the roots)."""
    N = int(true_num_agents)
    hidden = network_output.hidden_state
    dev = hidden.device
    B = hidden.shape[0]
    legal = _dev_i32(legal_actions_lst, dev) if legal_actions_lst is not None else \
        torch.ones(B, N, mcts.config.action_space_size, dtype=torch.int32, device=dev)
    torch_stream = isinstance(eps_uniforms, str)
    if torch_stream:
        if eps_uniforms != "torch":
            raise ValueError(f"eps_uniforms: {eps_uniforms!r} (a tuple of arrays or 'torch')")
        legal_host = np.ones((B, N, mcts.config.action_space_size), np.int64) if legal_actions_lst is None \
            else (legal_actions_lst.cpu().numpy() if isinstance(legal_actions_lst, torch.Tensor)
                  else np.asarray(legal_actions_lst))
        u_eps = torch.empty(N, B, dtype=torch.float32, device=dev)
        u_cat = torch.empty(N, B, dtype=torch.float64, device=dev)
    elif eps_uniforms is None:
        u_eps = torch.rand(N, B, dtype=torch.float32, device=dev)
        u_cat = torch.rand(N, B, dtype=torch.float64, device=dev)
    else:
        u_eps = torch.as_tensor(eps_uniforms[0], dtype=torch.float32).to(dev)
        u_cat = torch.as_tensor(eps_uniforms[1], dtype=torch.float64).to(dev)
    actions = torch.full((B, N), -1, dtype=torch.int32, device=dev)
    count_ent = torch.zeros(B, N, dtype=torch.float64, device=dev)
    outs = []
    for k in range(N):
        factor = actions[:, :k] if k > 0 else None
        out = mcts.batch_search_device(model, network_output, k, factor, N, legal_actions_lst, device,
                                       add_noise=True, sampled_tau=sampled_tau)
        outs.append(out)
        # select_action's np_random.choice: one double per root, in root order (:240-247)
        u = torch.from_numpy(_root_uniforms(mcts, B)).to(dev)
        if torch_stream:  # the agent's torch draws, root by root (:250-254)
            ue, uc = torch_eps_uniforms(legal_host[:, k, :])
            u_eps[k].copy_(torch.from_numpy(ue))
            u_cat[k].copy_(torch.from_numpy(uc))
        with torch.cuda.device(dev):
            _, act, ent = select_actions(out, u, temperature, deterministic=False)
            eps_greedy(out, act, legal[:, k, :], greedy_epsilon, u_eps[k], u_cat[k])  # :250-254
        actions[:, k] = act
        count_ent[:, k] = ent
    prob = torch.ones(B, dtype=torch.float64, device=dev)
    vent = torch.zeros(B, N, dtype=torch.float64, device=dev)
    with torch.cuda.device(dev):
        for k in range(N):  # :278-290
            a = actions[:, k].contiguous()
            e = torch.empty(B, dtype=torch.float64, device=dev)
            marginal_policy(outs[k], MZ_MARGINAL_GIVEN, a, prob, entropy=e)
            vent[:, k] = e
    return SelfPlayDecisions(actions, count_ent, prob, vent, outs[0].value, outs)


class ReanalyzePolicy(NamedTuple):
    """The targets of reanalyze_worker.py:345-366 (device tensors)."""

    sampled_actions: torch.Tensor   # int32 [B', 1, N]
    sampled_policies: torch.Tensor  # float32 [B', 1]
    sampled_imp_ratio: torch.Tensor  # float32 [B', 1] (ones)
    sampled_masks: torch.Tensor     # bool [B', 1]
    sampled_qvalues: torch.Tensor   # float32 [B', 1]: agent 0's root value
    root_mcts_values: torch.Tensor  # float32 [B', 1]
    root_pred_values: torch.Tensor  # network_output.value as [B', 1]


def reanalyze_policy_targets(mcts, model, network_output, legal_actions_lst, policy_mask, device=None
                             ) -> ReanalyzePolicy:
    """`_prepare_policy_re` after the initial inference (reanalyze_worker.py:266-366): per agent
    a search (add_noise=True, sampled_tau=1.0) conditioned on the earlier agents' chosen actions,
    action = argmax(marginal visits * legal), and the product of the agents' marginal
    distributions at the chosen actions.  Requires num_simulations >= 1: with no visits the
    reference draws the action from np_random instead."""
    if mcts.config.num_simulations < 1:
        raise ValueError("reanalyze_policy_targets needs num_simulations >= 1")
    hidden = network_output.hidden_state
    dev = hidden.device
    B = hidden.shape[0]
    legal_np = np.asarray(legal_actions_lst)
    N = legal_np.shape[1]
    legal = _dev_i32(legal_np, dev)
    current = torch.zeros(B, N, dtype=torch.int32, device=dev)
    prob = torch.ones(B, dtype=torch.float64, device=dev)
    value0 = None
    for k in range(N):
        factor = current[:, :k] if k > 0 else None
        out = mcts.batch_search_device(model, network_output, k, factor, N, legal_np, device, add_noise=True,
                                       sampled_tau=1.0)
        if k == 0:
            value0 = out.value.reshape(B, 1)
        a = torch.empty(B, dtype=torch.int32, device=dev)
        with torch.cuda.device(dev):
            marginal_policy(out, MZ_MARGINAL_ARGMAX, a, prob, legal=legal[:, k, :])
        current[:, k] = a
    masks = torch.as_tensor(np.asarray(policy_mask).reshape(B, 1).astype(np.bool_)).to(dev)
    pv = network_output.value
    pv = torch.as_tensor(pv).to(dev)
    if pv.ndim == 1:
        pv = pv.reshape(B, 1)
    return ReanalyzePolicy(current.reshape(B, 1, N), prob.to(torch.float32).reshape(B, 1),
                           torch.ones(B, 1, dtype=torch.float32, device=dev), masks, value0, value0, pv)
