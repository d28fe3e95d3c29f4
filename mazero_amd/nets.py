"""Networks and search config used to drive the search in tests and in the full-loop benchmark.

These are not part of the hot path. The driver only needs the reference model interface
(core/model.py:45-79): representation / prediction / dynamics, plus the inverse transforms.
`MuZeroShapedNet` has that interface and the tensor shapes of the SMAC MAMuZeroNet
(config/smac/model.py:405-572), with its MLP head option (`reward_head_type = value_head_type =
'mlp'`):
- per-agent hidden state H = 128;
- the dynamics input [h_i, onehot(a_i), mix_i] → [128, 128] → H, with a residual;
- a reward MLP over [B, N·(H+A)];
- a value MLP over [B, N·H];
- a per-agent policy MLP H → 32 → A;
- value/reward supports [-5, 5] (config/smac/__init__.py:26-28).
The agent-mixing feature is a mean over agents, standing in for the reference's attention encoder.
Weights are random (no checkpoints are available offline).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F


@dataclass
class SearchConfig:
    """The BaseConfig attributes the sampled-MCTS driver reads (core/config.py:76-91, 247-255)."""

    action_space_size: int
    num_simulations: int = 50
    sampled_action_times: int = 1
    pb_c_base: float = 19652.0
    pb_c_init: float = 1.25
    discount: float = 0.997
    tree_value_stat_delta_lb: float = 0.01
    root_dirichlet_alpha: float = 0.3
    root_exploration_fraction: float = 0.25
    mcts_rho: float = 0.75
    mcts_lambda: float = 0.8


def _mlp(inp: int, hidden: List[int], out: int) -> nn.Sequential:
    """Linear → LayerNorm → ReLU per hidden layer, plain final Linear (config/smac/model.py:20-71)."""
    sizes = [inp] + list(hidden) + [out]
    layers = []
    for i in range(len(sizes) - 1):
        layers.append(nn.Linear(sizes[i], sizes[i + 1]))
        if i < len(sizes) - 2:
            layers += [nn.LayerNorm(sizes[i + 1]), nn.ReLU()]
    return nn.Sequential(*layers)


def inverse_support_transform(logits: torch.Tensor, lo: int, hi: int) -> torch.Tensor:
    """Categorical support → scalar: softmax, expectation over [lo, hi], then the inverse of
    h(x) = sign(x)(sqrt(|x|+1)-1) + 0.001x (core/config.py:430-499)."""
    p = torch.softmax(logits, dim=-1)
    support = torch.arange(lo, hi + 1, device=logits.device, dtype=torch.float32).expand(p.shape)
    x = torch.sum(support * p, dim=-1, keepdim=True)
    eps = 0.001
    sign = torch.ones(x.shape, dtype=torch.float32, device=x.device)
    sign[x < 0] = -1.0
    out = (((torch.sqrt(1 + 4 * eps * (torch.abs(x) + 1 + eps)) - 1) / (2 * eps)) ** 2 - 1)
    out = sign * out
    out[torch.isnan(out)] = 0.0
    out[torch.abs(out) < eps] = 0.0
    return out


class NetworkOutput:
    """core/model.py:14-19."""

    def __init__(self, hidden_state, reward, value, policy_logits):
        self.hidden_state, self.reward, self.value, self.policy_logits = hidden_state, reward, value, policy_logits


class MuZeroShapedNet(nn.Module):
    def __init__(self, num_agents: int, obs_size: int, action_space_size: int, hidden: int = 128,
                 dyn_layers=(128, 128), reward_layers=(32,), value_layers=(32,), policy_layers=(32,),
                 support=(-5, 5), float_policy: bool = False):
        super().__init__()
        N, A, H = num_agents, action_space_size, hidden
        self.num_agents, self.action_space_size, self.hidden = N, A, H
        self.support = support
        self.float_policy = float_policy  # cast policy logits to float32 (exercises the f32 glue)
        S = support[1] - support[0] + 1
        self.rep_norm = nn.LayerNorm(obs_size)
        self.rep = _mlp(obs_size, [128, 128], H)
        self.mix = nn.Linear(H + A, H)
        self.dyn = _mlp(H + A + H, list(dyn_layers), H)
        self.reward_head = _mlp(N * (H + A), list(reward_layers), S)
        self.value_head = _mlp(N * H, list(value_layers), S)
        self.policy_head = _mlp(H, list(policy_layers), A)

    # core/model.py:45-79 interface --------------------------------------------------------------
    def representation(self, obs: torch.Tensor) -> torch.Tensor:
        B = obs.shape[0]
        x = self.rep(self.rep_norm(obs.reshape(B * self.num_agents, -1)))
        return x.reshape(B, -1)

    def prediction(self, h: torch.Tensor):
        B = h.shape[0]
        value_logits = self.value_head(h)
        policy = self.policy_head(h.reshape(B * self.num_agents, self.hidden)).reshape(B, self.num_agents, -1)
        if self.float_policy:
            policy = policy.float()
        return policy, value_logits

    def dynamics(self, h: torch.Tensor, action: torch.Tensor):
        B, N = h.shape[0], self.num_agents
        hs = h.reshape(B, N, self.hidden)
        onehot = F.one_hot(action.long(), num_classes=self.action_space_size).to(hs.dtype)
        mixed = torch.relu(self.mix(torch.cat([hs, onehot], dim=2)))
        mixed = mixed.mean(dim=1, keepdim=True).expand(B, N, self.hidden)
        upd = self.dyn(torch.cat([hs, onehot.to(mixed.dtype), mixed], dim=2).reshape(B * N, -1)).reshape(B, N, -1)
        nxt = upd + hs
        reward_logits = self.reward_head(torch.cat([nxt, onehot.to(nxt.dtype)], dim=2).reshape(B, -1))
        return nxt.reshape(B, -1), reward_logits

    def inverse_value_transform(self, logits):
        return inverse_support_transform(logits, *self.support)

    def inverse_reward_transform(self, logits):
        return inverse_support_transform(logits, *self.support)

    def initial_inference(self, obs: torch.Tensor) -> NetworkOutput:
        """config/smac/model.py:542-560 (eval mode: numpy reward / value / logits)."""
        h = self.representation(obs)
        policy, value_logits = self.prediction(h)
        S = self.support[1] - self.support[0] + 1
        reward_logits = torch.zeros(obs.shape[0], S, device=obs.device)
        if not self.training:
            return NetworkOutput(h, self.inverse_reward_transform(reward_logits).detach().cpu().numpy(),
                                 self.inverse_value_transform(value_logits).detach().cpu().numpy(),
                                 policy.detach().cpu().numpy())
        return NetworkOutput(h, reward_logits, value_logits, policy)

    def recurrent_inference(self, h: torch.Tensor, action: torch.Tensor) -> NetworkOutput:
        """config/smac/model.py:562-572 (eval mode: numpy reward / value / logits)."""
        nxt, reward_logits = self.dynamics(h, action)
        policy, value_logits = self.prediction(nxt)
        if not self.training:
            return NetworkOutput(nxt, self.inverse_reward_transform(reward_logits).detach().cpu().numpy(),
                                 self.inverse_value_transform(value_logits).detach().cpu().numpy(),
                                 policy.detach().cpu().numpy())
        return NetworkOutput(nxt, reward_logits, value_logits, policy)


def make_net(num_agents: int, action_space_size: int, obs_size: int = 64, seed: int = 0, device=None,
             float_policy: bool = False) -> MuZeroShapedNet:
    torch.manual_seed(seed)
    net = MuZeroShapedNet(num_agents, obs_size, action_space_size, float_policy=float_policy)
    if device is not None:
        net = net.to(device)
    return net.eval()


def make_root_batch(net: MuZeroShapedNet, B: int, obs_size: int, seed: int, device, legal_zero_frac: float = 0.0):
    """Synthetic observations → initial_inference under autocast (selfplay_worker.py:181-185), and
    a legal-action mask [B, N, A] with about `legal_zero_frac` illegal actions (at least one legal)."""
    rng = np.random.default_rng(seed)
    obs = torch.from_numpy(rng.standard_normal((B, net.num_agents, obs_size)).astype(np.float32)).to(device)
    with torch.no_grad(), torch.autocast("cuda", enabled=obs.is_cuda):
        out = net.initial_inference(obs)
    legal = (rng.random((B, net.num_agents, net.action_space_size)) >= legal_zero_frac).astype(np.int64)
    legal[..., 0] = np.where(legal.sum(-1) == 0, 1, legal[..., 0])
    return out, legal
