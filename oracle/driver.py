"""ORACLE (test infrastructure only): CPU restatement of the reference search driver
`SampledMCTS.batch_search` (core/mcts/tree_search/mcts_sampled.py:34-200).

Only tests/ and __graft_entry__.smoke() use this module, as the checker of the device-resident
driver mazero_amd.mcts_sampled. It follows the reference step by step:
- numpy glue on the host;
- a Python-list hidden-state pool with `torch.vstack` gathers;
- the model's eval-mode `recurrent_inference`, which returns numpy;
- three tree calls per simulation on an oracle tree library: the reference ctree built in place
  (oracle/_ref/libmzref.so) or the CPU port (oracle/_build/libmzport.so), through the
  `Tree_batch` ctypes shim.

Parity status: pinned.  oracle/gen_driver_golden.py runs the reference driver module itself
(imported in the build container) and records six searches (tests/golden/driver_*.npz); this
restatement reproduces every tree call, the network's inputs, the SearchOutput and the generator
state of each, on the CPU port and on the reference ctree (tests/test_driver.py).  The module is
not imported here: its package imports `ray` (core/game.py:5 via core/config.py:10), which this
image does not have, and nothing of the reference travels to the GPU box.
"""
from __future__ import annotations

import numpy as np
import torch


def _np(x):
    if isinstance(x, torch.Tensor):
        return x.detach().cpu().numpy()
    return np.asarray(x)


class OracleSampledMCTS:
    def __init__(self, config, np_random, tree_lib, record: bool = False, root_shard=None):
        self.config = config
        self.np_random = np_random
        self.lib = tree_lib
        self.record = record
        self.trace = []  # per simulation: the tree inputs (for replay / diagnosis)
        # (lo, hi, total): rows [lo, hi) of a batch sharded over ranks -- per-root draws are made
        # for the whole batch and sliced, trees seeded with their global index (needs the CPU port:
        # the reference ctree has no root offset)
        self.root_shard = root_shard

    def _rows(self, draw, B):
        if self.root_shard is None:
            return draw(B)
        lo, hi, total = self.root_shard
        assert hi - lo == B
        return draw(total)[lo:hi]

    def draw_root_uniforms(self, B):
        return np.asarray(self._rows(lambda n: self.np_random.random(n), B), dtype=np.float64)

    def batch_search(self, model, network_output, current_agent_idx, factor, true_num_agents,
                     legal_actions_lst=None, device=None, add_noise=False, sampled_tau=1.0):
        from mazero_amd.cytree import Tree_batch

        cfg = self.config
        c2, c1, disc = cfg.pb_c_base, cfg.pb_c_init, cfg.discount
        rho, lam = cfg.mcts_rho, cfg.mcts_lambda
        alpha, eps = cfg.root_dirichlet_alpha, cfg.root_exploration_fraction
        A, K = cfg.action_space_size, cfg.sampled_action_times
        B = network_output.hidden_state.shape[0]

        # mcts_sampled.py:57-83
        hs0 = network_output.hidden_state
        rewards = _np(network_output.reward)
        values = _np(network_output.value)
        logits = _np(network_output.policy_logits)[:, current_agent_idx, :].reshape(B, 1, A)
        probs = np.exp(logits - np.max(logits, axis=-1, keepdims=True))
        probs = probs / np.sum(probs, axis=-1, keepdims=True)
        noises = self._rows(lambda n: self.np_random.dirichlet([alpha] * A, n), B).astype(np.float32).reshape(B, 1, A)
        if not add_noise:
            eps = 0.0
        if legal_actions_lst is not None:
            legal = legal_actions_lst[:, current_agent_idx, :].reshape(B, 1, A)
            probs *= legal
            probs += legal * 1e-4
            probs = probs / np.sum(probs, axis=-1, keepdims=True)
            noises *= legal
            noises += legal * 1e-4
            noises = noises / np.sum(noises, axis=-1, keepdims=True)

        # mcts_sampled.py:86-106
        pool = [hs0]
        trees = Tree_batch(B, 1, A, K, cfg.num_simulations, cfg.tree_value_stat_delta_lb,
                           self.np_random.choice(256), rho, lam, lib=self.lib,
                           root_offset=0 if self.root_shard is None else self.root_shard[0])
        beta = probs * (1 - eps) + noises * eps
        beta = beta ** (1 / sampled_tau)
        if legal_actions_lst is not None:
            beta *= legal
        beta = beta / np.sum(beta, axis=-1, keepdims=True)
        trees.prepare(rewards.reshape(B).astype(np.float32), values.reshape(B).astype(np.float32),
                      probs.astype(np.float32), beta.astype(np.float32), K, eps, noises)

        # mcts_sampled.py:111-172
        with torch.no_grad():
            model.eval()
            for s in range(cfg.num_simulations):
                joint = np.zeros((B, true_num_agents), dtype=np.int32)
                if factor is not None:
                    for k in range(current_agent_idx):
                        joint[:, k] = factor[:, k]
                ix, iy, acts = trees.batch_selection(c2, c1, disc)
                joint[:, current_agent_idx] = acts.squeeze()
                leaf = torch.vstack([pool[x][y] for x, y in zip(ix, iy)])
                with torch.autocast("cuda", enabled=leaf.is_cuda):
                    pred_logits, _ = model.prediction(leaf)
                pred_logits = _np(pred_logits)
                for k in range(current_agent_idx + 1, true_num_agents):
                    joint[:, k] = np.argmax(pred_logits[:, k, :], axis=-1)
                joint_t = torch.from_numpy(joint).to(leaf.device)
                with torch.autocast("cuda", enabled=leaf.is_cuda):
                    out = model.recurrent_inference(leaf, joint_t)
                lg = out.policy_logits[:, current_agent_idx, :].reshape(B, 1, A)
                p = np.exp(lg - np.max(lg, axis=-1, keepdims=True))
                p = p / np.sum(p, axis=-1, keepdims=True)
                bt = p ** (1 / sampled_tau)
                bt = bt / np.sum(bt, axis=-1, keepdims=True)
                pool.append(out.hidden_state)
                r = out.reward.reshape(B).astype(np.float32)
                v = out.value.reshape(B).astype(np.float32)
                if self.record:
                    self.trace.append(dict(idx=np.asarray(ix, np.int32), act=np.asarray(acts).reshape(B).copy(),
                                           joint=joint.copy(), reward=r, value=v, probs=p.astype(np.float32),
                                           beta=bt.astype(np.float32)))
                trees.batch_expansion_and_backup(s + 1, disc, K, r, v, p.astype(np.float32), bt.astype(np.float32))

        # mcts_sampled.py:176-200
        return dict(
            value=trees.get_roots_values(),
            marginal_visit_count=trees.get_roots_marginal_visit_count(),
            marginal_priors=trees.get_roots_marginal_priors(),
            sampled_actions=trees.get_roots_sampled_actions(),
            sampled_visit_count=trees.get_roots_sampled_visit_count(),
            sampled_pred_probs=trees.get_roots_sampled_pred_probs(),
            sampled_beta=trees.get_roots_sampled_beta(),
            sampled_beta_hat=trees.get_roots_sampled_beta_hat(),
            sampled_priors=trees.get_roots_sampled_priors(),
            sampled_imp_ratio=trees.get_roots_sampled_imp_ratio(),
            sampled_pred_values=trees.get_roots_sampled_pred_values(),
            sampled_mcts_values=trees.get_roots_sampled_mcts_values(),
            sampled_rewards=trees.get_roots_sampled_rewards(),
            sampled_qvalues=trees.get_roots_sampled_qvalues(disc),
        )
