"""ORACLE (test infrastructure only): CPU restatement of the reference's consumers of the search
output -- the checker of mazero_amd.consume and include/mzconsume.h.  Only tests/ use it.

- `select_action`      core/utils.py:289-316 (the reference's Python, numpy and scipy calls)
- `eps_greedy_given`   core/utils.py:319-334 with its two torch draws passed in: the reference
                       draws `torch.rand_like` (float32) and `Categorical(mask).sample()` from
                       torch's global CPU generator; here they are the uniforms u_eps (float32)
                       and u_cat (float64, inverse cdf of the mask weights)
- `selfplay_step`      core/selfplay_worker.py:189-293, the decisions of one environment step
- `reanalyze_policy`   core/reanalyze_worker.py:266-366, `_prepare_policy_re` after the initial
                       inference

Parity status: the np_random consumption is pinned against numpy's own Generator / RandomState
`choice` (tests/test_consume.py).  The epsilon-greedy decision is pinned to the reference itself:
tests/golden/eps_greedy_torch.npz holds core/utils.py's eps_greedy_action run root after root under
a seeded torch generator (oracle/gen_driver_golden.py), and mazero_amd.consume.torch_eps_uniforms
+ eps_greedy_given (and the device kernel) reproduce those actions.
"""
from __future__ import annotations

import numpy as np
from scipy.stats import entropy


def select_action(visit_counts, temperature=1, deterministic=True, np_random=None):
    """core/utils.py:289-316."""
    assert sum(visit_counts) > 0, "invalid input: num_simulation = 0!!!"
    action_probs = [visit_count_i ** (1 / temperature) for visit_count_i in visit_counts]
    total_count = sum(action_probs)
    action_probs = [x / total_count for x in action_probs]
    action_probs = np.array(action_probs)
    if deterministic:
        action_pos = np.argmax([v for v in visit_counts])
    else:
        rs = np.random if np_random is None else np_random
        action_pos = rs.choice(len(visit_counts), p=action_probs)
    count_entropy = entropy(action_probs, base=2)
    return action_pos, count_entropy


def categorical_given(weights, u):
    """Categorical(weights).sample() as the inverse cdf of the weights at u in [0, 1)."""
    w = np.asarray(weights, dtype=np.int64)
    tot = int(w.sum())
    c = np.cumsum(w)
    for a in range(w.shape[0]):
        if float(c[a]) / float(tot) > u:
            return a
    return w.shape[0] - 1


def eps_greedy_given(greedy_action, legal_action_mask, eps, u_eps, u_cat):
    """core/utils.py:319-334 with the draws given; torch compares the float32 draw with eps in
    float32 (a Python scalar does not promote a float32 tensor)."""
    if not (np.float32(u_eps) < np.float32(eps)):
        return int(greedy_action)
    if int(np.asarray(legal_action_mask).sum()) <= 0:
        return int(greedy_action)
    return categorical_given(legal_action_mask, u_cat)


def selfplay_step(mcts, model, network_output, true_num_agents, legal_actions_lst, temperature, sampled_tau,
                  greedy_epsilon, np_random, u_eps, u_cat, device=None, root_shard=None):
    """core/selfplay_worker.py:189-293 for the active envs of one step.  `mcts` is an oracle
    driver (oracle/driver.py) sharing `np_random`; u_eps / u_cat [N, B] replace the per-root
    torch draws."""
    N = true_num_agents
    B = legal_actions_lst.shape[0]
    A = legal_actions_lst.shape[2]
    temp_agent_actions = np.full((B, N), -1, dtype=np.int32)
    temp_entropies = np.zeros((B, N))
    outs = []
    for agent_idx in range(N):
        factor = temp_agent_actions[:, :agent_idx].copy() if agent_idx > 0 else None
        so = mcts.batch_search(model, network_output, agent_idx, factor, N, legal_actions_lst, device=device,
                               add_noise=True, sampled_tau=sampled_tau)
        outs.append(so)
        if root_shard is not None:  # the other ranks' roots draw before and after this shard's
            np_random.random(root_shard[0])
        for i in range(B):
            sampled_actions = so["sampled_actions"][i]
            sampled_visit_counts = so["sampled_visit_count"][i]
            single_agent_legal_actions = legal_actions_lst[i, agent_idx, :]
            if not sampled_actions.size:
                legal_indices = np.where(single_agent_legal_actions == 1)[0]
                agent_action = np_random.choice(legal_indices) if legal_indices.size > 0 else 0
                visit_entropy_per_agent = 0.0
            else:
                action_pos, visit_entropy_per_agent = select_action(sampled_visit_counts, temperature=temperature,
                                                                    deterministic=False, np_random=np_random)
                agent_action = sampled_actions[action_pos, 0]
            agent_action = eps_greedy_given(agent_action, single_agent_legal_actions, greedy_epsilon,
                                            u_eps[agent_idx][i], u_cat[agent_idx][i])
            temp_agent_actions[i, agent_idx] = agent_action
            temp_entropies[i][agent_idx] = visit_entropy_per_agent
        if root_shard is not None:
            np_random.random(root_shard[2] - root_shard[1])
    prob = np.zeros(B)
    visit_entropy = np.zeros((B, N))
    for i in range(B):
        action = temp_agent_actions[i, :]
        prob_action = 1.0
        for ag_idx in range(N):
            ag_visits = outs[ag_idx]["marginal_visit_count"][i, 0, :]
            curr = 0.0
            if np.sum(ag_visits) > 0:
                prob_action_dist = ag_visits / np.sum(ag_visits)
                prob_action *= prob_action_dist[action[ag_idx]]
                curr = -np.sum(prob_action_dist * np.log(prob_action_dist + 1e-9))
            elif A > 0:
                prob_action *= (1.0 / A)
            visit_entropy[i, ag_idx] = curr
        prob[i] = prob_action
    return dict(actions=temp_agent_actions, count_entropy=temp_entropies, prob_action=prob,
                visit_entropy=visit_entropy, root_value=outs[0]["value"])


def reanalyze_policy(mcts, model, network_output, legal_actions_lst, policy_mask, np_random, device=None):
    """core/reanalyze_worker.py:266-366 (from the reshaped legal actions on)."""
    B_prime, N, A = legal_actions_lst.shape
    actions = np.full((B_prime, N), -1, dtype=np.int32)
    probs = np.zeros((B_prime, 1), dtype=np.float32)
    agent_policy_dist = [[None for _ in range(N)] for _ in range(B_prime)]
    current_actions = np.zeros_like(actions)
    agent0_root_value = None
    for agent_idx in range(N):
        factor = current_actions[:, :agent_idx].copy() if agent_idx > 0 else None
        sr = mcts.batch_search(model, network_output, agent_idx, factor, N, legal_actions_lst, device=device,
                               add_noise=True, sampled_tau=1.0)
        if agent_idx == 0:
            agent0_root_value = sr["value"].reshape(B_prime, 1)
        for s_idx in range(B_prime):
            sampled_actions = sr["sampled_actions"][s_idx]
            sampled_visits = sr["sampled_visit_count"][s_idx]
            marginal_visits = sr["marginal_visit_count"][s_idx, 0, :]
            legal_actions = legal_actions_lst[s_idx, agent_idx, :]
            agent_action = 0
            if sampled_actions.size > 0 and np.sum(sampled_visits) > 0:
                if np.sum(marginal_visits) > 0:
                    agent_action = np.argmax(marginal_visits * legal_actions)
                else:
                    legal_indices = np.where(legal_actions == 1)[0]
                    if legal_indices.size > 0:
                        agent_action = np_random.choice(legal_indices)
            else:
                legal_indices = np.where(legal_actions == 1)[0]
                if legal_indices.size > 0:
                    agent_action = np_random.choice(legal_indices)
            current_actions[s_idx, agent_idx] = agent_action
            if np.sum(marginal_visits) > 0:
                agent_policy_dist[s_idx][agent_idx] = marginal_visits / np.sum(marginal_visits)
            else:
                num_legal = np.sum(legal_actions)
                if num_legal > 0:
                    agent_policy_dist[s_idx][agent_idx] = legal_actions / num_legal
                else:
                    dummy = np.zeros(A)
                    if A > 0:
                        dummy[0] = 1.0
                    agent_policy_dist[s_idx][agent_idx] = dummy
    actions = current_actions
    for s_idx in range(B_prime):
        prob_prod = 1.0
        for k in range(N):
            prob_prod *= agent_policy_dist[s_idx][k][actions[s_idx, k]]
        probs[s_idx, 0] = prob_prod
    value = network_output.value
    value = value.detach().cpu().numpy() if hasattr(value, "detach") else np.asarray(value)
    return dict(sampled_actions=actions.reshape(B_prime, 1, N), sampled_policies=probs,
                sampled_imp_ratio=np.ones((B_prime, 1), dtype=np.float32),
                sampled_masks=np.asarray(policy_mask).reshape(B_prime, 1).astype(np.bool_),
                sampled_qvalues=agent0_root_value, root_mcts_values=agent0_root_value,
                root_pred_values=value.reshape(B_prime, 1) if value.ndim == 1 else value)
