"""Synthetic search inputs and a backend-agnostic search driver.

The inputs follow BASELINE.md §3 / SURVEY.md §8(d): per search and per simulation s, the network
outputs a search would receive, drawn once on the host so every backend (HIP product, reference
oracle, CPU port, pure-Python ptree) consumes byte-identical arrays:

    policy  = softmax(N(0,1))                   f32 [B, 1, A]     (beta = policy, tau = 1)
    reward  = 0.1 * N(0,1)                      f32 [B]
    value   = N(0,1)                            f32 [B]
    noise   = Dirichlet(0.3)                    f32 [B, 1, A]     (root only, eps = 0.25)
    seed    = rng.choice(256)                   tree seed, drawn after the noise like
                                                mcts_sampled.py:68,89

The root preprocessing (legal mask + 1e-4, renormalisation, beta = mix^(1/tau)) restates
mcts_sampled.py:64-100 in numpy float32/float64 exactly as the reference driver evaluates it.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

# MCTS knobs (core/config.py:26,75-91)
DEFAULTS = dict(
    pb_c_base=19652.0,
    pb_c_init=1.25,
    discount=0.997,
    delta_lb=0.01,
    dirichlet_alpha=0.3,
    exploration_fraction=0.25,
    rho=0.75,
    lam=0.8,
)

# SMAC map shapes: (n_agents, n_actions = 6 + n_enemies)  (smac_maps.py:17-133, StarCraft2_Env.py:268-270)
MAPS = {
    "matrix": (2, 3),
    "3m": (3, 9),
    "2s3z": (5, 11),
    "3s5z_vs_3s6z": (8, 15),
    "27m_vs_30m": (27, 36),
}
HIDDEN_PER_AGENT = 128  # config/smac/__init__.py:15


def softmax(x: np.ndarray) -> np.ndarray:
    e = np.exp(x - np.max(x, axis=-1, keepdims=True))
    return e / np.sum(e, axis=-1, keepdims=True)


@dataclass
class SearchInputs:
    B: int
    A: int
    S: int
    seed: int
    root_reward: np.ndarray
    root_value: np.ndarray
    root_policy: np.ndarray
    root_beta: np.ndarray
    root_noise: np.ndarray
    noise_eps: float
    reward: np.ndarray  # [S, B]
    value: np.ndarray  # [S, B]
    policy: np.ndarray  # [S, B, 1, A]
    beta: np.ndarray  # [S, B, 1, A]
    meta: dict = field(default_factory=dict)


def root_preprocess(logits, noises, legal, noise_eps, tau=1.0):
    """mcts_sampled.py:64-100 for one agent (agent_num = 1 trees)."""
    probs = np.exp(logits - np.max(logits, axis=-1, keepdims=True))
    probs = probs / np.sum(probs, axis=-1, keepdims=True)
    if legal is not None:
        probs = probs * legal
        probs = probs + legal * 1e-4
        probs = probs / np.sum(probs, axis=-1, keepdims=True)
        noises = noises * legal
        noises = noises + legal * 1e-4
        noises = noises / np.sum(noises, axis=-1, keepdims=True)
    beta = probs * (1 - noise_eps) + noises * noise_eps
    beta = beta ** (1 / tau)
    if legal is not None:
        beta = beta * legal
    beta = beta / np.sum(beta, axis=-1, keepdims=True)
    return probs.astype(np.float32), beta.astype(np.float32), noises.astype(np.float32)


def make_search_inputs(
    rng: np.random.Generator,
    B: int,
    A: int,
    S: int,
    noise_eps: float = 0.25,
    legal_zero_frac: float = 0.0,
    ties: bool = False,
    alpha: float = 0.3,
) -> SearchInputs:
    """One search's worth of synthetic network outputs."""
    if ties:
        logits = np.zeros((B, 1, A), np.float32)
        root_reward = np.zeros(B, np.float32)
        root_value = np.zeros(B, np.float32)
    else:
        logits = rng.standard_normal((B, 1, A)).astype(np.float32)
        root_reward = (0.1 * rng.standard_normal(B)).astype(np.float32)
        root_value = rng.standard_normal(B).astype(np.float32)
    noises = rng.dirichlet([alpha] * A, B).astype(np.float32).reshape(B, 1, A)
    legal = None
    if legal_zero_frac > 0:
        legal = (rng.random((B, 1, A)) >= legal_zero_frac).astype(np.float32)
        legal[:, :, 0] = 0.0  # action 0 (no-op of a dead unit) illegal
        legal[:, :, 1] = 1.0  # keep at least one legal action
    seed = int(rng.choice(256))
    policy, beta, noises = root_preprocess(logits, noises, legal, noise_eps)
    if ties:
        sim_policy = np.full((S, B, 1, A), 1.0 / A, np.float32)
        reward = np.zeros((S, B), np.float32)
        value = np.zeros((S, B), np.float32)
    else:
        sim_policy = softmax(rng.standard_normal((S, B, 1, A))).astype(np.float32)
        reward = (0.1 * rng.standard_normal((S, B))).astype(np.float32)
        value = rng.standard_normal((S, B)).astype(np.float32)
    sim_beta = sim_policy.copy()
    return SearchInputs(
        B=B,
        A=A,
        S=S,
        seed=seed,
        root_reward=root_reward,
        root_value=root_value,
        root_policy=policy,
        root_beta=beta,
        root_noise=noises,
        noise_eps=float(noise_eps),
        reward=reward,
        value=value,
        policy=sim_policy,
        beta=sim_beta,
        meta=dict(legal_zero_frac=legal_zero_frac, ties=ties),
    )


def make_deep_window_inputs(rng: np.random.Generator, B: int, S: int, A: int = 2, step: float = 0.2) -> SearchInputs:
    """Inputs whose searches grow one deep path with a tie at its bottom (round 6, the LDS window of
    engine words).  Every expansion draws both of A = 2 actions (beta uniform, K large) with priors
    of ~1e-8, so two unvisited children tie (their prior scores differ by less than the 1e-6 of
    select_child, cnode.cpp:355-370); rewards rising with the simulation make the visited child's
    value score the larger one, so each selection walks down the visited chain and draws one word
    for each level (cnode.cpp:373-377), the tie at the bottom included.  At K = 64 an expansion takes
    128 words, and at S = 190 the path passes ~130 levels: the selection's and the next expansion's
    words run past a launch's 256-word LDS window (k_tree's reads from the stream in HBM)."""
    logits = np.zeros((B, 1, A), np.float32)
    noises = rng.dirichlet([0.3] * A, B).astype(np.float32).reshape(B, 1, A)
    seed = int(rng.choice(256))
    policy, beta, noises = root_preprocess(logits, noises, None, 0.0)
    sim_policy = np.full((S, B, 1, A), 1e-8, np.float32)
    sim_beta = np.full((S, B, 1, A), 1.0 / A, np.float32)
    reward = np.tile((1.0 + step * np.arange(S, dtype=np.float32))[:, None], (1, B)).astype(np.float32)
    value = np.zeros((S, B), np.float32)
    return SearchInputs(B=B, A=A, S=S, seed=seed, root_reward=np.zeros(B, np.float32),
                        root_value=np.zeros(B, np.float32), root_policy=policy, root_beta=beta, root_noise=noises,
                        noise_eps=0.0, reward=reward, value=value, policy=sim_policy, beta=sim_beta,
                        meta=dict(deep_window=True, step=step))


def run_search(tb, inp: SearchInputs, K: int, knobs: dict | None = None, record: bool = True,
               per_sim: bool = True):
    """Drive a Tree_batch-compatible object through one full search (mcts_sampled.py:89-191
    minus the network), returning every selection and the final readbacks (`record`), plus the
    root values and marginal visit counts after every simulation (`per_sim`).

    `tb` needs the cytree.Tree_batch methods (prepare, batch_selection,
    batch_expansion_and_backup, get_roots_*).
    """
    k = dict(DEFAULTS)
    if knobs:
        k.update(knobs)
    c2, c1, g = k["pb_c_base"], k["pb_c_init"], k["discount"]
    tb.prepare(inp.root_reward, inp.root_value, inp.root_policy, inp.root_beta, K, inp.noise_eps, inp.root_noise)
    S, B = inp.S, inp.B
    sel_idx = np.zeros((S, B), np.int32)
    sel_act = np.zeros((S, B), np.int32)
    root_values = np.zeros((S, B), np.float32) if per_sim else None
    marginal = np.zeros((S, B, inp.A), np.int32) if per_sim else None
    for s in range(S):
        ix, iy, act = tb.batch_selection(c2, c1, g)
        if record:
            sel_idx[s] = np.asarray(ix, np.int32)
            sel_act[s] = np.asarray(act, np.int32).reshape(B, -1)[:, 0]
            assert list(iy) == list(range(B))
        tb.batch_expansion_and_backup(s + 1, g, K, inp.reward[s], inp.value[s], inp.policy[s], inp.beta[s])
        if record and per_sim:
            root_values[s] = tb.get_roots_values()
            marginal[s] = tb.get_roots_marginal_visit_count().reshape(B, -1)[:, : inp.A]
    out = dict(sel_idx=sel_idx, sel_act=sel_act)
    if per_sim:
        out.update(root_values_per_sim=root_values, marginal_per_sim=marginal)
    if record:
        out.update(readbacks(tb, g))
    return out


def readbacks(tb, discount: float) -> dict:
    """All final readbacks of mcts_sampled.py:176-191, padded per root to the max degree."""
    B = len(tb.get_roots_values())
    res = dict(
        root_values=tb.get_roots_values(),
        marginal_visit_count=tb.get_roots_marginal_visit_count(),
        marginal_priors=tb.get_roots_marginal_priors(),
    )
    lists = dict(
        actions=tb.get_roots_sampled_actions(),
        visit_count=tb.get_roots_sampled_visit_count(),
        pred_probs=tb.get_roots_sampled_pred_probs(),
        beta=tb.get_roots_sampled_beta(),
        beta_hat=tb.get_roots_sampled_beta_hat(),
        priors=tb.get_roots_sampled_priors(),
        imp_ratio=tb.get_roots_sampled_imp_ratio(),
        pred_values=tb.get_roots_sampled_pred_values(),
        mcts_values=tb.get_roots_sampled_mcts_values(),
        rewards=tb.get_roots_sampled_rewards(),
        qvalues=tb.get_roots_sampled_qvalues(discount),
    )
    deg = np.array([len(x) for x in lists["visit_count"]], np.int32)
    W = max(1, int(deg.max()) if B else 1)
    res["degree"] = deg
    for name, lst in lists.items():
        if name == "actions":
            arr = np.zeros((B, W), np.int32)
            for i, a in enumerate(lst):
                arr[i, : len(a)] = np.asarray(a).reshape(len(a), -1)[:, 0]
        else:
            arr = np.zeros((B, W), np.int32 if name == "visit_count" else np.float32)
            for i, a in enumerate(lst):
                arr[i, : len(a)] = a
        res["sampled_" + name] = arr
    return res


def inputs_digest(inp: SearchInputs) -> str:
    """SHA-256 over every input array of a search (shape, dtype and bytes, in a fixed order) and the
    tree seed: fixtures that regenerate their inputs from a seed check it first, so a change in
    numpy's generators cannot pass unnoticed."""
    import hashlib

    h = hashlib.sha256()
    h.update(np.int64([inp.B, inp.A, inp.S, inp.seed]).tobytes())
    h.update(np.float64([inp.noise_eps]).tobytes())
    for a in (inp.root_reward, inp.root_value, inp.root_policy, inp.root_beta, inp.root_noise, inp.reward, inp.value,
              inp.policy, inp.beta):
        a = np.ascontiguousarray(a)
        h.update(str((a.shape, a.dtype.str)).encode())
        h.update(a.tobytes())
    return h.hexdigest()

