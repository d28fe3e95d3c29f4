"""ORACLE — TEST INFRASTRUCTURE ONLY.  Records tests/golden/driver_<name>.npz: searches run by the
REFERENCE driver itself, `core.mcts.tree_search.mcts_sampled.SampledMCTS.batch_search`
(/root/reference/core/mcts/tree_search/mcts_sampled.py:34-200), imported from /root/reference.

Build container only (it reads /root/reference and needs oracle/_ref/libmzref.so, the reference
ctree built in place by oracle/Makefile).  Nothing here travels to or runs on the GPU box: the
box only reads the .npz files this script writes.

How the reference module is made importable:
- `ray`, `gymnasium`, `cv2` are not installed.  The reference package imports them at module
  level only (core/game.py:5, core/utils.py:2-3: decorators-free imports plus `gym.Wrapper`
  base classes); `batch_search` calls none of them.  Empty stand-in modules are registered in
  sys.modules for the import alone;
- the Cython binding `core.mcts.ctree.ctree_sampled.cytree` is registered as a module whose
  `Tree_batch` is mazero_amd.cytree.Tree_batch (same methods and return types as cytree.pyx:7-247)
  bound to libmzref.so (the reference's own cnode.cpp + utils.cpp), and records every call;
- no bytecode is written under /root/reference (sys.dont_write_bytecode).

The network is a deterministic CPU MuZero-shaped net (mazero_amd.nets.MuZeroShapedNet, hidden
16 per agent) in eval mode, wrapped to record every call; for the float16 cases its policy logits
are cast to float16, as CUDA autocast yields them (the reference's numpy glue then runs in
float16, mcts_sampled.py:64-65,158-161).

Recorded per case (see `record_case`):
  root inputs        hidden [B, N*H] f32, reward / value [B, 1] f32, logits [B, N, A] (f32|f16),
                     legal mask [B, N, A] int64 (or none), factor [B, agent] int32 (or none)
  per simulation s   the tree's selection (idx_x, idy, action), the joint action passed to
                     recurrent_inference, the model's outputs (prediction logits on the leaf, next
                     hidden state, reward, value, policy logits), and the expansion arguments the
                     driver passed to the tree (reward, value, probs, beta as float32)
  prepare            its arguments (rewards, values, probs, beta, K, eps, noises) and the seed
  SearchOutput       every field (per-root lists padded to the widest root, with degrees)
  np_random after    the next 4 doubles the generator draws after the search

and tests/golden/eps_greedy_torch.npz: core/utils.py's eps_greedy_action itself over 400 roots
under a seeded torch generator (record_eps_greedy).

Usage:  make -C oracle && python oracle/gen_driver_golden.py
"""
from __future__ import annotations

import ctypes as C
import json
import os
import sys
import types

sys.dont_write_bytecode = True  # nothing may be written under /root/reference

import numpy as np  # noqa: E402
import torch  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
REFERENCE = os.environ.get("MZ_REFERENCE", "/root/reference")
REF_LIB = os.path.join(HERE, "_ref", "libmzref.so")
GOLDEN = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, ROOT)

from mazero_amd import _capi  # noqa: E402
from mazero_amd import cytree as mz_cytree  # noqa: E402
from mazero_amd.nets import MuZeroShapedNet, SearchConfig  # noqa: E402

HIDDEN = 16

# name: (N, A, B, S, K, agent, legal_zero_frac (None = no mask), add_noise, logits dtype, rng kind, seed)
CASES = {
    "3m_k1_ag0": (3, 9, 48, 20, 1, 0, 0.0, True, "float32", "RandomState", 1),
    "3m_k5_ag2_f16": (3, 9, 48, 20, 5, 2, 0.3, True, "float16", "Generator", 2),
    "3m_k5_ag1_nonoise": (3, 9, 32, 16, 5, 1, 0.3, False, "float32", "RandomState", 3),
    "2s3z_k1_ag4_f16": (5, 11, 32, 16, 1, 4, 0.2, True, "float16", "Generator", 4),
    "matrix_k5_ag0_f16_nomask": (2, 3, 8, 25, 5, 0, None, True, "float16", "RandomState", 5),
    "3m_k10_ag1": (3, 9, 40, 24, 10, 1, 0.3, True, "float32", "Generator", 6),
}

SAMPLED = ("actions", "visit_count", "pred_probs", "beta", "beta_hat", "priors", "imp_ratio", "pred_values",
           "mcts_values", "rewards", "qvalues")


def _install_import_stubs(tree_lib, log):
    """Stand-ins for the modules the reference imports but batch_search never calls."""
    for name in ("ray", "cv2"):
        sys.modules.setdefault(name, types.ModuleType(name))
    gym = types.ModuleType("gymnasium")

    class Wrapper:  # base classes of core/utils.py's env wrappers (not used by the search)
        def __init__(self, env=None):
            self.env = env

    gym.Wrapper = Wrapper
    gym.ObservationWrapper = Wrapper
    gym.spaces = types.SimpleNamespace(Box=None)
    sys.modules.setdefault("gymnasium", gym)

    cy = types.ModuleType("core.mcts.ctree.ctree_sampled.cytree")

    class Tree_batch(mz_cytree.Tree_batch):
        """cytree.pyx:7 on the reference ctree; records the driver's tree calls."""

        def __init__(self, root_num, agent_num, action_space_size, sampled_times, simulation_num,
                     tree_value_stat_delta_lb, random_seed, rho, lam):
            log["tree"] = dict(root_num=int(root_num), agent_num=int(agent_num), A=int(action_space_size),
                               K=int(sampled_times), S=int(simulation_num), delta_lb=float(tree_value_stat_delta_lb),
                               seed=int(random_seed), rho=float(rho), lam=float(lam))
            super().__init__(root_num, agent_num, action_space_size, sampled_times, simulation_num,
                             tree_value_stat_delta_lb, random_seed, rho, lam, lib=tree_lib)

        def prepare(self, rewards, values, policy_probs, beta, sampled_times, noise_eps, noises):
            log["prepare"] = dict(rewards=np.array(rewards), values=np.array(values), probs=np.array(policy_probs),
                                  beta=np.array(beta), K=int(sampled_times), eps=float(noise_eps),
                                  noises=np.array(noises))
            return super().prepare(rewards, values, policy_probs, beta, sampled_times, noise_eps, noises)

        def batch_selection(self, pb_c_base, pb_c_init, discount):
            ix, iy, act = super().batch_selection(pb_c_base, pb_c_init, discount)
            log["sel"].append((np.asarray(ix, np.int32), np.asarray(iy, np.int32), np.array(act)))
            return ix, iy, act

        def batch_expansion_and_backup(self, hidden_state_index_x, discount, sampled_times, rewards, values,
                                       policy_probs, beta):
            log["exp"].append(dict(hsx=int(hidden_state_index_x), reward=np.array(rewards), value=np.array(values),
                                   probs=np.array(policy_probs), beta=np.array(beta)))
            return super().batch_expansion_and_backup(hidden_state_index_x, discount, sampled_times, rewards,
                                                      values, policy_probs, beta)

    cy.Tree_batch = Tree_batch
    sys.modules["core.mcts.ctree.ctree_sampled.cytree"] = cy
    if REFERENCE not in sys.path:
        sys.path.insert(0, REFERENCE)
    from core.mcts.tree_search import mcts_sampled  # the reference driver, mcts_sampled.py:1-200

    assert os.path.realpath(mcts_sampled.__file__).startswith(os.path.realpath(REFERENCE)), mcts_sampled.__file__
    return mcts_sampled


class RecordingNet(torch.nn.Module):
    """Eval-mode CPU net with the reference model interface (core/model.py:45-79,
    config/smac/model.py:562-572); policy logits in `logits_dtype`; records every call."""

    def __init__(self, net, logits_dtype, log):
        super().__init__()
        self.net, self.dt, self.log = net, logits_dtype, log

    def prediction(self, h):
        policy, value_logits = self.net.prediction(h)
        policy = policy.to(self.dt)
        self.log["pred"].append(policy.detach().numpy().copy())
        return policy, value_logits

    def recurrent_inference(self, h, action):
        self.log["leaf"].append(h.detach().numpy().copy())
        self.log["joint"].append(action.detach().numpy().copy())
        out = self.net.recurrent_inference(h, action)
        logits = out.policy_logits.astype(np.float16 if self.dt == torch.float16 else np.float32)
        self.log["rec"].append((out.hidden_state.detach().numpy().copy(), np.array(out.reward), np.array(out.value),
                                logits.copy()))
        return type(out)(out.hidden_state, out.reward, out.value, logits)


def _padded(lists, dtype, width_of=lambda a: a.shape[0]):
    deg = np.array([width_of(a) for a in lists], np.int32)
    W = max(1, int(deg.max()))
    out = np.zeros((len(lists), W), dtype)
    for i, a in enumerate(lists):
        out[i, : deg[i]] = a.reshape(-1)
    return out, deg


def record_case(mcts_sampled, tree_lib_log, name, spec):
    N, A, B, S, K, agent, lz, noise, ldt, rng_kind, seed = spec
    log = tree_lib_log
    log.clear()
    log.update(sel=[], exp=[], pred=[], leaf=[], joint=[], rec=[])
    cfg = SearchConfig(action_space_size=A, num_simulations=S, sampled_action_times=K)
    torch.manual_seed(1000 + seed)
    base = MuZeroShapedNet(N, 32, A, hidden=HIDDEN).eval()
    dt = torch.float16 if ldt == "float16" else torch.float32
    net = RecordingNet(base, dt, log).eval()
    g = np.random.default_rng(seed)
    obs = torch.from_numpy(g.standard_normal((B, N, 32)).astype(np.float32))
    with torch.no_grad():
        root = base.initial_inference(obs)
    root_logits = root.policy_logits.astype(np.float16 if dt == torch.float16 else np.float32)
    legal = None
    if lz is not None:
        legal = (g.random((B, N, A)) >= lz).astype(np.int64)
        legal[..., 0] = np.where(legal.sum(-1) == 0, 1, legal[..., 0])
    factor = g.integers(0, A, size=(B, agent)).astype(np.int32) if agent else None
    np_random = np.random.RandomState(seed) if rng_kind == "RandomState" else np.random.default_rng(seed)
    netout = type(root)(root.hidden_state, root.reward, root.value, root_logits)

    out = mcts_sampled.SampledMCTS(cfg, np_random).batch_search(
        net, netout, agent, factor, N, legal, device=torch.device("cpu"), add_noise=noise)
    rng_after = np.asarray(np_random.random(4), np.float64)

    assert len(log["sel"]) == S and len(log["exp"]) == S and len(log["rec"]) == S and len(log["pred"]) == S
    # the reference's leaf gather is pool[idx_x[i]][i] (mcts_sampled.py:130-134): the fixture keeps
    # the pool (root + next hidden states) and the selections, so the leaves are checked, not stored
    pool = np.stack([root.hidden_state.numpy()] + [r[0] for r in log["rec"]])
    for s in range(S):
        ix, iy, _ = log["sel"][s]
        assert np.array_equal(pool[ix, iy], log["leaf"][s]), (name, s)
    z = dict(
        meta=np.frombuffer(json.dumps(dict(
            name=name, N=N, A=A, B=B, S=S, K=K, H=HIDDEN, agent=agent, legal_zero_frac=lz, add_noise=noise,
            logits_dtype=ldt, rng_kind=rng_kind, rng_seed=seed, config=cfg.__dict__, tree=log["tree"],
            reference="core/mcts/tree_search/mcts_sampled.py:34-200 (imported), tree: oracle/_ref/libmzref.so",
        )).encode(), np.uint8),
        root_hidden=root.hidden_state.numpy().astype(np.float32),
        root_reward=np.asarray(root.reward, np.float32), root_value=np.asarray(root.value, np.float32),
        root_logits=root_logits,
        prep_rewards=log["prepare"]["rewards"], prep_values=log["prepare"]["values"],
        prep_probs=log["prepare"]["probs"], prep_beta=log["prepare"]["beta"], prep_noises=log["prepare"]["noises"],
        prep_eps=np.float64(log["prepare"]["eps"]),
        sel_idx=np.stack([t[0] for t in log["sel"]]), sel_idy=np.stack([t[1] for t in log["sel"]]),
        sel_act=np.stack([t[2] for t in log["sel"]]),
        sim_joint=np.stack(log["joint"]), sim_pred=np.stack(log["pred"]),
        sim_next_h=np.stack([r[0] for r in log["rec"]]).astype(np.float32),
        sim_reward=np.stack([r[1] for r in log["rec"]]), sim_value=np.stack([r[2] for r in log["rec"]]),
        sim_logits=np.stack([r[3] for r in log["rec"]]),
        exp_reward=np.stack([e["reward"] for e in log["exp"]]), exp_value=np.stack([e["value"] for e in log["exp"]]),
        exp_probs=np.stack([e["probs"] for e in log["exp"]]), exp_beta=np.stack([e["beta"] for e in log["exp"]]),
        rng_after=rng_after,
        out_value=out.value, out_marginal_visit_count=out.marginal_visit_count,
        out_marginal_priors=out.marginal_priors,
    )
    if legal is not None:
        z["legal"] = legal
    if factor is not None:
        z["factor"] = factor
    for f in SAMPLED:
        lists = getattr(out, "sampled_" + f)
        arr, deg = _padded(lists, lists[0].dtype)
        z["out_sampled_" + f] = arr
        z["out_degrees"] = deg
    return z


def record_eps_greedy():
    """core/utils.py:319-334 `eps_greedy_action` itself, root after root under a seeded torch
    global generator (as the self-play worker calls it, selfplay_worker.py:250-254), over random
    legal masks with zeros (int64, the reference's array dtype), for eps in {0.1, 0.5, 1.0}."""
    from core.utils import eps_greedy_action

    g = np.random.default_rng(7)
    R, A = 400, 11
    masks = (g.random((R, A)) >= 0.4).astype(np.int64)
    masks[:, 0] = np.where(masks.sum(-1) == 0, 1, masks[:, 0])
    greedy = g.integers(0, A, size=R).astype(np.int32)
    out = {}
    for j, eps in enumerate((0.1, 0.5, 1.0)):
        torch.manual_seed(100 + j)
        acts = np.array([int(eps_greedy_action(greedy[i], masks[i], eps)[0]) for i in range(R)], np.int64)
        out[f"actions_eps{j}"] = acts
    path = os.path.join(GOLDEN, "eps_greedy_torch.npz")
    np.savez_compressed(path, masks=masks, greedy=greedy, eps=np.array([0.1, 0.5, 1.0]),
                        seeds=np.array([100, 101, 102]), **out)
    print(f"{path}: {os.path.getsize(path)} B")


def main():
    if not os.path.exists(REF_LIB):
        sys.exit("oracle/_ref/libmzref.so missing: run `make -C oracle` first")
    tree_lib = _capi.bind(C.CDLL(REF_LIB))
    log = {}
    mcts_sampled = _install_import_stubs(tree_lib, log)
    os.makedirs(GOLDEN, exist_ok=True)
    for name, spec in CASES.items():
        z = record_case(mcts_sampled, log, name, spec)
        path = os.path.join(GOLDEN, f"driver_{name}.npz")
        np.savez_compressed(path, **z)
        print(f"{path}: {os.path.getsize(path)} B")
    record_eps_greedy()


if __name__ == "__main__":
    main()
