"""Replay of the reference-driver fixtures (tests/golden/driver_*.npz, written by
oracle/gen_driver_golden.py from core/mcts/tree_search/mcts_sampled.py:34-200 itself).

`ReplayNet` stands in for the network: on simulation s it returns the outputs the reference's
network produced on simulation s, and it records what the driver under test fed it (the gathered
leaf hidden states and the joint action), so a test can check both directions of every
simulation's network boundary.  It serves the host oracle driver (oracle/driver.py: eval-mode
`recurrent_inference` returning numpy) and the device driver (mazero_amd.mcts_sampled:
`recurrent_inference_device`, graph-capturable: the recorded inputs are copied into fixed device
buffers and the outputs are fixed device tensors, so a replayed graph repeats the same search).
"""
from __future__ import annotations

import glob
import json
import os

import numpy as np
import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
SAMPLED = ("actions", "visit_count", "pred_probs", "beta", "beta_hat", "priors", "imp_ratio", "pred_values",
           "mcts_values", "rewards", "qvalues")


def driver_fixtures():
    return sorted(glob.glob(os.path.join(GOLDEN, "driver_*.npz")))


class DriverFixture:
    def __init__(self, path):
        z = np.load(path)
        self.z = {k: z[k] for k in z.files}
        self.meta = json.loads(bytes(self.z["meta"]).decode())
        m = self.meta
        self.N, self.A, self.B, self.S, self.K, self.agent = m["N"], m["A"], m["B"], m["S"], m["K"], m["agent"]
        self.legal = self.z.get("legal")
        self.factor = self.z.get("factor")

    def config(self):
        from mazero_amd.nets import SearchConfig

        return SearchConfig(**self.meta["config"])

    def np_random(self):
        m = self.meta
        return (np.random.RandomState(m["rng_seed"]) if m["rng_kind"] == "RandomState"
                else np.random.default_rng(m["rng_seed"]))

    def root_output(self, device):
        from mazero_amd.nets import NetworkOutput

        h = torch.from_numpy(self.z["root_hidden"]).to(device)
        return NetworkOutput(h, self.z["root_reward"], self.z["root_value"], self.z["root_logits"])

    def leaves(self):
        """[S, B, N*H]: the leaf rows the reference gathered, pool[idx_x[i]][i] (mcts_sampled.py:130-134)."""
        pool = np.concatenate([self.z["root_hidden"][None], self.z["sim_next_h"]])
        return np.stack([pool[self.z["sel_idx"][s], self.z["sel_idy"][s]] for s in range(self.S)])

    def expected(self):
        """The reference's SearchOutput as {field: array | list of per-root arrays}."""
        z, deg = self.z, self.z["out_degrees"]
        out = dict(value=z["out_value"], marginal_visit_count=z["out_marginal_visit_count"],
                   marginal_priors=z["out_marginal_priors"])
        for f in SAMPLED:
            a = z["out_sampled_" + f]
            rows = [np.ascontiguousarray(a[i, : deg[i]]) for i in range(self.B)]
            out["sampled_" + f] = [r.reshape(-1, 1) for r in rows] if f == "actions" else rows
        return out


class ReplayNet(torch.nn.Module):
    def __init__(self, fx: DriverFixture, device):
        super().__init__()
        z, S, B = fx.z, fx.S, fx.B
        self.fx, self.device = fx, device
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)  # noqa: E731
        self.pred = t(z["sim_pred"])
        self.next_h = t(z["sim_next_h"])
        self.reward = t(z["sim_reward"])
        self.value = t(z["sim_value"])
        self.logits = t(z["sim_logits"])
        self.seen_h = torch.zeros_like(self.next_h)
        self.seen_a = torch.full((S, B, fx.N), -1, dtype=torch.int64, device=device)
        self.s = 0

    def reset(self):
        self.s = 0
        self.seen_h.zero_()
        self.seen_a.fill_(-1)

    # model interface (core/model.py:45-79) ---------------------------------------------------
    def prediction(self, h):
        return self.pred[self.s], None

    def recurrent_inference_device(self, h, action):
        s = self.s
        self.seen_h[s].copy_(h.reshape(self.seen_h[s].shape))
        self.seen_a[s].copy_(action)
        self.s += 1
        return self.next_h[s], self.reward[s], self.value[s], self.logits[s]

    def recurrent_inference(self, h, action):
        """Eval-mode form (config/smac/model.py:562-572): numpy reward / value / logits."""
        from mazero_amd.nets import NetworkOutput

        nh, r, v, lg = self.recurrent_inference_device(h, action)
        return NetworkOutput(nh, r.cpu().numpy(), v.cpu().numpy(), lg.cpu().numpy())

    def check_inputs(self):
        """The leaves and joint actions the driver fed the network equal the reference's."""
        fx = self.fx
        # (a graph replay runs no Python: the counter is not advanced, the recorded copies into
        # seen_h / seen_a are -- reset() cleared them, so every simulation's inputs must be rewritten)
        got_h = self.seen_h.cpu().numpy()
        exp_h = fx.leaves()
        for s in range(fx.S):
            assert np.array_equal(got_h[s].view(np.uint32), exp_h[s].view(np.uint32)), f"leaf rows differ at sim {s}"
        np.testing.assert_array_equal(self.seen_a.cpu().numpy(), fx.z["sim_joint"].astype(np.int64),
                                      err_msg="joint actions differ")
