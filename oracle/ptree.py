"""ORACLE — TEST INFRASTRUCTURE ONLY.  Pure-Python restatement ("ptree") of the reference sampled
MCTS tree, for small cases (BASELINE.json config #1: the 2-agent matrix game, 8 roots x 25 sims).

It mirrors the reference's own data structures -- per-node per-depth `big` / `small` multisets
(SubTreeValueSet, common_lib/utils.h:18-40) and one tree-wide multiset of q-values (CMinMaxStats,
utils.h:42-53) -- kept as sorted Python lists, and restates the two libstdc++ pieces the
reference uses (std::mt19937; std::discrete_distribution<int> with generate_canonical<double,53>)
with exact float32 / float64 rounding through numpy scalars.  It offers the cytree.Tree_batch
interface (cytree.pyx:7-247) so mazero_amd.synthetic.run_search can drive it.

Parity: pinned bit-exactly against tests/golden/trace_*.npz (recorded from the compiled reference)
and against tests/golden/kat_libstdcxx.json (libstdc++ known answers).  Any agent_num is supported.
"""
from __future__ import annotations

import bisect
import ctypes
import math

import numpy as np

# ucb_score calls logf (cnode.cpp:313 resolves to glibc's logf); numpy's float32 log is a
# different implementation, so call the C library's.
_libm = ctypes.CDLL("libm.so.6")
_libm.logf.restype = ctypes.c_float
_libm.logf.argtypes = [ctypes.c_float]

f32 = np.float32
FLOAT_MIN = f32(-1000000.0)  # utils.h:12


class MT19937:
    """std::mt19937 (libstdc++ bits/random.tcc)."""

    def __init__(self, seed: int):
        x = [0] * 624
        x[0] = seed & 0xFFFFFFFF
        for i in range(1, 624):
            x[i] = (1812433253 * (x[i - 1] ^ (x[i - 1] >> 30)) + i) & 0xFFFFFFFF
        self.x = x
        self.p = 624

    def _twist(self):
        x = self.x
        for k in range(624):
            y = (x[k] & 0x80000000) | (x[(k + 1) % 624] & 0x7FFFFFFF)
            x[k] = x[(k + 397) % 624] ^ (y >> 1) ^ (0x9908B0DF if y & 1 else 0)
        self.p = 0

    def __call__(self) -> int:
        if self.p >= 624:
            self._twist()
        z = self.x[self.p]
        self.p += 1
        z ^= z >> 11
        z ^= (z << 7) & 0x9D2C5680
        z ^= (z << 15) & 0xEFC60000
        z ^= z >> 18
        return z & 0xFFFFFFFF


class Discrete:
    """std::discrete_distribution<int> over float weights (random.tcc:2656-2713, 3348-3378)."""

    def __init__(self, w):
        self.cp = []
        if len(w) < 2:
            return
        s = 0.0
        for v in w:
            s += float(v)  # double accumulate
        acc = 0.0
        for i, v in enumerate(w):
            p = float(v) / s
            acc = p if i == 0 else acc + p
            self.cp.append(acc)
        self.cp[-1] = 1.0

    def __call__(self, g: MT19937) -> int:
        if not self.cp:
            return 0
        w1 = float(g())
        w2 = float(g())
        u = (w1 + w2 * 4294967296.0) / 18446744073709551616.0
        if u >= 1.0:
            u = math.nextafter(1.0, 0.0)
        return bisect.bisect_left(self.cp, u)


def _insort(lst, v):
    bisect.insort_right(lst, v)


class ValueSet:
    """SubTreeValueSet (utils.h:18-40, utils.cpp:20-77)."""

    __slots__ = ("ws", "tw", "rho", "lam", "big", "small", "count", "lam_pow")

    def __init__(self, rho, lam):
        self.ws = f32(0.0)
        self.tw = f32(0.0)
        self.rho = f32(rho)
        self.lam = f32(lam)
        self.big, self.small, self.count, self.lam_pow = [], [], [], []

    def update(self, key, depth):
        key = f32(key)
        if len(self.count) <= depth:
            self.big.append([])
            self.small.append([])
            self.count.append(0)
            self.lam_pow.append(f32(1.0) if depth == 0 else f32(self.lam_pow[depth - 1] * self.lam))
        self.count[depth] += 1
        big, small, lp = self.big[depth], self.small[depth], self.lam_pow[depth]
        cur = len(big)
        lim = max(1, int(math.ceil(float(f32(self.count[depth]) * f32(f32(1) - self.rho)))))
        if cur == lim:
            mb = big[0]
            if key < mb:
                _insort(small, key)
            else:
                _insort(small, mb)
                self.ws = f32(self.ws - f32(lp * mb))
                self.tw = f32(self.tw - lp)
                del big[0]
                _insort(big, key)
                self.tw = f32(self.tw + lp)
                self.ws = f32(self.ws + f32(lp * key))
        else:
            if cur + 1 != lim:
                raise RuntimeError("SubTreeValueSet::update: cur_size+1!=size_lim.")
            if not small:
                _insort(big, key)
                self.tw = f32(self.tw + lp)
                self.ws = f32(self.ws + f32(lp * key))
            else:
                ms = small[-1]
                if key > ms:
                    _insort(big, key)
                    self.tw = f32(self.tw + lp)
                    self.ws = f32(self.ws + f32(lp * key))
                else:
                    _insort(big, ms)
                    self.tw = f32(self.tw + lp)
                    self.ws = f32(self.ws + f32(lp * ms))
                    del small[-1]
                    _insort(small, key)

    def value(self):
        return f32(self.ws / self.tw)


class Node:
    """CNode (cnode.h:11-45)."""

    __slots__ = ("visit", "hsx", "reward", "pred_value", "prior", "pred_prob", "beta", "beta_hat", "is_root",
                 "vs", "children", "actions")

    def __init__(self, prior, pred_prob, beta, beta_hat, is_root, rho, lam):
        self.visit = 0
        self.hsx = -1
        self.reward = f32(0.0)
        self.pred_value = f32(0.0)
        self.prior, self.pred_prob, self.beta, self.beta_hat = f32(prior), f32(pred_prob), f32(beta), f32(beta_hat)
        self.is_root = is_root
        self.vs = ValueSet(rho, lam)
        self.children = []
        self.actions = []

    def expanded(self):
        return len(self.children) > 0

    def value(self):  # cnode.cpp:42-56
        return self.vs.value() if self.expanded() else f32(0.0)

    def qsa(self, discount):  # cnode.cpp:58-67
        return f32(self.reward + f32(f32(discount) * self.value()))


class MinMax:
    """CMinMaxStats (utils.cpp:79-103): a multiset of floats."""

    def __init__(self, delta_lb):
        self.se = []
        self.delta_lb = f32(delta_lb)

    def remove(self, v):
        i = bisect.bisect_left(self.se, v)
        if i == len(self.se) or self.se[i] != v:
            raise RuntimeError("CMinMaxStats::remove: value not found")
        del self.se[i]

    def insert(self, v):
        _insort(self.se, v)

    def normalize(self, v):
        if not self.se:
            return v
        mx, mn = self.se[-1], self.se[0]
        delta = f32(mx - mn)
        den = delta if self.delta_lb < delta else self.delta_lb
        return f32(f32(v - mn) / den)


class Tree:
    """CTree (cnode.h:59-105, cnode.cpp:186-530)."""

    def __init__(self, N, A, K, S, delta_lb, seed, rho, lam):
        self.gen = MT19937(seed)
        self.N, self.A, self.K, self.rho, self.lam = N, A, K, rho, lam
        self.mm = MinMax(delta_lb)
        self.root = None
        self.path = []

    def prepare(self, reward, value, policy, beta, K, eps, noises):  # cnode.cpp:205-222
        self.root = Node(1.0, 1.0, 1.0, 1.0, True, self.rho, self.lam)
        self.expand(self.root, 0, reward, value, policy, beta, K, eps, noises)
        self.root.visit += 1
        self.root.vs.update(value, 0)

    def expand(self, node, hsx, reward, value, policy, beta, K, eps, noises):  # cnode.cpp:224-295
        node.hsx = hsx
        node.reward = f32(reward)
        node.pred_value = f32(value)
        dists = [Discrete(beta[i]) for i in range(self.N)]
        counts, acts = {}, {}
        for _ in range(K):
            key = 0
            a = []
            for i in range(self.N):
                ai = dists[i](self.gen)
                a.append(ai)
                key = (key * 23333 + ai) & 0xFFFFFFFFFFFFFFFF
            key = key - (1 << 64) if key >= (1 << 63) else key  # std::map<long> order
            counts[key] = f32(counts.get(key, f32(0.0)) + f32(1.0))
            acts[key] = a
        for key in sorted(counts):
            a = acts[key]
            bh = f32(counts[key] / f32(K))
            bp, pp, prior = f32(1.0), f32(1.0), f32(1.0)
            for i in range(self.N):
                pa = f32(policy[i][a[i]])
                bp = f32(bp * f32(beta[i][a[i]]))
                pp = f32(pp * pa)
                if eps > 0:
                    e = f32(eps)
                    p = f32(f32(pa * f32(f32(1) - e)) + f32(f32(noises[i][a[i]]) * e))
                    prior = f32(prior * p)
                else:
                    prior = f32(prior * pa)
            prior = f32(f32(prior * bh) / bp)
            node.children.append(Node(prior, pp, bp, bh, False, self.rho, self.lam))
            node.actions.append(list(a))

    def ucb(self, child, parent_q, total, c2, c1, discount):  # cnode.cpp:297-335
        c2, c1 = f32(c2), f32(c1)
        x = f32(f32(f32(total) + c2) + f32(1.0))
        pb = f32(f32(_libm.logf(float(f32(x / c2)))) + c1)
        pb = f32(float(pb) * (math.sqrt(total) / float(child.visit + 1)))
        ps = f32(pb * child.prior)
        vs = f32(0.0) if child.visit == 0 else f32(child.qsa(discount) - parent_q)
        vs = self.mm.normalize(vs)
        if vs < 0:
            vs = f32(0.0)
        if vs > 1:
            vs = f32(1.0)
        return f32(ps + vs)

    def select_child(self, node, c2, c1, discount):  # cnode.cpp:337-379
        mx = FLOAT_MIN
        lst = []
        for j, ch in enumerate(node.children):
            s = self.ucb(ch, node.pred_value, node.visit - 1, c2, c1, discount)
            if mx < s:
                mx = s
                lst = [j]
            elif s >= f32(mx - f32(0.000001)):
                lst.append(j)
        if not lst:
            return 0
        return lst[self.gen() % len(lst)]

    def select_path(self, c2, c1, discount):  # cnode.cpp:381-413
        node = self.root
        self.path = [node]
        action = None
        while node.expanded():
            if node.is_root and node.visit <= len(node.children):
                ci = node.visit - 1
            else:
                ci = self.select_child(node, c2, c1, discount)
            action = node.actions[ci]
            node = node.children[ci]
            self.path.append(node)
        return self.path[-2].hsx, action

    def back_propagate(self, value, discount):  # cnode.cpp:415-450
        b = f32(value)
        D = len(self.path) - 1
        g = f32(discount)
        for i in range(D, -1, -1):
            node = self.path[i]
            if i != D and i != 0:
                self.mm.remove(f32(node.qsa(g) - self.path[i - 1].pred_value))
            node.visit += 1
            node.vs.update(b, D - i)
            if i != 0:
                self.mm.insert(f32(node.qsa(g) - self.path[i - 1].pred_value))
            b = f32(node.reward + f32(g * b))


class Tree_batch:
    """cytree.Tree_batch interface over Python trees (cnode.cpp:553-781)."""

    def __init__(self, root_num, agent_num, action_space_size, sampled_times, simulation_num,
                 tree_value_stat_delta_lb, random_seed, rho, lam, root_offset=0):
        self.B, self.N, self.A = root_num, agent_num, action_space_size
        seed = int(random_seed) & 0xFFFFFFFF
        self.trees = [Tree(agent_num, action_space_size, sampled_times, simulation_num, tree_value_stat_delta_lb,
                           (seed * 2333 + root_offset + i) & 0xFFFFFFFF, rho, lam) for i in range(root_num)]

    def _rows(self, x):
        return np.asarray(x, np.float32).reshape(self.B, self.N, self.A)

    def prepare(self, rewards, values, policy_probs, beta, sampled_times, noise_eps, noises):
        r = np.asarray(rewards, np.float32).reshape(-1)
        v = np.asarray(values, np.float32).reshape(-1)
        p, b, n = self._rows(policy_probs), self._rows(beta), self._rows(noises)
        for i, t in enumerate(self.trees):
            t.prepare(r[i], v[i], p[i], b[i], sampled_times, f32(noise_eps), n[i])

    def batch_selection(self, c2, c1, discount):
        ix, iy, acts = [], [], []
        for i, t in enumerate(self.trees):
            x, a = t.select_path(c2, c1, discount)
            ix.append(int(x))
            iy.append(i)
            acts.append(a)
        return ix, iy, np.asarray(acts, np.int32).reshape(self.B, self.N)

    def batch_expansion_and_backup(self, hsx, discount, sampled_times, rewards, values, policy_probs, beta):
        r = np.asarray(rewards, np.float32).reshape(-1)
        v = np.asarray(values, np.float32).reshape(-1)
        p, b = self._rows(policy_probs), self._rows(beta)
        for i, t in enumerate(self.trees):
            t.expand(t.path[-1], hsx, r[i], v[i], p[i], b[i], sampled_times, 0.0, None)
            t.back_propagate(v[i], discount)

    def get_roots_values(self):
        return np.array([t.root.value() for t in self.trees], np.float32)

    def get_roots_marginal_visit_count(self):
        out = np.zeros((self.B, self.N, self.A), np.int32)
        for i, t in enumerate(self.trees):
            for ch, a in zip(t.root.children, t.root.actions):
                for j in range(self.N):
                    out[i, j, a[j]] += ch.visit
        return out

    def get_roots_marginal_priors(self):
        out = np.zeros((self.B, self.N, self.A), np.float32)
        for i, t in enumerate(self.trees):
            for ch, a in zip(t.root.children, t.root.actions):
                for j in range(self.N):
                    out[i, j, a[j]] = f32(out[i, j, a[j]] + ch.prior)
        return out

    def _per_child(self, fn, dtype=np.float32):
        return [np.array([fn(c) for c in t.root.children], dtype) for t in self.trees]

    def get_roots_sampled_actions(self):
        return [np.array(t.root.actions, np.int32).reshape(-1, self.N) for t in self.trees]

    def get_roots_sampled_visit_count(self):
        return self._per_child(lambda c: c.visit, np.int32)

    def get_roots_sampled_pred_probs(self):
        return self._per_child(lambda c: c.pred_prob)

    def get_roots_sampled_beta(self):
        return self._per_child(lambda c: c.beta)

    def get_roots_sampled_beta_hat(self):
        return self._per_child(lambda c: c.beta_hat)

    def get_roots_sampled_priors(self):
        return self._per_child(lambda c: c.prior)

    def get_roots_sampled_imp_ratio(self):
        return self._per_child(lambda c: f32(f32(c.beta_hat / c.beta) * c.pred_prob))

    def get_roots_sampled_pred_values(self):
        return self._per_child(lambda c: c.pred_value)

    def get_roots_sampled_mcts_values(self):
        return self._per_child(lambda c: c.value())

    def get_roots_sampled_rewards(self):
        return self._per_child(lambda c: c.reward)

    def get_roots_sampled_qvalues(self, discount):
        return self._per_child(lambda c: c.qsa(discount))
