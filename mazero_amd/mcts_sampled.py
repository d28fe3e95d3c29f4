"""Device-resident `SampledMCTS.batch_search` — drop-in for the reference driver
core/mcts/tree_search/mcts_sampled.py:29-200.

Same constructor, same `batch_search` signature, same `SearchOutput` (numpy arrays and per-root
lists).  What changes is where the loop runs.  The reference moves every simulation's network
outputs to the host, prepares the next tree inputs with numpy and calls the CPU tree three times
per simulation.  Here the tree (mazero_amd.cytree on the MI355X library), the hidden-state pool
and the per-simulation glue stay on the device:

    select(s+1) + gather leaf rows          one kernel (fused with expand/backup of s)
    model.prediction(leaf)                  the model's own kernels (only when later agents exist)
    joint action                            mz_joint_action (numpy argmax semantics)
    model.dynamics + model.prediction       the model's own kernels, inverse transforms included
    policy softmax + beta                   mz_policy_glue (numpy float32/float16 arithmetic)

so a search has no host synchronisation between `prepare` and the final readback.  The root
preprocessing (mcts_sampled.py:51-106) is split: the host draws from `np_random` (the Dirichlet
noise, then the tree seed, in the reference's order) and packs the raw root inputs into one pinned
upload; the softmax, the legal masks and beta run on the device (mz_root_glue, numpy's dtype rules
restated) inside the recorded loop.  Inputs the kernel does not cover (float legal masks, other
logits dtypes) take the host path, `root_inputs`, numpy exactly as the reference computes it.

Model interface (core/model.py:45-79): `prediction(h) -> (policy_logits [B,N,A], value_logits)`,
`dynamics(h, joint_action [B,N]) -> (next_h, reward_logits)`, `inverse_value_transform`,
`inverse_reward_transform`; this is what MAMuZeroNet.recurrent_inference does in eval mode
(config/smac/model.py:562-572) minus the host copies.  A model may instead provide
`recurrent_inference_device(h, action) -> (next_h, reward [B,1], value [B,1], policy_logits)`.
"""
from __future__ import annotations

import ctypes as C
import os
import threading
import warnings
import weakref
from collections import OrderedDict
from typing import List, NamedTuple, Tuple

import numpy as np
import torch

from ._capi import INT_FIELDS, MZ_DT_F16, MZ_DT_F32, check
from .cytree import Tree_batch


class SearchOutput(NamedTuple):
    """mcts_sampled.py:12-26."""

    value: np.ndarray
    marginal_visit_count: np.ndarray
    marginal_priors: np.ndarray
    sampled_actions: List[np.ndarray]
    sampled_visit_count: List[np.ndarray]
    sampled_pred_probs: List[np.ndarray]
    sampled_beta: List[np.ndarray]
    sampled_beta_hat: List[np.ndarray]
    sampled_priors: List[np.ndarray]
    sampled_imp_ratio: List[np.ndarray]
    sampled_pred_values: List[np.ndarray]
    sampled_mcts_values: List[np.ndarray]
    sampled_rewards: List[np.ndarray]
    sampled_qvalues: List[np.ndarray]


_SAMPLED_FIELDS = ("actions", "visit_count", "pred_probs", "beta", "beta_hat", "priors", "imp_ratio",
                   "pred_values", "mcts_values", "rewards", "qvalues")


class DeviceSearchOutput(NamedTuple):
    """The search results as device tensors: per-root lists padded to the widest root degree
    (`degrees[i]` valid entries in row i).  `to_host()` gives the reference's SearchOutput."""

    value: torch.Tensor                  # f32 [B]
    marginal_visit_count: torch.Tensor   # i32 [B, 1, A]
    marginal_priors: torch.Tensor        # f32 [B, 1, A]
    degrees: torch.Tensor                # i32 [B]
    sampled: dict                        # field -> [B, maxdeg] (i32 for actions / visit_count)
    tree: object = None                  # the Tree_batch that ran the search (its stream; consumers)

    def to_host(self) -> SearchOutput:
        deg = self.degrees.cpu().numpy()
        host = {k: v.cpu().numpy() for k, v in self.sampled.items()}
        B = deg.shape[0]

        def lists(name):
            a = host[name]
            if name == "actions":
                return [np.ascontiguousarray(a[i, : deg[i]]).reshape(deg[i], 1) for i in range(B)]
            return [np.ascontiguousarray(a[i, : deg[i]]) for i in range(B)]

        return SearchOutput(self.value.cpu().numpy(), self.marginal_visit_count.cpu().numpy(),
                            self.marginal_priors.cpu().numpy(), *[lists(f) for f in _SAMPLED_FIELDS])


def _np(x):
    if isinstance(x, torch.Tensor):
        return x.detach().cpu().numpy()
    return np.asarray(x)


def _dtype_code(t: torch.Tensor) -> int:
    if t.dtype == torch.float32:
        return MZ_DT_F32
    if t.dtype == torch.float16:
        return MZ_DT_F16
    raise TypeError(f"policy logits must be float32 or float16, got {t.dtype}")


class _SearchLoop:
    """Static device buffers of one search configuration and, after the first (eager) search, a
    HIP graph of the whole simulation loop (prepare, S x [network, glue, fused tree kernel]).
    Every input is copied into the static buffers before a run, and the tree seed lives in device
    memory (mz_reseed), so replaying the graph is a new search."""

    def __init__(self, tb, B, A, N, cur, hidden, dev, model, root_mode=None):
        self.tb, self.B, self.A, self.N, self.cur, self.dev = tb, B, A, N, cur, dev
        ensure_half_exp(tb._lib, dev.index if dev.index is not None else torch.cuda.current_device())
        self.model_ref = weakref.ref(model)  # the captured graph reads this model's parameters
        self.root = torch.empty_like(hidden.reshape(B, -1))
        self.rin = [torch.empty(n, dtype=torch.float32, device=dev) for n in (B, B, B * A, B * A, B * A)]
        # root_mode = (logits dtype code, has legal): the root preprocessing runs on the device
        # (mz_root_glue) from one packed upload of the raw root inputs; None: the host computes the
        # prepare arguments (SampledMCTS.root_inputs)
        self.root_mode = root_mode
        if root_mode is not None:
            dt_code, has_legal = root_mode
            ld = np.float16 if dt_code == MZ_DT_F16 else np.float32
            secs = [("rewards", np.float32, B), ("values", np.float32, B), ("noise", np.float32, B * A)]
            if has_legal:
                secs.append(("legal", np.int32, B * A))
            secs.append(("logits", ld, B * A))
            off, self.sec = 0, {}
            for name, dt, n in secs:
                self.sec[name] = (off, dt, n)
                off += (np.dtype(dt).itemsize * n + 15) & ~15
            self.raw_host = torch.empty(off, dtype=torch.uint8, pin_memory=True)
            self.raw = torch.empty(off, dtype=torch.uint8, device=dev)
            self.raw_ev = None
            hv = self.raw_host.numpy()
            self.host_view = {k: hv[o:o + np.dtype(dt).itemsize * n].view(dt) for k, (o, dt, n) in self.sec.items()}
            tdt = {np.float32: torch.float32, np.float16: torch.float16, np.int32: torch.int32}
            self.dev_view = {k: self.raw[o:o + np.dtype(dt).itemsize * n].view(tdt[dt]) for k, (o, dt, n) in self.sec.items()}
        self.sel = (torch.empty(B, dtype=torch.int32, device=dev), torch.empty(B, dtype=torch.int32, device=dev),
                    torch.empty(B, 1, dtype=torch.int32, device=dev))
        self.joint = torch.empty(B, N, dtype=torch.int64, device=dev)
        self.probs = torch.empty(B, A, dtype=torch.float32, device=dev)
        self.beta = torch.empty(B, A, dtype=torch.float32, device=dev)
        self.fac = torch.zeros(B, max(cur, 1), dtype=torch.int32, device=dev)
        self.pool = None
        self.leaf = None
        self.pool_ref = None  # the shared _Pool the two above belong to (K > 1)
        self.graph = None  # None: not recorded yet; False: not replayable (capture found memset nodes)
        self.graph_nodes = None  # (nodes, memset nodes) of the recorded graph
        self.runs = 0
        self.storage = None  # _storage_signature(model) when the loop was made
        self.fused_rb = hasattr(tb._lib, "mz_expand_backup_readback")

    def load(self, hidden, root_arrays, factor):
        self.root.copy_(hidden.reshape(self.B, -1))
        if self.root_mode is None:
            for t, a in zip(self.rin, root_arrays):
                t.copy_(torch.from_numpy(np.ascontiguousarray(a).reshape(-1)))
        else:  # the raw root inputs: packed in pinned memory, one host->device copy
            if self.raw_ev is not None:
                self.raw_ev.synchronize()  # (the previous search's copy has read the pinned buffer)
            dev_logits = None
            for k, a in root_arrays.items():
                if isinstance(a, torch.Tensor):  # device logits: copied on the device below
                    dev_logits = a
                    continue
                np.copyto(self.host_view[k], np.asarray(a).reshape(-1), casting="no")
            self.raw.copy_(self.raw_host, non_blocking=True)
            self.raw_ev = torch.cuda.Event()
            self.raw_ev.record()
            if dev_logits is not None:
                self.dev_view["logits"].copy_(dev_logits.reshape(-1))
        if self.cur > 0:
            if isinstance(factor, torch.Tensor):  # previous agents' actions, already on the device
                self.fac.copy_(factor[:, : self.cur])
            else:
                self.fac.copy_(torch.from_numpy(np.ascontiguousarray(np.asarray(factor)[:, : self.cur], dtype=np.int32)))

    def run(self, model, cfg, eps, tau):
        """One search, mcts_sampled.py:106-172, all on the current stream."""
        tb, B, A, N, cur = self.tb, self.B, self.A, self.N, self.cur
        lib, h = tb._lib, tb._h
        c2, c1, disc = cfg.pb_c_base, cfg.pb_c_init, cfg.discount
        K, S = cfg.sampled_action_times, cfg.num_simulations
        r = self.rin
        model.eval()
        # bind the handle to the current stream first: the direct mz_* launches below (root glue,
        # joint action, policy glue) run on the handle's stream, which under a capture must be the
        # capturing one, or the launch runs at record time and is missing from the graph
        tb._sync_stream()
        if self.root_mode is not None:  # root preprocessing on the device, mcts_sampled.py:64-100
            dv = self.dev_view
            lg = dv.get("legal")
            check(lib, lib.mz_root_glue(h, C.c_void_p(dv["logits"].data_ptr()), self.root_mode[0], A, 0,
                                        None if lg is None else C.c_void_p(lg.data_ptr()), A,
                                        C.c_void_p(dv["noise"].data_ptr()), float(eps), float(tau),
                                        C.c_void_p(r[2].data_ptr()), C.c_void_p(r[3].data_ptr()),
                                        C.c_void_p(r[4].data_ptr())), "root_glue")
            r = [dv["rewards"], dv["values"], r[2], r[3], r[4]]
        # prepare + the first selection (the root's forced first child) in one launch
        tb.prepare_selection_device(r[0], r[1], r[2], r[3], K, eps, r[4], c2, c1, disc, out=self.sel)
        act = self.sel[2]
        leaf = self.root  # simulation 0 selects a child of every root: its parent is the root (slot 0)
        # One autocast context around the whole loop, its cast cache on: each fp32 weight is cast to
        # float16 once per search instead of once per simulation (the reference enters autocast per
        # simulation, mcts_sampled.py:150, so it casts every weight S times; the casts are identical).
        # The context opens and closes inside a capture, so the cached casts live in the graph's pool.
        # Inside a caller's own autocast context the cache would outlive this loop (it is cleared
        # when the outermost context exits), so there the casts stay per simulation.
        with torch.autocast("cuda", cache_enabled=not torch.is_autocast_enabled("cuda")):
            self._simulations(model, lib, h, leaf, act, B, A, N, cur, K, S, c2, c1, disc, tau)

    def _simulations(self, model, lib, h, leaf, act, B, A, N, cur, K, S, c2, c1, disc, tau):
        tb = self.tb
        for s in range(S):
            if cur + 1 < N:  # later agents' actions from the leaf policy, :136-145
                pred_logits, _ = model.prediction(leaf)
                pred_logits = pred_logits.contiguous()
                ptr, dt = C.c_void_p(pred_logits.data_ptr()), _dtype_code(pred_logits)
            else:
                ptr, dt = None, MZ_DT_F32
            check(lib, lib.mz_joint_action(h, ptr, dt, N, cur, C.c_void_p(self.fac.data_ptr()),
                                           self.fac.shape[1], C.c_void_p(act.data_ptr()),
                                           C.c_void_p(self.joint.data_ptr())), "joint_action")
            next_h, reward, value, logits = SampledMCTS._recurrent(model, leaf, self.joint)  # :150-156
            nh = next_h.reshape(B, -1)
            chain = K == 1
            if chain:
                # K = 1: every tree is a chain, so every selection of simulation s + 1 ends at the
                # child created by simulation s, whose parent holds hidden_state_index_x = s + 1 for
                # every root: the reference's gather pool[s + 1][i] (mcts_sampled.py:130-134) is row i
                # of this network output.  No pool and no gather: the output is the next leaf batch.
                pass
            else:
                if self.pool is None:
                    # one pool per (thread, device, S, B, row, dtype), shared by the agent loops of a
                    # geometry: searches on one thread run one after the other, and every search
                    # writes slot 0 and slots 1..S before it reads them
                    pdt = torch.promote_types(self.root.dtype, nh.dtype)
                    self.pool_ref = _shared_pool(self.dev, S, B, nh.shape[1], pdt)
                    self.pool, self.leaf = self.pool_ref.pool, self.pool_ref.leaf
                if s == 0:
                    self.pool[0].copy_(self.root)
                self.pool[s + 1].copy_(nh)  # :164
            logits = logits.contiguous()
            check(lib, lib.mz_policy_glue(h, C.c_void_p(logits.data_ptr()), _dtype_code(logits),
                                          logits.shape[1] * logits.shape[2], cur * A, float(tau),
                                          C.c_void_p(self.probs.data_ptr()), C.c_void_p(self.beta.data_ptr())),
                  "policy_glue")
            r32 = reward.reshape(B).float()
            v32 = value.reshape(B).float()
            if s + 1 < S:
                tb.expansion_backup_selection_device(s + 1, disc, K, r32, v32, self.probs, self.beta, c2, c1,
                                                     out=self.sel, pool=None if chain else self.pool,
                                                     gather_out=None if chain else self.leaf)
                leaf = nh if chain else self.leaf
            elif self.fused_rb:
                # the last expansion also writes the packed readback (mz_expand_backup_readback): the
                # SearchOutput getters then only copy it to the host
                tb.expansion_backup_readback_device(s + 1, disc, K, r32, v32, self.probs, self.beta,
                                                    readback_discount=disc)
            else:
                tb.batch_expansion_and_backup(s + 1, disc, K, r32, v32, self.probs, self.beta)

    def capture(self, model, cfg, eps, tau) -> bool:
        """Record the loop.  The recorded graph is checked before it is instantiated: under the HIP
        runtime's default graph packet capture a replayed memset node can write a stale fill
        pattern.  No mz_* call records one, but the model's ops might (a BLAS
        workspace clear, an output zeroing); then this loop stays eager (graph = False) and the
        caller runs it eagerly.  Returns whether a graph is ready to replay."""
        g = torch.cuda.CUDAGraph(keep_graph=True)
        with torch.cuda.graph(g):
            self.run(model, cfg, eps, tau)
        lib = self.tb._lib
        total, memsets = C.c_int(0), C.c_int(0)
        check(lib, lib.mz_graph_census(C.c_void_p(g.raw_cuda_graph()), C.byref(total), C.byref(memsets)),
              "graph_census")
        self.graph_nodes = (total.value, memsets.value)
        if memsets.value:
            warnings.warn(f"the captured search loop holds {memsets.value} memset node(s) of {total.value} "
                          "(recorded by the model's ops): a replayed memset node can write a stale value under "
                          "the HIP runtime's graph packet capture, so this search loop runs eagerly", RuntimeWarning)
            self.graph = False
            return False
        g.instantiate()
        self.graph = g
        return True


# Search-loop caches.  The reference builds a new Tree_batch and a new hidden-state pool per search
# (mcts_sampled.py:86,89) and frees both when the search returns; here a search geometry keeps its
# device arena (_TREES), each agent loop its captured graph (_LOOPS), and the loops of one geometry
# share one hidden-state pool (_POOLS), so that a 27-agent self-play step holds one [S+1, B, N*H]
# pool, not 27.  Every key carries the calling thread: two threads never share a handle (a handle is
# single-threaded, include/mzmcts.h) or a pool; a pool's key also carries the stream its first loop
# ran on.  Both caches are LRU-bounded (MZ_MAX_TREES,
# MZ_MAX_LOOPS); release() empties them.
_LOCK = threading.RLock()
_LOOPS: "OrderedDict" = OrderedDict()
_TREES: "OrderedDict" = OrderedDict()
_POOLS: "weakref.WeakValueDictionary" = weakref.WeakValueDictionary()
_MAX_LOOPS = int(os.environ.get("MZ_MAX_LOOPS", "64"))  # >= the agents of one self-play step
_MAX_TREES = int(os.environ.get("MZ_MAX_TREES", "8"))
_HALF_EXP: set = set()  # (library, device index) pairs holding the host's float16 exp table


class _Pool:
    """A hidden-state pool [S+1, B, cols] and its leaf-row buffer [B, cols]; freed when the last loop
    holding it goes."""

    __slots__ = ("pool", "leaf", "__weakref__")

    def __init__(self, pool, leaf):
        self.pool, self.leaf = pool, leaf


def _shared_pool(dev, S: int, B: int, cols: int, dtype) -> _Pool:
    # (the current stream too: loops that a thread runs on different streams may overlap on the
    # device, so they must not share a pool -- ADVICE round 5; loops on one stream run in order)
    stream = torch.cuda.current_stream(dev).cuda_stream if torch.device(dev).type == "cuda" else 0
    key = (threading.get_ident(), stream, str(dev), S + 1, B, int(cols), dtype)
    with _LOCK:
        p = _POOLS.get(key)
        if p is None:
            p = _Pool(torch.empty((S + 1, B, cols), dtype=dtype, device=dev), torch.empty((B, cols), dtype=dtype, device=dev))
            _POOLS[key] = p
        return p


def _evict_loops_of(tb) -> None:
    for k in [k for k, v in _LOOPS.items() if v.tb is tb]:
        del _LOOPS[k]


def release() -> int:
    """Drop every cached tree handle, search loop (its graph) and hidden-state pool, of every thread
    (what the reference frees after each search, mcts_sampled.py:86,89), then free the device arenas
    the destroyed handles returned to the library's cache (mz_trim_caches).  The next search of a
    geometry allocates and records again.  Returns the bytes the library released."""
    with _LOCK:
        _LOOPS.clear()
        _TREES.clear()
        _POOLS.clear()
    from ._lib import trim_caches

    return trim_caches()


def half_exp_table() -> np.ndarray:
    """np.exp of every float16 bit pattern as this host's numpy evaluates it (uint16 bits).  numpy's
    float16 exp is not always float32 exp rounded to half (its AVX512_SKX half loop differs in a
    few inputs), and the reference computes the root / leaf softmax with it under autocast."""
    with np.errstate(all="ignore"):
        return np.exp(np.arange(1 << 16, dtype=np.uint16).view(np.float16)).view(np.uint16).copy()


def ensure_half_exp(lib, device_index: int) -> None:
    """Give `lib`'s float16 glue kernels on device `device_index` the host's exp table (once)."""
    key = (id(lib), int(device_index))
    if key in _HALF_EXP or not hasattr(lib, "mz_set_half_exp_table"):
        return
    t = half_exp_table()
    with torch.cuda.device(int(device_index)):
        check(lib, lib.mz_set_half_exp_table(t.ctypes.data_as(C.c_void_p)), "set_half_exp_table")
    _HALF_EXP.add(key)


def _storage_signature(model) -> tuple:
    """Device addresses of the model's parameters and buffers (what a recorded graph reads)."""
    return tuple(t.data_ptr() for t in model.parameters()) + tuple(t.data_ptr() for t in model.buffers())


# One device arena per search geometry and thread, kept across searches and across SampledMCTS
# instances (the self-play worker makes a new SampledMCTS every environment step,
# selfplay_worker.py:187); a search reseeds it instead of allocating a new tree batch as the
# reference does (:89).


MAX_GLUE_ACTIONS = 64  # include/mzdriver.h: the glue kernels hold one action per lane


class SampledMCTS:
    """mcts_sampled.py:29-32.  `lib` selects the tree library (default: the MI355X product)."""

    def __init__(self, config, np_random: np.random.RandomState = None, *, lib=None, use_graph: bool = True,
                 root_shard: Tuple[int, int, int] = None, device_root: bool = True):
        """`root_shard` = (lo, hi, total): this instance searches roots [lo, hi) of a batch of `total`
        roots sharded over ranks (mazero_amd.workers).  Every rank holds the same `np_random` state;
        the per-root draws (Dirichlet noise here, select_action's uniforms in consume) are drawn for
        the whole batch and sliced, and tree i is seeded with its global index, so a rank's results
        equal rows [lo, hi) of the unsharded search."""
        self.config = config
        if int(config.action_space_size) > MAX_GLUE_ACTIONS:
            # the device driver glue (mz_policy_glue, mz_root_glue, mz_joint_action: one lane per
            # action) refuses wider action spaces; refused here, before any search launches (the
            # drop-in Tree_batch surface itself takes A <= 255)
            raise RuntimeError(f"SampledMCTS: action_space_size {config.action_space_size} > {MAX_GLUE_ACTIONS} "
                               "(the device driver glue takes one lane per action; mazero_amd.cytree.Tree_batch "
                               "takes up to 255)")
        self.np_random = np.random if np_random is None else np_random
        self._lib = lib
        if root_shard is not None:
            lo, hi, total = (int(x) for x in root_shard)
            if not 0 <= lo < hi <= total:
                raise ValueError(f"bad root shard {root_shard}")
            root_shard = (lo, hi, total)
        self.root_shard = root_shard
        self.use_graph = use_graph
        # root preprocessing (softmax, masks, beta) on the device (mz_root_glue); False: in numpy on
        # the host (root_inputs), as the reference computes it
        self.device_root = device_root

    # ---------------------------------------------------------------------------------------
    def root_inputs(self, network_output, current_agent_idx, legal_actions_lst, add_noise, sampled_tau):
        """Root preprocessing, mcts_sampled.py:51-106, in numpy on the host (it draws from
        np_random).  Returns the prepare() arguments and the tree seed."""
        cfg = self.config
        alpha, eps = cfg.root_dirichlet_alpha, cfg.root_exploration_fraction
        A = cfg.action_space_size
        B = network_output.hidden_state.shape[0]
        logits = _np(network_output.policy_logits)[:, current_agent_idx, :].reshape(B, 1, A)
        # softmax in the logits' own dtype (float16 under autocast), :64-65
        probs = np.exp(logits - np.max(logits, axis=-1, keepdims=True))
        probs = probs / np.sum(probs, axis=-1, keepdims=True)
        # Dirichlet noise is always drawn, then disabled for evaluation, :68-70
        noises = self.draw_rows(lambda n: self.np_random.dirichlet([alpha] * A, n), B)
        noises = noises.astype(np.float32).reshape(B, 1, A)
        if not add_noise:
            eps = 0.0
        mask = None
        if legal_actions_lst is not None:  # :73-83
            mask = legal_actions_lst[:, current_agent_idx, :].reshape(B, 1, A)
            probs *= mask
            probs += mask * 1e-4
            probs = probs / np.sum(probs, axis=-1, keepdims=True)
            noises *= mask
            noises += mask * 1e-4
            noises = noises / np.sum(noises, axis=-1, keepdims=True)
        seed = self.np_random.choice(256)  # drawn after the noise, :89
        beta = probs * (1 - eps) + noises * eps  # :93-100
        beta = beta ** (1 / sampled_tau)
        if mask is not None:
            beta *= mask
        beta = beta / np.sum(beta, axis=-1, keepdims=True)
        rewards = _np(network_output.reward).reshape(B).astype(np.float32)
        values = _np(network_output.value).reshape(B).astype(np.float32)
        return (rewards, values, probs.astype(np.float32), beta.astype(np.float32), eps,
                noises.astype(np.float32, copy=False)), seed

    def root_raw(self, network_output, current_agent_idx, legal_actions_lst, add_noise):
        """The raw root inputs of the device root preprocessing (mz_root_glue): the Dirichlet draws
        (np_random, then the tree seed, in the reference's order, mcts_sampled.py:68,89) and the
        arrays to upload, or None when the device path does not cover the inputs' dtypes (the host
        path, root_inputs, takes them).  Returns (arrays, (logits dtype code, has legal), eps, seed)."""
        cfg = self.config
        A = cfg.action_space_size
        B = network_output.hidden_state.shape[0]
        lg = network_output.policy_logits
        if isinstance(lg, torch.Tensor):
            if not lg.is_cuda or lg.dtype not in (torch.float32, torch.float16):
                return None
            logits = lg[:, current_agent_idx, :]
            code = _dtype_code(lg)
        else:
            lg = np.asarray(lg)
            if lg.dtype not in (np.float32, np.float16):
                return None
            logits = lg[:, current_agent_idx, :]
            code = MZ_DT_F16 if lg.dtype == np.float16 else MZ_DT_F32
        legal = None
        if legal_actions_lst is not None:
            la = _np(legal_actions_lst)
            if la.dtype.kind not in "iub":
                return None  # (float masks: numpy's float arithmetic differs; the host path)
            legal = la[:, current_agent_idx, :]
            if legal.dtype.kind != "b" and legal.size and (legal.min() < -(1 << 31) or legal.max() >= (1 << 31)):
                return None
            legal = legal.astype(np.int32)
        alpha, eps = cfg.root_dirichlet_alpha, cfg.root_exploration_fraction
        noise = self.draw_rows(lambda n: self.np_random.dirichlet([alpha] * A, n), B).astype(np.float32)
        if not add_noise:
            eps = 0.0
        seed = self.np_random.choice(256)  # drawn after the noise, :89
        arrays = dict(rewards=_np(network_output.reward).reshape(B).astype(np.float32),
                      values=_np(network_output.value).reshape(B).astype(np.float32), noise=noise, logits=logits)
        if legal is not None:
            arrays["legal"] = legal
        return arrays, (code, legal is not None), eps, seed

    def draw_rows(self, draw, B: int) -> np.ndarray:
        """`draw(n)` -> n per-root rows from np_random; with a root shard the whole batch's rows are
        drawn (same generator consumption on every rank) and this shard's rows returned."""
        if self.root_shard is None:
            return draw(B)
        lo, hi, total = self.root_shard
        if hi - lo != B:
            raise ValueError(f"batch of {B} roots but the root shard is [{lo}, {hi})")
        return draw(total)[lo:hi]

    def draw_root_uniforms(self, B: int) -> np.ndarray:
        """One double per root in root order, as B np_random.choice(n, p) calls draw them."""
        return np.asarray(self.draw_rows(lambda n: self.np_random.random(n), B), dtype=np.float64)

    def _tree(self, B, seed, device):
        cfg = self.config
        # (pb_c_base, pb_c_init) select the handle's pUCT tables, which a graph replay does not
        # rewrite: a handle serves one pair only
        key = (threading.get_ident(), B, cfg.action_space_size, cfg.sampled_action_times, cfg.num_simulations,
               float(cfg.tree_value_stat_delta_lb), float(cfg.mcts_rho), float(cfg.mcts_lambda),
               float(cfg.pb_c_base), float(cfg.pb_c_init), str(device), id(self._lib), self._root_offset())
        with _LOCK:
            tb = _TREES.get(key)
            if tb is None:
                tb = Tree_batch(B, 1, cfg.action_space_size, cfg.sampled_action_times, cfg.num_simulations,
                                cfg.tree_value_stat_delta_lb, int(seed), cfg.mcts_rho, cfg.mcts_lambda,
                                root_offset=self._root_offset(), lib=self._lib)
                _TREES[key] = tb
                while len(_TREES) > max(_MAX_TREES, 1):  # least recently used first, with its loops
                    _, old = _TREES.popitem(last=False)
                    _evict_loops_of(old)
            else:
                _TREES.move_to_end(key)
                tb.reseed(int(seed))
            return tb

    def _root_offset(self) -> int:
        return 0 if self.root_shard is None else self.root_shard[0]

    # ---------------------------------------------------------------------------------------
    def batch_search(self, model, network_output, current_agent_idx: int, factor: np.ndarray,
                     true_num_agents: int, legal_actions_lst: np.ndarray = None, device: torch.device = None,
                     add_noise: bool = False, sampled_tau: float = 1.0,
                     sampled_actions_res: Tuple[np.ndarray, np.ndarray] = None) -> SearchOutput:
        """mcts_sampled.py:34-200; results identical to the reference driver given the same model."""
        out = self.batch_search_device(model, network_output, current_agent_idx, factor, true_num_agents,
                                       legal_actions_lst, device, add_noise, sampled_tau, sampled_actions_res,
                                       _host_readback=True)
        return out

    def batch_search_device(self, model, network_output, current_agent_idx: int, factor, true_num_agents: int,
                            legal_actions_lst=None, device=None, add_noise: bool = False, sampled_tau: float = 1.0,
                            sampled_actions_res=None, _host_readback: bool = False):
        """The search with device-resident outputs (DeviceSearchOutput), for on-device consumers."""
        if sampled_actions_res is not None:
            raise NotImplementedError  # as the reference, mcts_sampled.py:108-109
        cfg = self.config
        c2, c1, disc = cfg.pb_c_base, cfg.pb_c_init, cfg.discount
        A, K, S = cfg.action_space_size, cfg.sampled_action_times, cfg.num_simulations
        N, cur = int(true_num_agents), int(current_agent_idx)
        hidden = network_output.hidden_state
        if not (isinstance(hidden, torch.Tensor) and hidden.is_cuda):
            raise ValueError("network_output.hidden_state must be a GPU tensor")
        dev = hidden.device
        B = hidden.shape[0]

        raw = self.root_raw(network_output, cur, legal_actions_lst, add_noise) if self.device_root else None
        if raw is not None:
            root_arrays, root_mode, eps, seed = raw
        else:
            (rr, rv, rp, rb, eps, rn), seed = self.root_inputs(network_output, cur, legal_actions_lst, add_noise,
                                                               sampled_tau)
            root_arrays, root_mode = (rr, rv, rp, rb, rn), None
        with torch.cuda.device(dev):
            tb = self._tree(B, seed, dev)
            # the discount is a kernel argument of the recorded launches
            key = (threading.get_ident(), id(tb), id(model), N, cur, float(eps), float(sampled_tau), float(disc),
                   tuple(hidden.shape), hidden.dtype, root_mode)
            with _LOCK:
                for k in [k for k, v in _LOOPS.items() if v.model_ref() is None]:
                    del _LOOPS[k]  # loops (graph, pool) of models that no longer exist
                st = _LOOPS.get(key)
                sig = _storage_signature(model)
                # ids are reused once an object is freed; a recorded graph reads the parameters at the
                # addresses it was recorded with (re-homed weights, weights.FlatWeights, need a new one)
                if st is None or st.model_ref() is not model or st.storage != sig or st.tb is not tb:
                    st = _LOOPS[key] = _SearchLoop(tb, B, A, N, cur, hidden, dev, model, root_mode)
                    st.storage = sig
                _LOOPS.move_to_end(key)
                while len(_LOOPS) > max(_MAX_LOOPS, 1):  # least recently used first
                    _LOOPS.popitem(last=False)
            st.load(hidden, root_arrays, factor)
            with torch.no_grad():
                if self.use_graph and st.runs > 0 and st.graph is None:
                    st.capture(model, cfg, eps, sampled_tau)  # (records only: nothing runs)
                if self.use_graph and st.runs > 0 and st.graph:
                    st.graph.replay()
                    if st.fused_rb:  # (its last launch left the packed readback)
                        tb.readback_ready(disc)
                    else:
                        tb.state_changed()
                else:
                    st.run(model, cfg, eps, sampled_tau)  # eager (the first search also warms up)
                st.runs += 1

            if _host_readback:  # :176-191 (one packed device->host copy)
                return SearchOutput(
                    tb.get_roots_values(), tb.get_roots_marginal_visit_count(), tb.get_roots_marginal_priors(),
                    tb.get_roots_sampled_actions(), tb.get_roots_sampled_visit_count(),
                    tb.get_roots_sampled_pred_probs(), tb.get_roots_sampled_beta(), tb.get_roots_sampled_beta_hat(),
                    tb.get_roots_sampled_priors(), tb.get_roots_sampled_imp_ratio(),
                    tb.get_roots_sampled_pred_values(), tb.get_roots_sampled_mcts_values(),
                    tb.get_roots_sampled_rewards(), tb.get_roots_sampled_qvalues(disc))
            # every output in one readback launch (mz_get_roots_device)
            W, Nt = tb.max_children(), tb.agent_num  # (the trees' agent_num, mcts_sampled.py:89)
            value = torch.empty(B, dtype=torch.float32, device=dev)
            mv = torch.empty(B, Nt, A, dtype=torch.int32, device=dev)
            mp = torch.empty(B, Nt, A, dtype=torch.float32, device=dev)
            deg = torch.empty(B, dtype=torch.int32, device=dev)
            sampled = {f: torch.empty(B, W * Nt if f == "actions" else W,
                                      dtype=torch.int32 if f in INT_FIELDS else torch.float32, device=dev)
                       for f in _SAMPLED_FIELDS}
            tb.get_roots_device(disc, values=value, marginal_visit_count=mv, marginal_priors=mp, degrees=deg,
                                sampled=sampled)
            return DeviceSearchOutput(value, mv, mp, deg, sampled, tb)

    @staticmethod
    def _recurrent(model, hidden, action):
        """(next_h, reward [B,1], value [B,1], policy_logits [B,N,A]) on the device, as
        MAMuZeroNet.recurrent_inference computes them in eval mode (config/smac/model.py:562-572)."""
        fn = getattr(model, "recurrent_inference_device", None)
        if fn is not None:
            return fn(hidden, action)
        next_h, reward_logits = model.dynamics(hidden, action)
        policy_logits, value_logits = model.prediction(next_h)
        reward = model.inverse_reward_transform(reward_logits)
        value = model.inverse_value_transform(value_logits)
        return next_h, reward, value, policy_logits
