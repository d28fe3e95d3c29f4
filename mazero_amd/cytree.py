"""Drop-in replacement for the reference's Cython binding `cytree.Tree_batch`
(core/mcts/ctree/ctree_sampled/cytree.pyx:7-247), backed by the C-ABI of include/mzmcts.h.

Same constructor arguments, same methods, same return types (Python lists of int for the
selection indices, numpy int32/float32 arrays for everything else, per-root lists for the
`get_roots_sampled_*` readbacks).  Inputs follow cytree.pyx:22-47: any shape, reshaped to 1-D,
made C-contiguous, and they must be float32 (Cython raises ValueError on a dtype mismatch, so
does this class).

Besides numpy arrays, every input may be a torch tensor already on the GPU: it is then passed
zero-copy as a device pointer and the call is enqueued on the current torch stream instead of
synchronising.  The `*_device` variants return torch tensors and never synchronise; they are what
the device-resident driver (mazero_amd.mcts_sampled) uses.

By default the product HIP library is used; `lib=` lets the tests drive an oracle library
through this very class.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _capi
from ._capi import FIELDS, INT_FIELDS, MZ_MEM_DEVICE, MZ_MEM_HOST, ReadbackOut, check

try:  # torch is plumbing for device memory/streams; the host path works without it
    import torch
except Exception:  # pragma: no cover
    torch = None


def _is_device_tensor(x) -> bool:
    return torch is not None and isinstance(x, torch.Tensor) and x.is_cuda


def _raw_stream_of(device: int) -> int:
    """The handle of torch's current stream on `device` (what torch.cuda.current_stream(device)
    .cuda_stream returns, without building a Stream object on every call)."""
    f = getattr(torch._C, "_cuda_getCurrentRawStream", None)
    return f(device) if f is not None else torch.cuda.current_stream(device).cuda_stream


def _f32_host(x) -> np.ndarray:
    if type(x) is np.ndarray and x.dtype == np.float32 and x.flags.c_contiguous:  # the common case
        return x.reshape(-1)
    if torch is not None and isinstance(x, torch.Tensor):
        x = x.detach().cpu().numpy()
    x = np.asarray(x).reshape(-1)
    if x.dtype != np.float32:
        raise ValueError(f"Buffer dtype mismatch, expected 'float' but got '{x.dtype}'")
    if not x.flags["C_CONTIGUOUS"]:
        x = np.ascontiguousarray(x)
    return x


def _f32_dev(x):
    x = x.reshape(-1)
    if x.dtype != torch.float32:
        raise ValueError(f"Buffer dtype mismatch, expected 'float' but got '{x.dtype}'")
    return x.contiguous()


def _check_out(t, numel: int, dtype, what: str, device: int) -> None:
    """A caller-provided device output of a readback launch: the kernel writes `numel` elements of
    `dtype` from its data pointer, so anything smaller, of another dtype, strided or on another
    device than the tree's (`device`) would be overwritten out of bounds.  None = field not
    requested."""
    if t is None:
        return
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise ValueError(f"{what}: a CUDA tensor is required")
    if t.device.index != device:
        raise ValueError(f"{what}: on {t.device}, but the tree lives on cuda:{device}")
    if t.dtype != dtype:
        raise ValueError(f"{what}: dtype {t.dtype}, expected {dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{what}: must be contiguous")
    if t.numel() < numel:
        raise ValueError(f"{what}: {t.numel()} elements, the readback writes {numel}")


class Tree_batch:
    """cytree.pyx:7 `cdef class Tree_batch` — one batch of independent sampled-MCTS trees."""

    def __init__(
        self,
        root_num: int,
        agent_num: int,
        action_space_size: int,
        sampled_times: int,
        simulation_num: int,
        tree_value_stat_delta_lb: float,
        random_seed: int,
        rho: float,
        lam: float,
        *,
        root_offset: int = 0,
        lib=None,
    ):
        if lib is None:
            from ._lib import load

            lib = load()
        self._lib = lib
        self.root_num = int(root_num)
        self.agent_num = int(agent_num)
        self.action_space_size = int(action_space_size)
        self._h = C.c_void_p()
        rc = lib.mz_create(
            self.root_num,
            self.agent_num,
            self.action_space_size,
            int(sampled_times),
            int(simulation_num),
            float(tree_value_stat_delta_lb),
            int(random_seed) & 0xFFFFFFFF,
            float(rho),
            float(lam),
            int(root_offset),
            C.byref(self._h),
        )
        check(lib, rc, "Tree_batch")
        self._keep = []  # host buffers that must outlive an enqueued call
        self._stream_ptr = None
        # device backends follow torch's current stream on every call (oracle libraries are host-only)
        self._on_device = torch is not None and lib.mz_backend() == b"hip-gfx950"
        # the device the handle's arena lives on (mz_create allocates on the current device)
        self.device_index = torch.cuda.current_device() if self._on_device else None
        self._maxdeg = None

    # -- lifetime ---------------------------------------------------------------------------
    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                self._lib.mz_destroy(h)
            except Exception:
                pass
            self._h = None

    def _sync_stream(self):
        """Bind the handle to torch's current stream, so its work is ordered with torch's (also
        for host-buffer calls and readbacks: a graph replay or torch kernel on the current stream
        must finish before the tree is read)."""
        if not self._on_device:
            return
        s = _raw_stream_of(self.device_index)
        if s != self._stream_ptr:
            check(self._lib, self._lib.mz_set_stream(self._h, C.c_void_p(s)), "set_stream")
            self._stream_ptr = s

    def _inputs(self, *arrays):
        """Returns (pointers, mem, keepalive)."""
        dev = [_is_device_tensor(a) for a in arrays]
        if any(dev):
            if not all(dev):
                raise ValueError("mix of host and device inputs")
            ts = [_f32_dev(a) for a in arrays]
            self._sync_stream()
            return [C.c_void_p(t.data_ptr()) for t in ts], MZ_MEM_DEVICE, ts
        hs = [_f32_host(a) for a in arrays]
        self._sync_stream()
        return [h.ctypes.data for h in hs], MZ_MEM_HOST, hs

    # -- search (cytree.pyx:21-91) --------------------------------------------------------------
    def prepare(self, rewards, values, policy_probs, beta, sampled_times, noise_eps, noises):
        ptrs, mem, keep = self._inputs(rewards, values, policy_probs, beta, noises)
        rc = self._lib.mz_prepare(
            self._h, ptrs[0], ptrs[1], ptrs[2], ptrs[3], int(sampled_times), float(noise_eps), ptrs[4], mem
        )
        check(self._lib, rc, "prepare")
        self._maxdeg = None

    def batch_selection(self, pb_c_base, pb_c_init, discount):
        B, N = self.root_num, self.agent_num
        out = np.empty((2 + N) * B, np.int32)  # idx | idy | actions, one buffer
        p = out.ctypes.data
        self._sync_stream()
        rc = self._lib.mz_select(self._h, float(pb_c_base), float(pb_c_init), float(discount), p, p + 4 * B,
                                 p + 8 * B, MZ_MEM_HOST)
        check(self._lib, rc, "batch_selection")
        return out[:B].tolist(), out[B:2 * B].tolist(), out[2 * B:].reshape(B, N)

    def batch_expansion_and_backup(self, hidden_state_index_x, discount, sampled_times, rewards, values,
                                   policy_probs, beta):
        ptrs, mem, keep = self._inputs(rewards, values, policy_probs, beta)
        rc = self._lib.mz_expand_backup(
            self._h, int(hidden_state_index_x), float(discount), int(sampled_times), ptrs[0], ptrs[1], ptrs[2],
            ptrs[3], mem
        )
        check(self._lib, rc, "batch_expansion_and_backup")

    # -- device-resident variants (no host synchronisation) ------------------------------------
    def batch_selection_device(self, pb_c_base, pb_c_init, discount, out=None):
        """Like batch_selection but returns device int32 tensors (idx_x [B], idy [B], actions [B,N])."""
        B, N = self.root_num, self.agent_num
        if out is None:
            dev = torch.device("cuda", self.device_index)  # (the arena's device)
            out = (
                torch.empty(B, dtype=torch.int32, device=dev),
                torch.empty(B, dtype=torch.int32, device=dev),
                torch.empty(B, N, dtype=torch.int32, device=dev),
            )
        self._sync_stream()
        rc = self._lib.mz_select(
            self._h, float(pb_c_base), float(pb_c_init), float(discount),
            C.c_void_p(out[0].data_ptr()), C.c_void_p(out[1].data_ptr()), C.c_void_p(out[2].data_ptr()),
            MZ_MEM_DEVICE,
        )
        check(self._lib, rc, "batch_selection_device")
        return out

    def prepare_selection_device(self, rewards, values, policy_probs, beta, sampled_times, noise_eps, noises,
                                 pb_c_base, pb_c_init, discount, out):
        """prepare + batch_selection_device in one launch (include/mzmcts.h mz_prepare_select): the
        first selection after prepare is the root's forced first child (cnode.cpp:398-399)."""
        ts = [_f32_dev(t) for t in (rewards, values, policy_probs, beta, noises)]
        self._sync_stream()
        rc = self._lib.mz_prepare_select(
            self._h, *[C.c_void_p(t.data_ptr()) for t in ts[:4]], int(sampled_times), float(noise_eps),
            C.c_void_p(ts[4].data_ptr()), float(pb_c_base), float(pb_c_init), float(discount),
            C.c_void_p(out[0].data_ptr()), C.c_void_p(out[1].data_ptr()), C.c_void_p(out[2].data_ptr()),
        )
        check(self._lib, rc, "prepare_selection_device")
        self._maxdeg = None
        return out

    def expansion_backup_selection_device(self, hidden_state_index_x, discount, sampled_times, rewards, values,
                                          policy_probs, beta, pb_c_base, pb_c_init, out, pool=None,
                                          gather_out=None):
        """Fused expand+backup of simulation s and selection of s+1 (+ optional hidden-state gather)."""
        ts = [_f32_dev(t) for t in (rewards, values, policy_probs, beta)]
        self._sync_stream()
        if pool is not None:
            slot_stride = pool.stride(0) * pool.element_size()
            row_bytes = pool[0, 0].numel() * pool.element_size()
            pool_ptr = C.c_void_p(pool.data_ptr())
            g_ptr = C.c_void_p(gather_out.data_ptr())
        else:
            slot_stride = row_bytes = 0
            pool_ptr = g_ptr = None
        rc = self._lib.mz_expand_backup_select(
            self._h, int(hidden_state_index_x), float(discount), int(sampled_times),
            *[C.c_void_p(t.data_ptr()) for t in ts], float(pb_c_base), float(pb_c_init),
            C.c_void_p(out[0].data_ptr()), C.c_void_p(out[1].data_ptr()), C.c_void_p(out[2].data_ptr()),
            pool_ptr, int(slot_stride), int(row_bytes), g_ptr,
        )
        check(self._lib, rc, "expansion_backup_selection_device")
        return out

    def gather_rows(self, pool, idx_x, out):
        """out[i] = pool[idx_x[i], i] on the device (mcts_sampled.py:130-134); pool [slots, B, ...]."""
        self._sync_stream()
        rc = self._lib.mz_gather_rows(
            self._h, C.c_void_p(pool.data_ptr()), int(pool.stride(0) * pool.element_size()),
            int(pool[0, 0].numel() * pool.element_size()), C.c_void_p(idx_x.data_ptr()), C.c_void_p(out.data_ptr()),
        )
        check(self._lib, rc, "gather_rows")
        return out

    def reseed(self, random_seed: int):
        """Same trees as a fresh Tree_batch(..., random_seed, ...) from the next prepare on
        (include/mzdriver.h, product library only)."""
        self._sync_stream()
        check(self._lib, self._lib.mz_reseed(self._h, int(random_seed) & 0xFFFFFFFF), "reseed")

    def state_changed(self):
        """Drop host-side readback caches after replaying a captured graph of this handle's calls."""
        self._sync_stream()
        check(self._lib, self._lib.mz_state_changed(self._h), "state_changed")

    # -- device readbacks (no host synchronisation) -------------------------------------------
    def get_roots_values_device(self, out=None):
        dev = torch.device("cuda", self.device_index)  # (the arena's device)
        out = torch.empty(self.root_num, dtype=torch.float32, device=dev) if out is None else out
        self._sync_stream()
        check(self._lib, self._lib.mz_get_roots_values(self._h, C.c_void_p(out.data_ptr()), MZ_MEM_DEVICE),
              "get_roots_values_device")
        return out

    def get_roots_marginal_device(self, visit_out=None, prior_out=None):
        """(marginal visit counts int32 [B, N, A], marginal priors f32 [B, N, A]) on the device."""
        dev = torch.device("cuda", self.device_index)  # (the arena's device)
        shape = (self.root_num, self.agent_num, self.action_space_size)
        visit_out = torch.empty(shape, dtype=torch.int32, device=dev) if visit_out is None else visit_out
        prior_out = torch.empty(shape, dtype=torch.float32, device=dev) if prior_out is None else prior_out
        self._sync_stream()
        check(self._lib, self._lib.mz_get_roots_marginal_visit_count(self._h, C.c_void_p(visit_out.data_ptr()),
                                                                      MZ_MEM_DEVICE), "marginal_visit_count_device")
        check(self._lib, self._lib.mz_get_roots_marginal_priors(self._h, C.c_void_p(prior_out.data_ptr()),
                                                                 MZ_MEM_DEVICE), "marginal_priors_device")
        return visit_out, prior_out

    def _readback_out(self, values, marginal_visit_count, marginal_priors, degrees, sampled, what):
        """The mz_readback_out list of caller-provided device tensors (checked: see _check_out)."""
        B, NA = self.root_num, self.agent_num * self.action_space_size
        W = self.max_children() if sampled else 0
        dv = self.device_index
        _check_out(values, B, torch.float32, "values", dv)
        _check_out(marginal_visit_count, B * NA, torch.int32, "marginal_visit_count", dv)
        _check_out(marginal_priors, B * NA, torch.float32, "marginal_priors", dv)
        _check_out(degrees, B, torch.int32, "degrees", dv)
        o = ReadbackOut()
        ptr = lambda x: None if x is None else x.data_ptr()  # noqa: E731
        o.values, o.marginal_visit_count = ptr(values), ptr(marginal_visit_count)
        o.marginal_priors, o.degrees = ptr(marginal_priors), ptr(degrees)
        for name, t in (sampled or {}).items():
            if name not in FIELDS:
                raise ValueError(f"{what}: unknown sampled field {name!r}")
            width = W * self.agent_num if name == "actions" else W
            _check_out(t, B * width, torch.int32 if name in INT_FIELDS else torch.float32, f"sampled[{name!r}]", dv)
            o.sampled[FIELDS[name]] = t.data_ptr()
        return o

    def get_roots_device(self, discount: float = 0.0, values=None, marginal_visit_count=None, marginal_priors=None,
                         degrees=None, sampled=None):
        """Every requested readback of all roots in ONE launch, written into the given device tensors
        (include/mzmcts.h mz_get_roots_device): values [B] f32, marginal_* [B, N, A], degrees [B] int32,
        sampled {field name: [B, max_children(*N)]} as get_roots_sampled_padded_device lays them out."""
        o = self._readback_out(values, marginal_visit_count, marginal_priors, degrees, sampled, "get_roots_device")
        self._sync_stream()
        check(self._lib, self._lib.mz_get_roots_device(self._h, float(discount), C.byref(o)), "get_roots_device")

    def expansion_backup_readback_device(self, hidden_state_index_x, discount, sampled_times, rewards, values,
                                         policy_probs, beta, readback_discount: float = 0.0, out: dict = None):
        """The search's last batch_expansion_and_backup (device inputs) and the readback of every root
        output in one launch (include/mzdriver.h mz_expand_backup_readback).  `out`: get_roots_device's
        keyword arguments (values, marginal_visit_count, marginal_priors, degrees, sampled) as a dict;
        None writes the handle's packed readback buffer instead, which the host getters then copy."""
        ts = [_f32_dev(t) for t in (rewards, values, policy_probs, beta)]
        o = None
        if out is not None:
            o = self._readback_out(out.get("values"), out.get("marginal_visit_count"), out.get("marginal_priors"),
                                   out.get("degrees"), out.get("sampled"), "expansion_backup_readback_device")
        self._sync_stream()
        rc = self._lib.mz_expand_backup_readback(
            self._h, int(hidden_state_index_x), float(discount), int(sampled_times),
            *[C.c_void_p(t.data_ptr()) for t in ts], float(readback_discount), None if o is None else C.byref(o))
        check(self._lib, rc, "expansion_backup_readback_device")

    def readback_ready(self, discount: float):
        """After replaying a graph that ended with expansion_backup_readback_device(packed=True): the
        packed readback is current for `discount` (include/mzdriver.h mz_readback_ready)."""
        self._sync_stream()
        check(self._lib, self._lib.mz_readback_ready(self._h, float(discount)), "readback_ready")

    def get_roots_sampled_padded_device(self, name: str, discount: float = 0.0, degrees_out=None):
        """Device form of get_roots_sampled_padded: (tensor [B, maxdeg(*N)], degrees int32 [B])."""
        B, N = self.root_num, self.agent_num
        W = self.max_children()
        dev = torch.device("cuda", self.device_index)  # (the arena's device)
        width = W * N if name == "actions" else W
        out = torch.empty(B, width, dtype=torch.int32 if name in INT_FIELDS else torch.float32, device=dev)
        self._sync_stream()
        rc = self._lib.mz_get_roots_sampled_padded(
            self._h, FIELDS[name], float(discount), C.c_void_p(out.data_ptr()),
            C.c_void_p(degrees_out.data_ptr()) if degrees_out is not None else None, MZ_MEM_DEVICE,
        )
        check(self._lib, rc, f"get_roots_sampled_{name}_device")
        return out, degrees_out

    # -- readbacks (cytree.pyx:93-241) ----------------------------------------------------------
    def get_roots_values(self):
        self._sync_stream()
        out = np.empty(self.root_num, np.float32)
        check(self._lib, self._lib.mz_get_roots_values(self._h, out.ctypes.data_as(C.c_void_p), MZ_MEM_HOST),
              "get_roots_values")
        return out

    def get_roots_marginal_visit_count(self):
        self._sync_stream()
        out = np.empty(self.root_num * self.agent_num * self.action_space_size, np.int32)
        check(self._lib, self._lib.mz_get_roots_marginal_visit_count(self._h, out.ctypes.data_as(C.c_void_p),
                                                                      MZ_MEM_HOST), "get_roots_marginal_visit_count")
        return out.reshape(self.root_num, self.agent_num, self.action_space_size)

    def get_roots_marginal_priors(self):
        self._sync_stream()
        out = np.empty(self.root_num * self.agent_num * self.action_space_size, np.float32)
        check(self._lib, self._lib.mz_get_roots_marginal_priors(self._h, out.ctypes.data_as(C.c_void_p),
                                                                 MZ_MEM_HOST), "get_roots_marginal_priors")
        return out.reshape(self.root_num, self.agent_num, self.action_space_size)

    def max_children(self) -> int:
        if self._maxdeg is None:
            v = C.c_int32()
            check(self._lib, self._lib.mz_max_children(self._h, C.byref(v)), "max_children")
            self._maxdeg = max(1, v.value)
        return self._maxdeg

    def get_roots_sampled_padded(self, name: str, discount: float = 0.0):
        """One batched readback: (array [B, maxdeg(, N)], degrees [B])."""
        B, N = self.root_num, self.agent_num
        W = self.max_children()
        dt = np.int32 if name in INT_FIELDS else np.float32
        width = W * N if name == "actions" else W
        out = np.zeros(B * width, dt)
        deg = np.zeros(B, np.int32)
        self._sync_stream()
        rc = self._lib.mz_get_roots_sampled_padded(
            self._h, FIELDS[name], float(discount), out.ctypes.data_as(C.c_void_p), deg.ctypes.data_as(C.c_void_p),
            MZ_MEM_HOST,
        )
        check(self._lib, rc, f"get_roots_sampled_{name}")
        return out.reshape(B, width), deg

    def _sampled_lists(self, name, discount=0.0):
        arr, deg = self.get_roots_sampled_padded(name, discount)
        if name == "actions":
            N = self.agent_num
            return [np.ascontiguousarray(arr[i, : deg[i] * N]).reshape(deg[i], N) for i in range(self.root_num)]
        return [np.ascontiguousarray(arr[i, : deg[i]]) for i in range(self.root_num)]

    def get_roots_sampled_visit_count(self):
        return self._sampled_lists("visit_count")

    def get_roots_sampled_actions(self):
        return self._sampled_lists("actions")

    def get_roots_sampled_pred_probs(self):
        return self._sampled_lists("pred_probs")

    def get_roots_sampled_beta(self):
        return self._sampled_lists("beta")

    def get_roots_sampled_beta_hat(self):
        return self._sampled_lists("beta_hat")

    def get_roots_sampled_priors(self):
        return self._sampled_lists("priors")

    def get_roots_sampled_imp_ratio(self):
        return self._sampled_lists("imp_ratio")

    def get_roots_sampled_pred_values(self):
        return self._sampled_lists("pred_values")

    def get_roots_sampled_mcts_values(self):
        return self._sampled_lists("mcts_values")

    def get_roots_sampled_rewards(self):
        return self._sampled_lists("rewards")

    def get_roots_sampled_qvalues(self, discount):
        return self._sampled_lists("qvalues", discount)

    # -- diagnostics ------------------------------------------------------------------------------
    def stats(self) -> dict:
        out = (C.c_int64 * _capi_stats_count())()
        self._sync_stream()
        check(self._lib, self._lib.mz_get_stats(self._h, out), "stats")
        return dict(zip(_capi.STATS, list(out)))

    def fused_kernel(self) -> str:
        """Name of the kernel a fused simulation step launches on this handle (include/mzdriver.h
        mz_fused_kernel; product library only)."""
        buf = C.create_string_buffer(64)
        check(self._lib, self._lib.mz_fused_kernel(self._h, buf, len(buf)), "fused_kernel")
        return buf.value.decode()

    def synchronize(self):
        self._sync_stream()
        check(self._lib, self._lib.mz_synchronize(self._h), "synchronize")

    def print(self):
        self._lib.mz_print(self._h)


def _capi_stats_count() -> int:
    return len(_capi.STATS)
