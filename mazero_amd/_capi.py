"""ctypes binding of the C-ABI declared in include/mzmcts.h, include/mzdriver.h and
include/mzconsume.h.

`bind(lib)` declares argument/return types on any shared library exporting that ABI.  The product
loads its own HIP library through `mazero_amd._lib.load()`; the tests use the same binder on the
oracle libraries (oracle/_ref/libmzref.so, oracle/_build/libmzport.so) to drive all backends
through one code path.
"""
from __future__ import annotations

import ctypes as C

MZ_OK, MZ_ERR_ARG, MZ_ERR_RUNTIME, MZ_ERR_DEVICE, MZ_ERR_UNSUPPORTED = 0, 1, 2, 3, 4
MZ_MEM_HOST, MZ_MEM_DEVICE = 0, 1

# enum mz_field (include/mzmcts.h), in the order of the cytree.pyx readbacks (cytree.pyx:111-241)
FIELDS = {
    "actions": 0,
    "visit_count": 1,
    "pred_probs": 2,
    "beta": 3,
    "beta_hat": 4,
    "priors": 5,
    "imp_ratio": 6,
    "pred_values": 7,
    "mcts_values": 8,
    "rewards": 9,
    "qvalues": 10,
}
INT_FIELDS = {"actions", "visit_count"}


class ReadbackOut(C.Structure):
    """mz_readback_out (include/mzmcts.h): device destinations of mz_get_roots_device."""
    _fields_ = [
        ("values", C.c_void_p),
        ("marginal_visit_count", C.c_void_p),
        ("marginal_priors", C.c_void_p),
        ("degrees", C.c_void_p),
        ("sampled", C.c_void_p * len(FIELDS)),
    ]

STATS = [
    "selects",
    "path_edges",
    "scored",
    "expands",
    "new_children",
    "backup_nodes",
    "entries_read",
    "entries_written",
    "minmax_nodes",
    "mm_moved",
    "rng_tie_beyond",
    "rng_nxt_beyond",
    "cyc_header",
    "cyc_stage1",
    "cyc_stage2",
    "cyc_expand",
    "cyc_backup",
    "cyc_minmax",
    "cyc_select",
    "cyc_gather",
    "cyc_epilogue",
    "stamped",
    "cyc_w1_round1",
    "cyc_w1_stage2",
    "cyc_w1_backup",
    "cyc_w1_sync",
    "cyc_exp_cdf",
    "cyc_exp_draw",
    "cyc_exp_nodes",
    "cyc_bak_boot",
    "cyc_bak_wait",
    "cyc_bak_nodes",
]

EXPORTS = [
    "mz_last_error",
    "mz_abi_version",
    "mz_backend",
    "mz_create",
    "mz_destroy",
    "mz_set_stream",
    "mz_synchronize",
    "mz_prepare",
    "mz_select",
    "mz_expand_backup",
    "mz_expand_backup_select",
    "mz_prepare_select",
    "mz_gather_rows",
    "mz_get_roots_values",
    "mz_get_roots_marginal_visit_count",
    "mz_get_roots_marginal_priors",
    "mz_get_num_children_of_root",
    "mz_get_root_sampled",
    "mz_max_children",
    "mz_get_roots_sampled_padded",
    "mz_get_roots_device",
    "mz_get_stats",
    "mz_print",
]

_p = C.c_void_p
_i = C.c_int
_f = C.c_float
_i64 = C.c_int64

# include/mzdriver.h (device glue of the driver loop; exported by the product library only)
MZ_DT_F32, MZ_DT_F16 = 0, 1
DRIVER_SIGNATURES = {
    "mz_reseed": (_i, [_p, C.c_uint32]),
    "mz_state_changed": (_i, [_p]),
    "mz_policy_glue": (_i, [_p, _p, _i, _i64, _i64, C.c_double, _p, _p]),
    "mz_root_glue": (_i, [_p, _p, _i, _i64, _i64, _p, _i64, _p, C.c_double, C.c_double, _p, _p, _p]),
    "mz_joint_action": (_i, [_p, _p, _i, _i, _i, _p, _i, _p, _p]),
    "mz_graph_census": (_i, [_p, C.POINTER(_i), C.POINTER(_i)]),
    "mz_fused_kernel": (_i, [_p, C.c_char_p, _i]),
    "mz_set_half_exp_table": (_i, [_p]),
    "mz_expand_backup_readback": (_i, [_p, _i, _f, _i, _p, _p, _p, _p, _f, _p]),
    "mz_readback_ready": (_i, [_p, _f]),
    "mz_trim_caches": (_i, [C.POINTER(_i64)]),
    "mz_debug_paths": (_i, [_p, _p, _p, _i]),
    "mz_arena_info": (_i, [_p, _p, _i]),
}
DRIVER_EXPORTS = sorted(DRIVER_SIGNATURES)

# include/mzconsume.h (on-device consumers of the search output; product library only)
MZ_MARGINAL_GIVEN, MZ_MARGINAL_ARGMAX = 0, 1
CONSUME_SIGNATURES = {
    "mz_select_actions": (_i, [_p, _p, _p, _p, _i, C.c_double, _i, _p, _p, _p, _p]),
    "mz_eps_greedy": (_i, [_p, _p, _i64, _f, _p, _p, _p]),
    "mz_marginal_policy": (_i, [_p, _p, _i64, _p, _i64, _i, _p, _p, _p]),
}
CONSUME_EXPORTS = sorted(CONSUME_SIGNATURES)


def bind(lib: C.CDLL) -> C.CDLL:
    sig = {
        "mz_last_error": (C.c_char_p, []),
        "mz_abi_version": (_i, []),
        "mz_backend": (C.c_char_p, []),
        "mz_create": (_i, [_i, _i, _i, _i, _i, _f, C.c_uint32, _f, _f, _i, C.POINTER(_p)]),
        "mz_destroy": (_i, [_p]),
        "mz_set_stream": (_i, [_p, _p]),
        "mz_synchronize": (_i, [_p]),
        "mz_prepare": (_i, [_p, _p, _p, _p, _p, _i, _f, _p, _i]),
        "mz_select": (_i, [_p, _f, _f, _f, _p, _p, _p, _i]),
        "mz_expand_backup": (_i, [_p, _i, _f, _i, _p, _p, _p, _p, _i]),
        "mz_expand_backup_select": (
            _i,
            [_p, _i, _f, _i, _p, _p, _p, _p, _f, _f, _p, _p, _p, _p, _i64, _i64, _p],
        ),
        "mz_prepare_select": (_i, [_p, _p, _p, _p, _p, _i, _f, _p, _f, _f, _f, _p, _p, _p]),
        "mz_gather_rows": (_i, [_p, _p, _i64, _i64, _p, _p]),
        "mz_get_roots_values": (_i, [_p, _p, _i]),
        "mz_get_roots_marginal_visit_count": (_i, [_p, _p, _i]),
        "mz_get_roots_marginal_priors": (_i, [_p, _p, _i]),
        "mz_get_num_children_of_root": (_i, [_p, _i, _p]),
        "mz_get_root_sampled": (_i, [_p, _i, _i, _f, _p]),
        "mz_max_children": (_i, [_p, _p]),
        "mz_get_roots_sampled_padded": (_i, [_p, _i, _f, _p, _p, _i]),
        "mz_get_roots_device": (_i, [_p, _f, _p]),
        "mz_get_stats": (_i, [_p, _p]),
        "mz_print": (_i, [_p]),
    }
    if hasattr(lib, "mz_policy_glue"):  # include/mzdriver.h: product library only
        # (an experiment build of an older source, MZ_LIB_OVERRIDE, may lack newer entry points:
        # bound when present; tests/test_capi.py checks that the product exports every one)
        sig.update({k: v for k, v in {**DRIVER_SIGNATURES, **CONSUME_SIGNATURES}.items() if hasattr(lib, k)})
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


class MZError(RuntimeError):
    """Raised for a non-zero mz_* status; a RuntimeError like the reference's `except +`."""


def check(lib: C.CDLL, rc: int, what: str) -> None:
    if rc != MZ_OK:
        msg = lib.mz_last_error()
        msg = msg.decode() if msg else ""
        if rc == MZ_ERR_ARG:
            raise ValueError(f"{what}: {msg}")
        raise MZError(f"{what}: {msg}" if msg else f"{what}: status {rc}")
