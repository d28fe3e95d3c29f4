"""The C-ABI boundary (CPU only: no device compute here).

* every entry point declared in include/mzmcts.h is exported by the product library and by both
  oracle libraries; include/mzdriver.h (driver glue) and include/mzconsume.h (consumers) by the
  product library
* the product library loads on a machine without a GPU and fails loudly (no silent fallback)
* the Tree_batch shim mirrors cytree.pyx's argument handling (dtype check -> ValueError,
  invariant violations -> RuntimeError)
"""
from __future__ import annotations

import ctypes as C
import os
import re

import numpy as np
import pytest

from conftest import PORT_LIB, REF_LIB, ROOT

from mazero_amd import _capi
from mazero_amd.cytree import Tree_batch

HEADER = os.path.join(ROOT, "include", "mzmcts.h")
DRIVER_HEADER = os.path.join(ROOT, "include", "mzdriver.h")
CONSUME_HEADER = os.path.join(ROOT, "include", "mzconsume.h")


def declared_symbols(header=HEADER):
    txt = open(header).read()
    return sorted(set(re.findall(r"\b(mz_[a-z_]+)\s*\(", txt)))


def test_driver_header_matches_binding_table():
    assert declared_symbols(DRIVER_HEADER) == _capi.DRIVER_EXPORTS
    from mazero_amd import build

    raw = C.CDLL(build.build(verbose=False))
    for name in _capi.DRIVER_EXPORTS:
        assert hasattr(raw, name), name
    # internal hooks of the driver TU stay hidden
    assert not hasattr(raw, "mz_internal_fail")
    assert not hasattr(raw, "mz_internal_agent_num")


def test_consume_header_matches_binding_table():
    assert declared_symbols(CONSUME_HEADER) == _capi.CONSUME_EXPORTS
    from mazero_amd import build

    raw = C.CDLL(build.build(verbose=False))
    for name in _capi.CONSUME_EXPORTS:
        assert hasattr(raw, name), name


def test_header_matches_binding_table():
    assert declared_symbols() == sorted(_capi.EXPORTS)


def test_product_library_builds_and_exports():
    from mazero_amd import build

    lib_path = build.build(verbose=False)
    raw = C.CDLL(lib_path)
    for name in declared_symbols():
        assert hasattr(raw, name), name
    from mazero_amd._lib import load

    lib = load()
    assert lib.mz_backend() == b"hip-gfx950"
    assert lib.mz_abi_version() == 2


def test_abi_version_and_stat_table_match_header():
    """MZ_ABI_VERSION, the enum mz_stat order and MZ_S_COUNT of include/mzmcts.h agree with the
    binding's STATS table and the loader's ABI check (round 5 renumbered the stamp slots without a
    version bump: ADVICE round 5)."""
    from mazero_amd import _lib

    txt = open(HEADER).read()
    assert int(re.search(r"#define MZ_ABI_VERSION (\d+)", txt).group(1)) == _lib.ABI
    enum = dict((k, int(v)) for k, v in re.findall(r"\b(MZ_S_[A-Z0-9_]+)\s*=\s*(\d+)", txt))
    count = enum.pop("MZ_S_COUNT")
    assert sorted(enum.values()) == list(range(count)) and len(_capi.STATS) == count
    for name, v in enum.items():
        assert _capi.STATS[v] == name[len("MZ_S_"):].lower(), name


@pytest.mark.parametrize("path", [PORT_LIB, REF_LIB], ids=["port", "ref"])
def test_oracle_libraries_export(path, port_lib):
    if not os.path.exists(path):
        pytest.skip("not built here")
    raw = C.CDLL(path)
    for name in declared_symbols():
        assert hasattr(raw, name), name


def test_no_gpu_fails_loudly():
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(Exception):
        Tree_batch(4, 1, 9, 1, 10, 0.01, 3, 0.75, 0.8)


def test_dtype_mismatch_is_value_error(port_lib):
    tb = Tree_batch(2, 1, 3, 1, 5, 0.01, 0, 0.75, 0.8, lib=port_lib)
    with pytest.raises(ValueError):
        tb.prepare(np.zeros(2), np.zeros(2, np.float32), np.ones((2, 1, 3), np.float32) / 3,
                   np.ones((2, 1, 3), np.float32) / 3, 1, 0.0, np.ones((2, 1, 3), np.float32) / 3)


def test_shapes_and_types_like_cytree(port_lib):
    B, A, K, S = 3, 4, 2, 4
    tb = Tree_batch(B, 1, A, K, S, 0.01, 5, 0.75, 0.8, lib=port_lib)
    p = np.full((B, 1, A), 1.0 / A, np.float32)
    tb.prepare(np.zeros(B, np.float32), np.ones(B, np.float32), p, p, K, 0.25, p)
    ix, iy, act = tb.batch_selection(19652.0, 1.25, 0.997)
    assert isinstance(ix, list) and isinstance(iy, list) and iy == [0, 1, 2]
    assert act.dtype == np.int32 and act.shape == (B, 1)
    tb.batch_expansion_and_backup(1, 0.997, K, np.zeros(B, np.float32), np.ones(B, np.float32), p, p)
    assert tb.get_roots_values().dtype == np.float32
    assert tb.get_roots_marginal_visit_count().shape == (B, 1, A)
    assert tb.get_roots_marginal_visit_count().dtype == np.int32
    sa = tb.get_roots_sampled_actions()
    assert len(sa) == B and sa[0].dtype == np.int32 and sa[0].shape[1] == 1
    sv = tb.get_roots_sampled_visit_count()
    assert all(v.sum() == 1 for v in sv)  # one simulation -> one child visit


def test_pool_overflow_is_runtime_error(port_lib):
    B, A, K, S = 2, 3, 1, 2
    tb = Tree_batch(B, 1, A, K, S, 0.01, 5, 0.75, 0.8, lib=port_lib)
    p = np.full((B, 1, A), 1.0 / A, np.float32)
    z = np.zeros(B, np.float32)
    tb.prepare(z, z, p, p, K, 0.0, p)
    with pytest.raises(RuntimeError):
        for s in range(10):
            tb.batch_selection(19652.0, 1.25, 0.997)
            tb.batch_expansion_and_backup(s + 1, 0.997, K, z, z, p, p)
