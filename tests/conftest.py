"""Test configuration.

Markers:
  gpu   needs an MI355X (run with `pytest -m gpu` on the GPU box); everything else runs on CPU.

The oracle libraries (oracle/_build/libmzport.so, and oracle/_ref/libmzref.so where the reference
sources exist) are built on demand here by `make -C oracle`; they are test infrastructure only.
"""
from __future__ import annotations

import ctypes as C
import glob
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import mazero_amd  # noqa: E402,F401  (HIP runtime settings, before anything initialises HIP)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

GOLDEN = os.path.join(ROOT, "tests", "golden")
PORT_LIB = os.path.join(ROOT, "oracle", "_build", "libmzport.so")
REF_LIB = os.path.join(ROOT, "oracle", "_ref", "libmzref.so")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD Instinct MI355X (gfx950)")


def _ensure_oracle_built():
    if not os.path.exists(PORT_LIB):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "port"], check=True,
                       stdout=subprocess.DEVNULL)


@pytest.fixture(scope="session")
def port_lib():
    from mazero_amd import _capi

    _ensure_oracle_built()
    return _capi.bind(C.CDLL(PORT_LIB))


@pytest.fixture(scope="session")
def ref_lib():
    from mazero_amd import _capi

    if not os.path.exists(REF_LIB):
        pytest.skip("reference oracle not built (needs /root/reference; build container only)")
    return _capi.bind(C.CDLL(REF_LIB))


def golden_traces():
    return sorted(glob.glob(os.path.join(GOLDEN, "trace_*.npz")))


def load_trace(path):
    """Returns (SearchInputs, knobs dict, K, expected outputs dict)."""
    from mazero_amd.synthetic import SearchInputs

    z = np.load(path)
    B, A, K, S, seed = [int(x) for x in z["cfg"]]
    c2, c1, g, dl, rho, lam, eps = [float(x) for x in z["knobs"]]
    inp = SearchInputs(B, A, S, seed, z["in_root_reward"], z["in_root_value"], z["in_root_policy"],
                       z["in_root_beta"], z["in_root_noise"], eps, z["in_reward"], z["in_value"], z["in_policy"],
                       z["in_beta"])
    knobs = dict(pb_c_base=c2, pb_c_init=c1, discount=g, delta_lb=dl, rho=rho, lam=lam)
    expected = {k[4:]: z[k] for k in z.files if k.startswith("out_")}
    return inp, knobs, K, expected


def assert_same(out, expected, where=""):
    """Bit-exact comparison of every recorded output (int and float alike)."""
    for k, v in expected.items():
        got = np.asarray(out[k])
        assert got.shape == v.shape, f"{where}{k}: shape {got.shape} != {v.shape}"
        if v.dtype.kind == "f":
            same = np.array_equal(got.view(np.uint32), v.astype(np.float32).view(np.uint32))
        else:
            same = np.array_equal(got, v)
        if not same:
            bad = np.argwhere(got != v)
            raise AssertionError(f"{where}{k}: {len(bad)} mismatches, first at {bad[:3].tolist()}")


def full_fixtures():
    return sorted(glob.glob(os.path.join(GOLDEN, "full_*.npz")))


def load_full(path):
    """A BASELINE-size fixture (oracle/gen_golden.py --full): the inputs regenerated from the
    recorded generator seed and checked against the recorded SHA-256, then
    (SearchInputs, K, expected outputs dict)."""
    from mazero_amd.synthetic import inputs_digest, make_search_inputs

    z = np.load(path)
    B, A, K, S, tree_seed = [int(x) for x in z["cfg"]]
    eps, lz, ties = [float(x) for x in z["gen_args"]]
    inp = make_search_inputs(np.random.default_rng(int(z["gen_seed"][0])), B, A, S, noise_eps=eps,
                             legal_zero_frac=lz, ties=bool(ties))
    assert inp.seed == tree_seed, f"{os.path.basename(path)}: regenerated tree seed differs"
    assert inputs_digest(inp) == bytes(z["inputs_sha256"]).hex(), (
        f"{os.path.basename(path)}: regenerated inputs differ from the recorded ones (numpy generator drift)")
    expected = {k[4:]: z[k] for k in z.files if k.startswith("out_")}
    return inp, K, expected

