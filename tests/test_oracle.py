"""The oracle itself, pinned before it is trusted (CPU only).

* libstdc++ known answers (tests/golden/kat_libstdcxx.json, made by oracle/kat_libstdcxx.cpp):
  the restated std::mt19937 and std::discrete_distribution of oracle/ptree.py
* the golden traces (tests/golden/trace_*.npz, recorded from the compiled reference ctree by
  oracle/gen_golden.py) replayed through the pure-Python ptree and the C++ CPU port
* the reference oracle itself, when it is built here, reproduces the committed traces
"""
from __future__ import annotations

import ctypes as C
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, assert_same, full_fixtures, golden_traces, load_full, load_trace

import ptree
from mazero_amd.cytree import Tree_batch
from mazero_amd.synthetic import make_search_inputs, run_search


@pytest.fixture(scope="module")
def kat():
    with open(os.path.join(GOLDEN, "kat_libstdcxx.json")) as f:
        return json.load(f)


def test_mt19937_known_answers(kat):
    for seed, words in kat["mt"]:
        g = ptree.MT19937(seed)
        assert [g() for _ in range(len(words))] == words, f"seed {seed}"
    g = ptree.MT19937(5489)
    for _ in range(9999):
        g()
    assert g() == kat["mt10000_5489"] == 4123659995  # C++ standard [rand.predef]/3


def test_discrete_distribution_known_answers(kat):
    for seed, weights, draws, consumed in kat["dd"]:
        w = np.asarray(weights, np.float32)
        g = ptree.MT19937(seed)
        d = ptree.Discrete(w)
        got = [d(g) for _ in range(len(draws))]
        assert got == draws, f"seed {seed} weights {weights}"
        assert consumed == (0 if len(w) < 2 else 2 * len(draws))


def test_pbc_table_known_answers(kat):
    """glibc logf as ucb_score evaluates it (cnode.cpp:313)."""
    libm = C.CDLL("libm.so.6")
    libm.logf.restype = C.c_float
    libm.logf.argtypes = [C.c_float]
    f32 = np.float32
    for c2, c1, n, bits in kat["pbc_logf_bits"]:
        x = f32(f32(f32(n) + f32(c2)) + f32(1.0))
        v = f32(f32(libm.logf(float(f32(x / f32(c2))))) + f32(c1))
        assert int(v.view(np.uint32)) == bits


@pytest.mark.parametrize("path", golden_traces(), ids=lambda p: os.path.basename(p)[6:-4])
def test_port_matches_golden(path, port_lib):
    inp, knobs, K, expected = load_trace(path)
    tb = Tree_batch(inp.B, 1, inp.A, K, inp.S, knobs["delta_lb"], inp.seed, knobs["rho"], knobs["lam"], lib=port_lib)
    assert_same(run_search(tb, inp, K, knobs), expected, "port ")


SMALL = [p for p in golden_traces() if not any(s in p for s in ("deep", "27m_k5"))]


@pytest.mark.parametrize("path", SMALL, ids=lambda p: os.path.basename(p)[6:-4])
def test_ptree_matches_golden(path):
    inp, knobs, K, expected = load_trace(path)
    tb = ptree.Tree_batch(inp.B, 1, inp.A, K, inp.S, knobs["delta_lb"], inp.seed, knobs["rho"], knobs["lam"])
    assert_same(run_search(tb, inp, K, knobs), expected, "ptree ")


@pytest.mark.parametrize("path", golden_traces()[:4], ids=lambda p: os.path.basename(p)[6:-4])
def test_reference_reproduces_golden(path, ref_lib):
    inp, knobs, K, expected = load_trace(path)
    tb = Tree_batch(inp.B, 1, inp.A, K, inp.S, knobs["delta_lb"], inp.seed, knobs["rho"], knobs["lam"], lib=ref_lib)
    assert_same(run_search(tb, inp, K, knobs), expected, "ref ")


@pytest.mark.parametrize("K,A,ties,lz", [(1, 9, False, 0.0), (5, 9, False, 0.3), (10, 15, True, 0.0)])
def test_port_matches_reference_fresh(ref_lib, port_lib, K, A, ties, lz):
    """Beyond the committed traces: fresh random searches, reference vs port, bit-exact."""
    rng = np.random.default_rng(K * 100 + A)
    inp = make_search_inputs(rng, 32, A, 50, legal_zero_frac=lz, ties=ties)
    outs = []
    for lib in (ref_lib, port_lib):
        tb = Tree_batch(inp.B, 1, A, K, inp.S, 0.01, inp.seed, 0.75, 0.8, lib=lib)
        outs.append(run_search(tb, inp, K))
    assert_same(outs[1], outs[0], "port vs ref ")


@pytest.mark.parametrize("chunk", range(int(os.environ.get("MZ_FUZZ_CHUNKS", "4"))))  # (as the GPU fuzz)
def test_port_matches_reference_fuzz(ref_lib, port_lib, chunk):
    """The GPU fuzz configurations (tests/fuzz_configs.py: A 1-64, K 1-70, S 1-60, B 1-48, every
    search knob, masks, ties, noise), the CPU port against the reference ctree, bit for bit: the
    GPU's comparison partner is pinned on the same cases."""
    from dataclasses import replace

    from fuzz_configs import fuzz_configs

    for B, A, K, S, knobs, lz, ties, eps, s in fuzz_configs(1234 + chunk, 10):
        rng = np.random.default_rng(s)
        inp = replace(make_search_inputs(rng, B, A, S, legal_zero_frac=lz, ties=ties), noise_eps=eps)
        outs = []
        for lib in (ref_lib, port_lib):
            tb = Tree_batch(inp.B, 1, A, K, inp.S, knobs["delta_lb"], inp.seed, knobs["rho"], knobs["lam"], lib=lib)
            outs.append(run_search(tb, inp, K, knobs))
        assert_same(outs[1], outs[0], f"port vs ref B={B} A={A} K={K} S={S} knobs={knobs}: ")


def test_ptree_joint_action_matches_reference(ref_lib):
    """agent_num = 2 joint-action trees (upstream MAZero semantics)."""
    rng = np.random.default_rng(7)
    B, N, A, K, S = 4, 2, 3, 5, 20
    pol = rng.dirichlet([1.0] * A, (B, N)).astype(np.float32)
    noise = rng.dirichlet([0.3] * A, (B, N)).astype(np.float32)
    r = np.zeros(B, np.float32)
    v = rng.standard_normal(B).astype(np.float32)
    trees = [Tree_batch(B, N, A, K, S, 0.01, 11, 0.75, 0.8, lib=ref_lib),
             ptree.Tree_batch(B, N, A, K, S, 0.01, 11, 0.75, 0.8)]
    res = [[], []]
    for k, tb in enumerate(trees):
        tb.prepare(r, v, pol, pol, K, 0.25, noise)
        for s in range(S):
            ix, _, act = tb.batch_selection(19652.0, 1.25, 0.997)
            res[k].append((list(ix), np.asarray(act).tolist()))
            p = rng.dirichlet([1.0] * A, (B, N)).astype(np.float32) if k == 0 else saved[s][0]
            if k == 0:
                saved.append((p,))
            tb.batch_expansion_and_backup(s + 1, 0.997, K, r, v, p, p)
        res[k].append(tb.get_roots_marginal_visit_count().tolist())
        res[k].append(tb.get_roots_values().tolist())
    assert res[0] == res[1]


saved = []


def test_port_joint_action_trees_match_reference(ref_lib, port_lib):
    """agent_num > 1 on the CPU port vs the reference ctree: the checker of the GPU joint-action
    kernels (tests/test_gpu_parity.py::test_joint_action_trees_vs_port), incl. int64 key wrap."""
    import test_gpu_parity as T

    for name, B, N, A, K, S in T.JOINT:
        rr, orf = T._joint_run(ref_lib, B, N, A, K, S, 3)
        rp, op = T._joint_run(port_lib, B, N, A, K, S, 3)
        for (ia, aa), (ib, ab) in zip(rr, rp):
            assert np.array_equal(ia, ib) and np.array_equal(aa, ab), name
        for k in ("values", "mv", "mp"):
            assert np.array_equal(orf[k].view(np.int32), op[k].view(np.int32)), (name, k)
        for k in ("q", "acts", "vc", "pr", "bh"):
            assert all(np.array_equal(g.view(np.int32), c.view(np.int32)) for g, c in zip(orf[k], op[k])), (name, k)


FULL = full_fixtures()


@pytest.mark.parametrize("path", FULL, ids=[os.path.basename(p)[5:-4] for p in FULL])
def test_port_matches_reference_at_baseline_sizes(port_lib, path):
    """The CPU port against the reference ctree's own outputs at the BASELINE sizes (3m 256 x 50,
    2s3z 1024 x 50, 3s5z 512 x 100, 27m 256 x 200; ties; 30 % masked actions), recorded by
    oracle/gen_golden.py --full; the regenerated inputs are checked against the recorded digest."""
    inp, K, expected = load_full(path)
    tb = Tree_batch(inp.B, 1, inp.A, K, inp.S, 0.01, inp.seed, 0.75, 0.8, lib=port_lib)
    assert_same(run_search(tb, inp, K, per_sim=False), expected, "port ")



def test_port_under_sanitizers():
    """the CPU restatement built with AddressSanitizer + UBSan (make -C oracle asan)
    replays every golden trace and three BASELINE-size fixtures bit-exactly with no report (the
    sanitizer runtime aborts the child process on the first error)."""
    import subprocess
    import sys

    root = os.path.dirname(GOLDEN.rstrip("/"))
    root = os.path.dirname(root)
    subprocess.run(["make", "-C", os.path.join(root, "oracle"), "asan"], check=True, stdout=subprocess.DEVNULL)
    asan = subprocess.check_output(["g++", "-print-file-name=libasan.so"], text=True).strip()
    if not os.path.isabs(asan):
        pytest.skip("libasan not available")
    env = dict(os.environ)
    env["LD_PRELOAD"] = ":".join(x for x in (asan, os.environ.get("LD_PRELOAD", "")) if x)
    env["ASAN_OPTIONS"] = "detect_leaks=0:abort_on_error=1"
    env["UBSAN_OPTIONS"] = "halt_on_error=1:print_stacktrace=1"
    code = f"""
import ctypes as C, os, sys
sys.path[:0] = [{root!r}, {os.path.join(root, "tests")!r}, {os.path.join(root, "oracle")!r}]
from conftest import assert_same, full_fixtures, golden_traces, load_full, load_trace
from mazero_amd import _capi
from mazero_amd.cytree import Tree_batch
from mazero_amd.synthetic import run_search
lib = _capi.bind(C.CDLL(os.path.join({root!r}, "oracle", "_build", "libmzport_asan.so")))
n = 0
for p in golden_traces():
    inp, knobs, K, exp = load_trace(p)
    tb = Tree_batch(inp.B, 1, inp.A, K, inp.S, knobs["delta_lb"], inp.seed, knobs["rho"], knobs["lam"], lib=lib)
    assert_same(run_search(tb, inp, K, knobs), exp, os.path.basename(p)); n += 1
for p in [f for f in full_fixtures() if any(k in f for k in ("3m_k5_ties", "3m_k10", "27m_k1"))]:
    inp, K, exp = load_full(p)
    tb = Tree_batch(inp.B, 1, inp.A, K, inp.S, 0.01, inp.seed, 0.75, 0.8, lib=lib)
    assert_same(run_search(tb, inp, K, per_sim=False), exp, os.path.basename(p)); n += 1
print("sanitized replays", n)
"""
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    assert f"sanitized replays {len(golden_traces()) + 3}" in r.stdout
