"""Device-resident search driver (mazero_amd.mcts_sampled) and its glue kernels
(include/mzdriver.h), checked against numpy and against the oracle driver (oracle/driver.py, a
restatement of core/mcts/tree_search/mcts_sampled.py:34-200 over the oracle tree).

CPU tests pin the arithmetic the glue kernels restate:
- numpy's float32 SIMD exp: the constants are parsed from mzdriver.hip and emulated with exact
  FMAs;
- numpy's pairwise summation order.
GPU tests compare the kernels with numpy bit for bit, then compare whole searches with the
oracle driver running the same network on the same GPU.
"""
from __future__ import annotations

import ctypes as C
import math
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIP = os.path.join(ROOT, "mazero_amd", "csrc", "mzdriver.hip")


# ------------------------------------------------------------------------------------------------
# numpy arithmetic the kernels restate (CPU)
# ------------------------------------------------------------------------------------------------
def _kernel_constants():
    src = open(HIP).read()
    names = ["kLog2e", "kLn2Hi", "kLn2Lo", "kP0", "kP1", "kP2", "kP3", "kP4", "kP5", "kQ0", "kQ1", "kQ2"]
    out = {}
    for n in names:
        m = re.search(rf"constexpr float {n} = ([-+0-9.eE]+)f;", src)
        assert m, n
        out[n] = np.float32(float(m.group(1)))
    return out


def _fma(a, b, c):
    # float32 operands: the product is exact in float64; one rounding of the sum to float64 and
    # then to float32 equals the single fused rounding except for double-rounding ties, which
    # the sweep below would expose as mismatches.
    return (a.astype(np.float64) * b.astype(np.float64) + c.astype(np.float64)).astype(np.float32)


def np_expf_emulated(x):
    k = _kernel_constants()
    x = np.asarray(x, np.float32)
    q = np.rint((x * k["kLog2e"]).astype(np.float32))
    full = lambda v: np.full_like(x, v)  # noqa: E731
    y = _fma(q, full(k["kLn2Hi"]), x)
    y = _fma(q, full(k["kLn2Lo"]), y)
    num = _fma(full(k["kP5"]), y, full(k["kP4"]))
    for c in ("kP3", "kP2", "kP1", "kP0"):
        num = _fma(num, y, full(k[c]))
    den = _fma(full(k["kQ2"]), y, full(k["kQ1"]))
    den = _fma(den, y, full(k["kQ0"]))
    r = (num / den).astype(np.float32)
    with np.errstate(all="ignore"):
        out = np.ldexp(r, np.clip(q, -300, 300).astype(np.int32)).astype(np.float32)
    out = np.where(x < -104.0, np.float32(0), out)
    return out


def np_row_sum_emulated(a):
    """numpy's pairwise summation of one contiguous row of n <= 128 float32 values."""
    a = np.asarray(a, np.float32)
    n = len(a)
    if n < 8:
        r = np.float32(0)
        for v in a:
            r = np.float32(r + v)
        return r
    acc = list(a[:8])
    n8 = n - n % 8
    for i in range(8, n8, 8):
        for j in range(8):
            acc[j] = np.float32(acc[j] + a[i + j])
    res = np.float32(np.float32(np.float32(acc[0] + acc[1]) + np.float32(acc[2] + acc[3]))
                     + np.float32(np.float32(acc[4] + acc[5]) + np.float32(acc[6] + acc[7])))
    for i in range(n8, n):
        res = np.float32(res + a[i])
    return res


def test_numpy_float32_exp_restatement():
    rng = np.random.default_rng(0)
    xs = [
        ((rng.random(1_000_000) * 2 - 1) * 20).astype(np.float32),
        (-rng.random(500_000) * 110).astype(np.float32),  # softmax range incl. denormals / zero
        (-110 + 25 * rng.random(500_000)).astype(np.float32),
        np.arange(0x80000000, 0xBF800001, 4099, dtype=np.uint64).astype(np.uint32).view(np.float32),  # [-1, 0]
    ]
    for x in xs:
        got = np_expf_emulated(x)
        ref = np.exp(x)
        bad = np.flatnonzero(got.view(np.uint32) != ref.view(np.uint32))
        assert bad.size == 0, f"{bad.size} mismatches, e.g. x={x[bad[:3]]} got={got[bad[:3]]} numpy={ref[bad[:3]]}"


def test_numpy_pairwise_sum_restatement():
    rng = np.random.default_rng(1)
    for n in list(range(1, 70)):
        X = (rng.random((200, n)) * rng.choice([1e-3, 1.0, 1e3], size=(200, n))).astype(np.float32)
        S = np.sum(X, axis=-1, keepdims=True)[:, 0]
        for i in range(200):
            assert np_row_sum_emulated(X[i]) == S[i], (n, i)


def test_numpy_float16_sum_restatement():
    rng = np.random.default_rng(2)
    for n in (3, 9, 11, 15, 36):
        X = rng.random((300, n)).astype(np.float16)
        S = np.sum(X, axis=-1, keepdims=True)[:, 0]
        for i in range(300):
            assert np.float16(np_row_sum_emulated(X[i].astype(np.float32))) == S[i]


TAUS = (0.5, 2.0, 1.5, 0.3, 3.0, 0.7, 0.25, 1.1)


def _cr_pow(x: np.ndarray, tau: float) -> np.ndarray:
    """x ** (1 / tau) as the glue kernels evaluate it (mzdriver.hip np_pow_as): the exponent cast
    to x's dtype (NEP 50), the float64 pow (libm, correctly rounded) rounded to float, then to x's
    dtype."""
    e = float(x.dtype.type(1 / tau))
    flat = x.astype(np.float32).ravel()
    r = np.array([math.pow(float(v), e) for v in flat], dtype=np.float32).reshape(x.shape)
    return r.astype(x.dtype)


def _numpy_policy_glue(logits, tau=1.0, cr_pow=False):
    """mcts_sampled.py:158-161 + astype(np.float32) (:169-170), in the logits' dtype.  cr_pow: the
    power correctly rounded (_cr_pow) instead of numpy's own."""
    p = np.exp(logits - np.max(logits, axis=-1, keepdims=True))
    p = p / np.sum(p, axis=-1, keepdims=True)
    b = _cr_pow(p, tau) if cr_pow and tau != 1.0 else p ** (1 / tau)
    b = b / np.sum(b, axis=-1, keepdims=True)
    return p.astype(np.float32), b.astype(np.float32)


def test_oracle_driver_runs_on_cpu(port_lib):
    """The oracle driver itself (CPU network, CPU port tree): search invariants."""
    import torch

    from mazero_amd.nets import SearchConfig, make_net, make_root_batch
    from driver import OracleSampledMCTS

    N, A, B, S = 3, 9, 6, 12
    cfg = SearchConfig(action_space_size=A, num_simulations=S, sampled_action_times=5)
    net = make_net(N, A, seed=0)
    out, legal = make_root_batch(net, B, 64, seed=1, device=torch.device("cpu"), legal_zero_frac=0.3)
    res = OracleSampledMCTS(cfg, np.random.RandomState(0), port_lib).batch_search(
        net, out, 1, np.zeros((B, 1), np.int32), N, legal, add_noise=True)
    assert res["marginal_visit_count"].shape == (B, 1, A)
    assert (res["marginal_visit_count"].sum(axis=(1, 2)) == S).all()
    for i in range(B):
        assert res["sampled_visit_count"][i].sum() == S
        assert legal[i, 1, res["sampled_actions"][i][:, 0]].all()


# ------------------------------------------------------------------------------------------------
# GPU
# ------------------------------------------------------------------------------------------------
def _handle(B, A):
    import torch

    from mazero_amd.cytree import Tree_batch
    from mazero_amd.mcts_sampled import ensure_half_exp

    tb = Tree_batch(B, 1, A, 1, 4, 0.01, 0, 0.75, 0.8)
    ensure_half_exp(tb._lib, torch.cuda.current_device())  # (as the search loop does)
    return tb


def test_half_exp_table_is_numpy():
    """The float16 exp table the glue kernels read is numpy's own np.exp of every half (the SIMD half
    loop where numpy has one); where it differs from float32 exp rounded to half is host-dependent."""
    from mazero_amd.mcts_sampled import half_exp_table

    t = half_exp_table()
    assert t.dtype == np.uint16 and t.shape == (65536,)
    x = np.arange(65536, dtype=np.uint16).view(np.float16)
    fin = np.isfinite(x)
    with np.errstate(all="ignore"):
        np.testing.assert_array_equal(t[fin], np.exp(x[fin]).view(np.uint16))


@pytest.mark.parametrize("tau", TAUS)
def test_numpy_half_power_is_correctly_rounded(tau):
    """numpy's float16 `p ** (1 / tau)` over every half p in [0, 1] (the softmax's range) is the
    correctly rounded power with the exponent cast to half, which the glue kernels evaluate; and for
    float32 arrays the exponents 2 and 0.5 (np.square / np.sqrt) are too.  numpy's other float32
    powers are host-dependent (SVML on AVX-512 hosts, not correctly rounded)."""
    h = np.arange(0x3C01, dtype=np.uint16).view(np.float16)
    np.testing.assert_array_equal((h ** (1 / tau)).view(np.uint16), _cr_pow(h, tau).view(np.uint16))
    if 1 / tau in (2.0, 0.5):
        x = np.random.default_rng(3).random(100_000).astype(np.float32)
        np.testing.assert_array_equal((x ** (1 / tau)).view(np.uint32), _cr_pow(x, tau).view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["float32", "float16"])
@pytest.mark.parametrize("A", [3, 9, 15, 36, 64])
def test_policy_glue_matches_numpy(dtype, A):
    import torch

    from mazero_amd._capi import MZ_DT_F16, MZ_DT_F32, check

    B, N, cur = 512, 3, 1
    rng = np.random.default_rng(A)
    logits = (rng.standard_normal((B, N, A)) * rng.choice([0.1, 1, 4, 30], size=(B, 1, 1))).astype(dtype)
    logits[:7, cur, 0] = -np.inf          # masked-out actions
    logits[7:14, cur, :] = logits[7:14, cur, :1]  # all-equal rows
    if A > 1:
        logits[14:20, cur, 1] = 60.0      # one dominant logit (others underflow)
    tb = _handle(B, A)
    dev = torch.device("cuda", 0)
    x = torch.from_numpy(logits).to(dev)
    probs = torch.empty(B, A, device=dev)
    beta = torch.empty(B, A, device=dev)
    tb._sync_stream()
    rc = tb._lib.mz_policy_glue(tb._h, C.c_void_p(x.data_ptr()), MZ_DT_F16 if dtype == "float16" else MZ_DT_F32,
                                N * A, cur * A, 1.0, C.c_void_p(probs.data_ptr()), C.c_void_p(beta.data_ptr()))
    check(tb._lib, rc, "policy_glue")
    with np.errstate(all="ignore"):
        ep, eb = _numpy_policy_glue(logits[:, cur, :].reshape(B, 1, A))
    gp, gb = probs.cpu().numpy(), beta.cpu().numpy()
    np.testing.assert_array_equal(gp.view(np.uint32), ep.reshape(B, A).view(np.uint32))
    np.testing.assert_array_equal(gb.view(np.uint32), eb.reshape(B, A).view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["float32", "float16"])
@pytest.mark.parametrize("tau", TAUS)
def test_policy_glue_sampled_tau(dtype, tau):
    """sampled_tau != 1 (mcts_sampled.py:160): bit-exact against numpy for float16 logits and for
    the float32 exponents 2 and 0.5; other float32 exponents bit-exact against the correctly
    rounded power and within 1e-6 of this host's numpy (SVML on AVX-512 hosts)."""
    import torch

    from mazero_amd._capi import MZ_DT_F16, MZ_DT_F32, check

    B, N, cur, A = 2048, 2, 1, 64
    rng = np.random.default_rng(int(tau * 100))
    logits = (rng.standard_normal((B, N, A)) * rng.choice([0.1, 1, 4, 12], size=(B, 1, 1))).astype(dtype)
    logits[:5, cur, 1] = 60.0  # one dominant logit (others underflow to 0)
    tb = _handle(B, A)
    dev = torch.device("cuda", 0)
    x = torch.from_numpy(logits).to(dev)
    probs, beta = torch.empty(B, A, device=dev), torch.empty(B, A, device=dev)
    tb._sync_stream()
    rc = tb._lib.mz_policy_glue(tb._h, C.c_void_p(x.data_ptr()), MZ_DT_F16 if dtype == "float16" else MZ_DT_F32,
                                N * A, cur * A, tau, C.c_void_p(probs.data_ptr()), C.c_void_p(beta.data_ptr()))
    check(tb._lib, rc, "policy_glue")
    gp, gb = probs.cpu().numpy(), beta.cpu().numpy()
    row = logits[:, cur, :].reshape(B, 1, A)
    with np.errstate(all="ignore"):
        ep, eb = _numpy_policy_glue(row, tau)
        cp, cb = _numpy_policy_glue(row, tau, cr_pow=True)
    np.testing.assert_array_equal(gp.view(np.uint32), ep.reshape(B, A).view(np.uint32))
    np.testing.assert_array_equal(gb.view(np.uint32), cb.reshape(B, A).view(np.uint32))
    if dtype == "float16" or 1 / tau in (2.0, 0.5):
        np.testing.assert_array_equal(gb.view(np.uint32), eb.reshape(B, A).view(np.uint32))
    else:
        np.testing.assert_allclose(gb, eb.reshape(B, A), rtol=1e-6, atol=1e-30)


@pytest.mark.gpu
@pytest.mark.parametrize("tau", (0.5, 2.0, 1.5))
def test_root_glue_sampled_tau(tau):
    """mz_root_glue with sampled_tau != 1 (mcts_sampled.py:94) against the host root preprocessing:
    bit-exact for the exponents 2 and 0.5 (np.square / np.sqrt of the float32 beta), within 1e-6
    otherwise (numpy's float32 power is SVML's on AVX-512 hosts)."""
    import torch

    from mazero_amd._capi import check
    from mazero_amd.mcts_sampled import SampledMCTS
    from mazero_amd.nets import NetworkOutput, SearchConfig

    B, N, cur, A = 300, 3, 1, 15
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(17)
    tb = _handle(B, A)
    cfg = SearchConfig(action_space_size=A)
    for dtype in ("float32", "float16"):
        for legal_kind in ("none", "int64"):
            logits = (rng.standard_normal((B, N, A)) * 3).astype(dtype)
            legal = None
            if legal_kind == "int64":
                legal = (rng.random((B, N, A)) >= 0.3).astype(np.int64)
                legal[..., 0] = 1
            out = NetworkOutput(torch.zeros(B, 4, device=dev), rng.standard_normal((B, 1)).astype(np.float32),
                                rng.standard_normal((B, 1)).astype(np.float32), logits)
            m_host, m_dev = SampledMCTS(cfg, np.random.RandomState(9)), SampledMCTS(cfg, np.random.RandomState(9))
            (rr, rv, rp, rb, eps, rn), _ = m_host.root_inputs(out, cur, legal, True, tau)
            arrays, mode, eps_d, _ = m_dev.root_raw(out, cur, legal, True)
            t = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in arrays.items()}
            probs, beta, nz = (torch.empty(B, A, device=dev) for _ in range(3))
            tb._sync_stream()
            lg = t.get("legal")
            check(tb._lib, tb._lib.mz_root_glue(tb._h, C.c_void_p(t["logits"].data_ptr()), mode[0], A, 0,
                                                None if lg is None else C.c_void_p(lg.data_ptr()), A,
                                                C.c_void_p(t["noise"].data_ptr()), float(eps_d), tau,
                                                C.c_void_p(probs.data_ptr()), C.c_void_p(beta.data_ptr()),
                                                C.c_void_p(nz.data_ptr())), "root_glue")
            where = f"{dtype} legal={legal_kind} tau={tau}"
            np.testing.assert_array_equal(probs.cpu().numpy().view(np.uint32), rp.reshape(B, A).view(np.uint32),
                                          err_msg=where)
            gb = beta.cpu().numpy()
            if 1 / tau in (2.0, 0.5):
                np.testing.assert_array_equal(gb.view(np.uint32), rb.reshape(B, A).view(np.uint32), err_msg=where)
            else:
                np.testing.assert_allclose(gb, rb.reshape(B, A), rtol=1e-6, atol=1e-30, err_msg=where)


def _half_exp_exceptions() -> np.ndarray:
    """Non-positive float16 values d where this host's np.exp(d) differs from np.exp in float32
    rounded to half (numpy's SIMD half loop; the softmax evaluates exp(x - max) <= 1)."""
    x = np.arange(1 << 16, dtype=np.uint16).view(np.float16)
    x = x[np.isfinite(x) & (x <= 0)]
    with np.errstate(all="ignore"):
        diff = np.exp(x).view(np.uint16) != np.exp(x.astype(np.float32)).astype(np.float16).view(np.uint16)
    return x[diff]


@pytest.mark.gpu
@pytest.mark.parametrize("A", [9, 15])
def test_glue_half_exp_exceptions(A):
    """Rows built so that x - max lands on the half values where numpy's float16 exp is not float32
    exp rounded to half: mz_policy_glue and mz_root_glue against numpy through the exp table."""
    import torch

    from mazero_amd._capi import MZ_DT_F16, check
    from mazero_amd.mcts_sampled import SampledMCTS
    from mazero_amd.nets import NetworkOutput, SearchConfig

    exc = _half_exp_exceptions()
    if exc.size == 0:
        pytest.skip("this host's numpy evaluates float16 exp as float32 exp rounded (no exceptions)")
    B, N, cur = 256, 3, 2
    rng = np.random.default_rng(11 + A)
    logits = rng.standard_normal((B, N, A)).astype(np.float16)
    for i in range(B):  # the row's max is 0, the other entries exception values (and a few normal ones)
        row = rng.choice(exc, size=A)
        row[rng.integers(A)] = 0.0
        row[rng.integers(A)] = np.float16(rng.standard_normal()) - np.float16(4.0)
        logits[i, cur] = row
    dev = torch.device("cuda", 0)
    tb = _handle(B, A)
    x = torch.from_numpy(logits).to(dev)
    probs, beta = torch.empty(B, A, device=dev), torch.empty(B, A, device=dev)
    tb._sync_stream()
    check(tb._lib, tb._lib.mz_policy_glue(tb._h, C.c_void_p(x.data_ptr()), MZ_DT_F16, N * A, cur * A, 1.0,
                                          C.c_void_p(probs.data_ptr()), C.c_void_p(beta.data_ptr())), "policy_glue")
    with np.errstate(all="ignore"):
        ep, eb = _numpy_policy_glue(logits[:, cur, :].reshape(B, 1, A))
    np.testing.assert_array_equal(probs.cpu().numpy().view(np.uint32), ep.reshape(B, A).view(np.uint32))
    np.testing.assert_array_equal(beta.cpu().numpy().view(np.uint32), eb.reshape(B, A).view(np.uint32))
    # the root preprocessing (softmax, then an int64 mask and the noise)
    legal = (rng.random((B, N, A)) >= 0.2).astype(np.int64)
    legal[..., 0] = 1
    out = NetworkOutput(torch.zeros(B, 4, device=dev), rng.standard_normal((B, 1)).astype(np.float32),
                        rng.standard_normal((B, 1)).astype(np.float32), logits)
    cfg = SearchConfig(action_space_size=A)
    m_host, m_dev = SampledMCTS(cfg, np.random.RandomState(5)), SampledMCTS(cfg, np.random.RandomState(5))
    for lg in (None, legal):
        (rr, rv, rp, rb, eps, rn), _ = m_host.root_inputs(out, cur, lg, True, 1.0)
        arrays, mode, eps_d, _ = m_dev.root_raw(out, cur, lg, True)
        t = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in arrays.items()}
        p2, b2, n2 = (torch.empty(B, A, device=dev) for _ in range(3))
        tb._sync_stream()
        lgt = t.get("legal")
        check(tb._lib, tb._lib.mz_root_glue(tb._h, C.c_void_p(t["logits"].data_ptr()), mode[0], A, 0,
                                            None if lgt is None else C.c_void_p(lgt.data_ptr()), A,
                                            C.c_void_p(t["noise"].data_ptr()), float(eps_d), 1.0,
                                            C.c_void_p(p2.data_ptr()), C.c_void_p(b2.data_ptr()),
                                            C.c_void_p(n2.data_ptr())), "root_glue")
        for got, exp in ((p2, rp), (b2, rb), (n2, rn)):
            np.testing.assert_array_equal(got.cpu().numpy().view(np.uint32), exp.reshape(B, A).view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["float32", "float16"])
def test_joint_action_matches_numpy(dtype):
    import torch

    from mazero_amd._capi import MZ_DT_F16, MZ_DT_F32, check

    B, N, A = 300, 5, 11
    rng = np.random.default_rng(7)
    pred = rng.integers(-3, 3, size=(B, N, A)).astype(dtype)  # many ties
    pred[:10, 3, 4] = np.nan
    pred[10:20, 4, :] = pred[10:20, 4, :1]
    dev = torch.device("cuda", 0)
    tb = _handle(B, A)
    for cur in range(N):
        factor = rng.integers(0, A, size=(B, max(cur, 1))).astype(np.int32)
        act = rng.integers(0, A, size=B).astype(np.int32)
        joint = torch.empty(B, N, dtype=torch.int64, device=dev)
        p, f, a = (torch.from_numpy(v).to(dev) for v in (pred, factor, act))
        tb._sync_stream()
        rc = tb._lib.mz_joint_action(tb._h, C.c_void_p(p.data_ptr()), MZ_DT_F16 if dtype == "float16" else MZ_DT_F32,
                                     N, cur, C.c_void_p(f.data_ptr()), factor.shape[1], C.c_void_p(a.data_ptr()),
                                     C.c_void_p(joint.data_ptr()))
        check(tb._lib, rc, "joint_action")
        exp = np.zeros((B, N), np.int64)  # mcts_sampled.py:116-145
        exp[:, :cur] = factor[:, :cur]
        exp[:, cur] = act
        for k in range(cur + 1, N):
            exp[:, k] = np.argmax(pred[:, k, :], axis=-1)
        np.testing.assert_array_equal(joint.cpu().numpy(), exp)


def _compare_outputs(got, exp):
    for name in exp:
        g = getattr(got, name)
        e = exp[name]
        if isinstance(e, list):
            assert len(g) == len(e), name
            for i, (gi, ei) in enumerate(zip(g, e)):
                assert gi.dtype == ei.dtype and gi.shape == ei.shape, (name, i, gi.dtype, ei.dtype, gi.shape, ei.shape)
                np.testing.assert_array_equal(gi.view(np.uint32) if gi.dtype == np.float32 else gi,
                                              ei.view(np.uint32) if ei.dtype == np.float32 else ei, err_msg=f"{name}[{i}]")
        else:
            assert g.dtype == e.dtype and g.shape == e.shape, name
            np.testing.assert_array_equal(g.view(np.uint32) if g.dtype == np.float32 else g,
                                          e.view(np.uint32) if e.dtype == np.float32 else e, err_msg=name)


DRIVER_CASES = [
    # (N, A, B, S, K, agent, legal_zero_frac, add_noise, float_policy)
    (3, 9, 64, 20, 1, 0, 0.0, True, False),
    (3, 9, 64, 20, 5, 1, 0.3, True, False),
    (3, 9, 64, 20, 5, 2, 0.3, False, False),
    (5, 11, 48, 16, 10, 2, 0.2, True, True),
    (2, 3, 8, 25, 5, 0, 0.0, True, True),
    (8, 15, 32, 30, 5, 5, 0.3, True, False),
]


@pytest.mark.gpu
@pytest.mark.parametrize("case", DRIVER_CASES, ids=lambda c: f"N{c[0]}A{c[1]}B{c[2]}S{c[3]}K{c[4]}ag{c[5]}")
def test_driver_matches_oracle_driver(case, port_lib):
    import torch

    from driver import OracleSampledMCTS
    from mazero_amd.mcts_sampled import SampledMCTS
    from mazero_amd.nets import SearchConfig, make_net, make_root_batch

    N, A, B, S, K, cur, zf, noise, fpol = case
    dev = torch.device("cuda", 0)
    cfg = SearchConfig(action_space_size=A, num_simulations=S, sampled_action_times=K)
    net = make_net(N, A, seed=3, device=dev, float_policy=fpol)
    out, legal = make_root_batch(net, B, 64, seed=4, device=dev, legal_zero_frac=zf)
    factor = np.random.default_rng(5).integers(0, A, size=(B, max(cur, 1))).astype(np.int32)[:, :cur] if cur else None
    exp = OracleSampledMCTS(cfg, np.random.RandomState(11), port_lib).batch_search(
        net, out, cur, factor, N, legal, device=dev, add_noise=noise)
    got = SampledMCTS(cfg, np.random.RandomState(11)).batch_search(
        net, out, cur, factor, N, legal, device=dev, add_noise=noise)
    _compare_outputs(got, exp)


@pytest.mark.gpu
def test_driver_device_outputs_and_reuse(port_lib):
    """Back-to-back searches reuse one device arena (reseeded); the device-output form agrees
    with the host form; the np_random stream advances exactly as the reference's."""
    import torch

    from driver import OracleSampledMCTS
    from mazero_amd.mcts_sampled import SampledMCTS
    from mazero_amd.nets import SearchConfig, make_net, make_root_batch

    N, A, B, S = 3, 9, 32, 15
    dev = torch.device("cuda", 0)
    cfg = SearchConfig(action_space_size=A, num_simulations=S, sampled_action_times=3)
    net = make_net(N, A, seed=8, device=dev)
    out, legal = make_root_batch(net, B, 64, seed=9, device=dev, legal_zero_frac=0.2)
    rs_o, rs_d = np.random.RandomState(21), np.random.RandomState(21)
    oracle = OracleSampledMCTS(cfg, rs_o, port_lib)
    drv = SampledMCTS(cfg, rs_d)
    for agent in range(N):  # the self-play agent loop, selfplay_worker.py:196-211
        factor = np.zeros((B, agent), np.int32) if agent else None
        exp = oracle.batch_search(net, out, agent, factor, N, legal, device=dev, add_noise=True)
        if agent == 1:
            dout = drv.batch_search_device(net, out, agent, factor, N, legal, device=dev, add_noise=True)
            got = dout.to_host()
        else:
            got = drv.batch_search(net, out, agent, factor, N, legal, device=dev, add_noise=True)
        _compare_outputs(got, exp)
    assert rs_o.randint(1 << 30) == rs_d.randint(1 << 30)


@pytest.mark.gpu
def test_graph_reuse_keys_on_search_constants(port_lib):
    """Two configurations of one shape that differ only in discount, then only in pb_c_init /
    pb_c_base, searched alternately (eager, capture, replays): every search matches the oracle
    with its own constants (the discount is a recorded kernel argument, the pUCT constants pick the
    device tables, which a replay does not rewrite)."""
    import dataclasses

    import torch

    from driver import OracleSampledMCTS
    from mazero_amd.mcts_sampled import SampledMCTS
    from mazero_amd.nets import SearchConfig, make_net, make_root_batch

    N, A, B, S, cur = 3, 9, 32, 12, 0
    dev = torch.device("cuda", 0)
    base = SearchConfig(action_space_size=A, num_simulations=S, sampled_action_times=3)
    cfgs = [base, dataclasses.replace(base, discount=0.9), dataclasses.replace(base, pb_c_init=2.5, pb_c_base=500.0)]
    net = make_net(N, A, seed=31, device=dev)
    for step in range(3):
        for j, cfg in enumerate(cfgs):
            out, legal = make_root_batch(net, B, 64, seed=200 + 10 * step + j, device=dev, legal_zero_frac=0.2)
            rs_o, rs_d = np.random.RandomState(step), np.random.RandomState(step)
            exp = OracleSampledMCTS(cfg, rs_o, port_lib).batch_search(net, out, cur, None, N, legal, device=dev,
                                                                       add_noise=True)
            got = SampledMCTS(cfg, rs_d).batch_search(net, out, cur, None, N, legal, device=dev, add_noise=True)
            _compare_outputs(got, exp)


@pytest.mark.gpu
def test_graph_after_weights_rehomed(port_lib):
    """A search graph recorded before weights.FlatWeights re-homes the model's parameters is not
    replayed against the freed storage: the next search records a new graph and matches the
    oracle with the re-homed (and then updated) weights."""
    import torch

    from driver import OracleSampledMCTS
    from mazero_amd.mcts_sampled import SampledMCTS
    from mazero_amd.nets import SearchConfig, make_net, make_root_batch
    from mazero_amd.weights import FlatWeights

    N, A, B, S, cur = 3, 9, 32, 12, 1
    dev = torch.device("cuda", 0)
    cfg = SearchConfig(action_space_size=A, num_simulations=S, sampled_action_times=1)
    net = make_net(N, A, seed=41, device=dev)
    factor = np.zeros((B, cur), np.int32)

    def check(step):
        out, legal = make_root_batch(net, B, 64, seed=300 + step, device=dev, legal_zero_frac=0.2)
        rs_o, rs_d = np.random.RandomState(step), np.random.RandomState(step)
        exp = OracleSampledMCTS(cfg, rs_o, port_lib).batch_search(net, out, cur, factor, N, legal, device=dev,
                                                                   add_noise=True)
        got = SampledMCTS(cfg, rs_d).batch_search(net, out, cur, factor, N, legal, device=dev, add_noise=True)
        _compare_outputs(got, exp)

    for step in range(3):  # eager, capture + replay, replay
        check(step)
    flat = FlatWeights(net)  # frees the parameters' old storage
    torch.cuda.empty_cache()
    for step in range(3, 5):
        check(step)
    with torch.no_grad():  # new weights written in place (what a broadcast does)
        for f in flat.tensors():
            f.mul_(0.5)
    for step in range(5, 7):
        check(step)


@pytest.mark.gpu
@pytest.mark.parametrize("K", [1, 5])
def test_driver_graph_replay_matches_oracle(K, port_lib):
    """Repeated searches of one configuration: the first runs eagerly, the second is captured into
    a HIP graph and replayed, later ones replay it -- each with new roots, seed and factor."""
    import torch

    from driver import OracleSampledMCTS
    from mazero_amd.mcts_sampled import SampledMCTS
    from mazero_amd.nets import SearchConfig, make_net, make_root_batch

    N, A, B, S, cur = 3, 9, 64, 20, 1
    dev = torch.device("cuda", 0)
    cfg = SearchConfig(action_space_size=A, num_simulations=S, sampled_action_times=K)
    net = make_net(N, A, seed=12, device=dev)
    rs_o, rs_d = np.random.RandomState(5), np.random.RandomState(5)
    oracle = OracleSampledMCTS(cfg, rs_o, port_lib)
    drv = SampledMCTS(cfg, rs_d, use_graph=True)
    for step in range(6):  # eager, capture + replay, then four pure replays
        out, legal = make_root_batch(net, B, 64, seed=100 + step, device=dev, legal_zero_frac=0.25)
        factor = np.random.default_rng(step).integers(0, A, size=(B, cur)).astype(np.int32)
        exp = oracle.batch_search(net, out, cur, factor, N, legal, device=dev, add_noise=True)
        got = drv.batch_search(net, out, cur, factor, N, legal, device=dev, add_noise=True)
        _compare_outputs(got, exp)


@pytest.mark.gpu
def test_driver_inside_caller_autocast(port_lib):
    """batch_search called inside the caller's own autocast context (the search loop then keeps the
    casts per simulation: a cast cache would outlive the loop and its capture): eager, captured and
    replayed searches equal the oracle driver's."""
    import torch

    from driver import OracleSampledMCTS
    from mazero_amd.mcts_sampled import SampledMCTS
    from mazero_amd.nets import SearchConfig, make_net, make_root_batch

    N, A, B, S, cur = 3, 9, 32, 12, 0
    dev = torch.device("cuda", 0)
    cfg = SearchConfig(action_space_size=A, num_simulations=S, sampled_action_times=1)
    net = make_net(N, A, seed=21, device=dev)
    rs_o, rs_d = np.random.RandomState(9), np.random.RandomState(9)
    oracle = OracleSampledMCTS(cfg, rs_o, port_lib)
    drv = SampledMCTS(cfg, rs_d, use_graph=True)
    for step in range(4):
        out, legal = make_root_batch(net, B, 64, seed=300 + step, device=dev, legal_zero_frac=0.2)
        exp = oracle.batch_search(net, out, cur, None, N, legal, device=dev, add_noise=True)
        with torch.autocast("cuda"):
            got = drv.batch_search(net, out, cur, None, N, legal, device=dev, add_noise=True)
        _compare_outputs(got, exp)


@pytest.mark.gpu
def test_graph_replay_after_eager_launches(port_lib):
    """A captured search graph replayed after thousands of ordinary launches (eager searches of the
    same configuration, then the oracle's eager network calls) still matches the oracle, under the
    HIP runtime's default graph packet capture.  In round 1 this sequence failed in agent 1's
    replay: the graph then held a hipMemsetAsync node (clearing the error word), and under packet
    capture a replayed memset node wrote a stale fill pattern (0x78787878) once enough ordinary
    work had run (scripts/memset_graph_repro.py).  Captured paths now set words with a kernel."""
    import torch

    from consume import eps_greedy_given, select_action
    from driver import OracleSampledMCTS
    from mazero_amd.mcts_sampled import SampledMCTS
    from mazero_amd.nets import SearchConfig, make_net, make_root_batch

    N, A, B, S = 3, 9, 256, 50
    dev = torch.device("cuda", 0)
    cfg = SearchConfig(action_space_size=A, num_simulations=S, sampled_action_times=1)
    net = make_net(N, A, seed=0, device=dev)
    roots = [make_root_batch(net, B, 64, seed=10 + i, device=dev, legal_zero_frac=0.2) for i in range(3)]
    for n_steps, use_graph in ((7, True), (3, False)):  # graph captures + replays, then eager searches
        m = SampledMCTS(cfg, np.random.RandomState(0), use_graph=use_graph)
        for i in range(n_steps):
            out, legal = roots[i % 3]
            acts = np.zeros((B, N), np.int32)
            for agent in range(N):
                r = m.batch_search(net, out, agent, acts[:, :agent].copy() if agent else None, N, legal, device=dev,
                                   add_noise=True)
                acts[:, agent] = [int(a[np.argmax(v), 0]) for a, v in zip(r.sampled_actions, r.sampled_visit_count)]
    # a self-play step: per agent the oracle driver first (eager network calls on the device), then
    # the graph replay of the device driver on the same inputs
    ur = np.random.default_rng(1)
    u_eps, u_cat = ur.random((N, B)).astype(np.float32), ur.random((N, B))
    rs_o, rs_d = np.random.default_rng(3), np.random.default_rng(3)
    oracle, drv = OracleSampledMCTS(cfg, rs_o, port_lib), SampledMCTS(cfg, rs_d)
    out, legal = roots[0]
    acts = np.full((B, N), -1, np.int32)
    for agent in range(N):
        fac = acts[:, :agent].copy() if agent else None
        exp = oracle.batch_search(net, out, agent, fac, N, legal, device=dev, add_noise=True)
        got = drv.batch_search(net, out, agent, fac, N, legal, device=dev, add_noise=True)
        _compare_outputs(got, exp)
        for i in range(B):
            select_action(exp["sampled_visit_count"][i], 1.0, False, rs_o)
            pos, _ = select_action(got.sampled_visit_count[i], 1.0, False, rs_d)
            acts[i, agent] = eps_greedy_given(got.sampled_actions[i][pos, 0], legal[i, agent], 0.1,
                                              u_eps[agent, i], u_cat[agent, i])
    assert rs_o.random() == rs_d.random()


@pytest.mark.gpu
def test_captured_memset_node_keeps_loop_eager(port_lib):
    """A model whose forward records a runtime memset node into the captured search loop (here a
    hipMemsetAsync through ctypes on the capture stream, as a BLAS workspace clear would) is never
    replayed: under the HIP runtime's packet capture a replayed memset node can write a stale fill
    (DESIGN.md §7).  The census of the recorded graph (mz_graph_census) finds it, the search warns
    and runs eagerly, and every search still matches the oracle.  The same loop without the memset
    records a graph with no memset node and replays it."""
    import torch

    from driver import OracleSampledMCTS
    from mazero_amd.mcts_sampled import _LOOPS, SampledMCTS
    from mazero_amd.nets import SearchConfig, make_net, make_root_batch

    N, A, B, S, cur = 3, 9, 32, 10, 0
    dev = torch.device("cuda", 0)
    cfg = SearchConfig(action_space_size=A, num_simulations=S, sampled_action_times=1)
    hip = C.CDLL("libamdhip64.so.7")
    hip.hipMemsetAsync.argtypes = [C.c_void_p, C.c_int, C.c_size_t, C.c_void_p]
    scratch = torch.empty(64, dtype=torch.int32, device=dev)

    def loop_of(net):
        return [v for v in _LOOPS.values() if v.model_ref() is net][0]

    for with_memset in (False, True):
        net = make_net(N, A, seed=51, device=dev)
        if with_memset:
            dyn = net.dynamics

            def dynamics(h, a, dyn=dyn):
                st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
                assert hip.hipMemsetAsync(C.c_void_p(scratch.data_ptr()), 0, 256, st) == 0
                return dyn(h, a)

            net.dynamics = dynamics
        rs_o, rs_d = np.random.RandomState(7), np.random.RandomState(7)
        oracle, drv = OracleSampledMCTS(cfg, rs_o, port_lib), SampledMCTS(cfg, rs_d)
        for step in range(3):  # eager, capture (+ replay or eager), again
            out, legal = make_root_batch(net, B, 64, seed=400 + step, device=dev, legal_zero_frac=0.2)
            exp = oracle.batch_search(net, out, cur, None, N, legal, device=dev, add_noise=True)
            if with_memset and step == 1:
                with pytest.warns(RuntimeWarning, match="memset"):
                    got = drv.batch_search(net, out, cur, None, N, legal, device=dev, add_noise=True)
            else:
                got = drv.batch_search(net, out, cur, None, N, legal, device=dev, add_noise=True)
            _compare_outputs(got, exp)
        lp = loop_of(net)
        nodes, memsets = lp.graph_nodes
        assert nodes > 2 * S
        if with_memset:
            assert memsets == S and lp.graph is False
        else:
            assert memsets == 0 and isinstance(lp.graph, torch.cuda.CUDAGraph)


@pytest.mark.gpu
def test_agent_loops_share_one_pool(port_lib):
    """A 27-agent self-play step at K = 5 (27m-shaped: 27 agents x 36 actions, H = 128 per agent)
    holds ONE hidden-state pool [S+1, B, N*H] for its 27 agent loops, not one per loop (round 4
    held ~19 GB at 256 x 200); a second root count adds one pool of its own; release() frees both.
    The reference frees its pool after every search (mcts_sampled.py:86,89).  Agents 0, 1 and 26
    are checked against the oracle driver bit for bit."""
    import gc

    import torch

    from driver import OracleSampledMCTS
    from mazero_amd import mcts_sampled as ms
    from mazero_amd.nets import SearchConfig, make_net, make_root_batch

    N, A, S, K = 27, 36, 60, 5
    dev = torch.device("cuda", 0)
    cfg = SearchConfig(action_space_size=A, num_simulations=S, sampled_action_times=K)
    net = make_net(N, A, seed=61, device=dev)
    ms.release()
    gc.collect()
    torch.cuda.synchronize()

    def pool_bytes(B):  # (the pool's dtype is the network's output dtype under autocast: float16 here)
        pools = [v.pool for v in ms._LOOPS.values() if v.pool is not None and v.pool.shape[1] == B]
        assert pools, B
        assert pools[0].shape == (S + 1, B, N * net.hidden)
        return pools[0].nbytes

    def step(B):
        out, legal = make_root_batch(net, B, 64, seed=B, device=dev, legal_zero_frac=0.2)
        rs_o, rs_d = np.random.RandomState(B), np.random.RandomState(B)
        oracle, drv = OracleSampledMCTS(cfg, rs_o, port_lib), ms.SampledMCTS(cfg, rs_d)
        acts = np.zeros((B, N), np.int32)
        mem = []
        for agent in range(N):
            fac = acts[:, :agent].copy() if agent else None
            got = drv.batch_search(net, out, agent, fac, N, legal, device=dev, add_noise=True)
            if agent in (0, 1, N - 1):
                exp = oracle.batch_search(net, out, agent, fac, N, legal, device=dev, add_noise=True)
                _compare_outputs(got, exp)
            else:  # (the oracle's np_random must advance as the driver's)
                rs_o.set_state(rs_d.get_state())
            acts[:, agent] = [int(a[np.argmax(v), 0]) for a, v in zip(got.sampled_actions, got.sampled_visit_count)]
            torch.cuda.synchronize()
            mem.append(torch.cuda.memory_allocated())
        return mem

    base = torch.cuda.memory_allocated()
    m1 = step(256)
    assert m1[0] - base >= pool_bytes(256)  # the first loop made the pool
    # ... and the 26 other loops share it (their own buffers are [B, N*H] each)
    assert m1[-1] - m1[0] < pool_bytes(256), (m1[0], m1[-1], pool_bytes(256))
    m2 = step(128)
    assert m2[-1] - m1[-1] < pool_bytes(128) + pool_bytes(256), (m1[-1], m2[-1])
    assert len({id(v.pool_ref) for v in ms._LOOPS.values() if v.pool_ref is not None}) == 2
    import weakref

    pools = [weakref.ref(v.pool) for v in ms._LOOPS.values() if v.pool is not None]
    assert pools
    ms.release()
    gc.collect()
    assert all(r() is None for r in pools)  # release() freed every pool
    ms.release()  # (the handles' arenas, returned to the library's cache when they died: freed)
    from mazero_amd._lib import trim_caches

    assert trim_caches() == 0


# ------------------------------------------------------------------------------------------------
# Reference-driver fixtures (oracle/gen_driver_golden.py: core/mcts/tree_search/mcts_sampled.py
# itself, imported in the build container, over the reference ctree)
# ------------------------------------------------------------------------------------------------
from driver_fixture import DriverFixture, ReplayNet, driver_fixtures  # noqa: E402

_DRIVER_FX = driver_fixtures()
_fx_id = lambda p: os.path.basename(p)[7:-4]  # noqa: E731


def test_driver_fixtures_present():
    assert len(_DRIVER_FX) >= 6, "tests/golden/driver_*.npz missing (python oracle/gen_driver_golden.py)"


def _u32(a):
    a = np.asarray(a)
    return a.view(np.uint32) if a.dtype == np.float32 else a


@pytest.mark.parametrize("path", _DRIVER_FX, ids=_fx_id)
def test_root_inputs_match_reference_driver(path):
    """The product's host-side root preprocessing (SampledMCTS.root_inputs) against the arguments
    the reference driver passed to prepare (mcts_sampled.py:64-106) and the tree seed it drew
    (:89), bit for bit, and the generator consumed identically."""
    import torch

    from mazero_amd.mcts_sampled import SampledMCTS

    fx = DriverFixture(path)
    z = fx.z
    rng = fx.np_random()
    (rr, rv, rp, rb, eps, rn), seed = SampledMCTS(fx.config(), rng).root_inputs(
        fx.root_output(torch.device("cpu")), fx.agent, fx.legal, fx.meta["add_noise"], 1.0)
    assert seed == fx.meta["tree"]["seed"]
    assert eps == float(z["prep_eps"])
    for got, key in ((rr, "prep_rewards"), (rv, "prep_values"), (rp, "prep_probs"), (rb, "prep_beta"),
                     (rn, "prep_noises")):
        exp = z[key]
        assert got.dtype == exp.dtype and got.shape == exp.shape, key
        np.testing.assert_array_equal(_u32(got), _u32(exp), err_msg=key)


@pytest.mark.parametrize("tree", ["port", "ref"])
@pytest.mark.parametrize("path", _DRIVER_FX, ids=_fx_id)
def test_oracle_driver_matches_reference_driver(path, tree, request):
    """oracle/driver.py (the restatement every GPU driver test checks against) reproduces the
    reference driver's run: the tree calls of every simulation, the network's inputs, the
    SearchOutput and the generator state afterwards."""
    import types

    import torch

    from driver import OracleSampledMCTS

    lib = request.getfixturevalue("port_lib" if tree == "port" else "ref_lib")
    fx = DriverFixture(path)
    z = fx.z
    cpu = torch.device("cpu")
    net = ReplayNet(fx, cpu)
    rng = fx.np_random()
    drv = OracleSampledMCTS(fx.config(), rng, lib, record=True)
    res = drv.batch_search(net, fx.root_output(cpu), fx.agent, fx.factor, fx.N, fx.legal, device=cpu,
                           add_noise=fx.meta["add_noise"])
    net.check_inputs()
    for s, t in enumerate(drv.trace):
        np.testing.assert_array_equal(t["idx"], z["sel_idx"][s], err_msg=f"idx_x sim {s}")
        np.testing.assert_array_equal(t["act"], z["sel_act"][s].reshape(-1), err_msg=f"action sim {s}")
        for k in ("reward", "value", "probs", "beta"):
            np.testing.assert_array_equal(_u32(t[k]).reshape(-1), _u32(z["exp_" + k][s]).reshape(-1),
                                          err_msg=f"{k} sim {s}")
    _compare_outputs(types.SimpleNamespace(**res), fx.expected())
    np.testing.assert_array_equal(np.asarray(rng.random(4)), z["rng_after"])


@pytest.mark.gpu
@pytest.mark.parametrize("device_root", [True, False], ids=["device_root", "host_root"])
@pytest.mark.parametrize("path", _DRIVER_FX, ids=_fx_id)
def test_device_driver_matches_reference_driver(path, device_root):
    """mazero_amd.mcts_sampled.SampledMCTS, fed the reference network's recorded outputs,
    reproduces the reference driver's search bit for bit: the leaf rows it gathers and the joint
    actions it builds (the network's inputs), every SearchOutput field and the np_random state
    after the search -- eagerly, then captured into a HIP graph and replayed, then replayed again."""
    import torch

    from mazero_amd.mcts_sampled import _LOOPS, SampledMCTS

    fx = DriverFixture(path)
    dev = torch.device("cuda", 0)
    net = ReplayNet(fx, dev)
    root = fx.root_output(dev)
    for run in range(3):  # eager, capture + replay, replay
        net.reset()
        rng = fx.np_random()
        got = SampledMCTS(fx.config(), rng, device_root=device_root).batch_search(
            net, root, fx.agent, fx.factor, fx.N, fx.legal, device=dev, add_noise=fx.meta["add_noise"])
        torch.cuda.synchronize()
        net.check_inputs()
        _compare_outputs(got, fx.expected())
        np.testing.assert_array_equal(np.asarray(rng.random(4)), fx.z["rng_after"])
    loop = [v for v in _LOOPS.values() if v.model_ref() is net and (v.root_mode is not None) == device_root][0]
    assert isinstance(loop.graph, torch.cuda.CUDAGraph), "the third search did not replay a graph"


@pytest.mark.gpu
def test_graph_census_counts_child_graph_memsets():
    """mz_graph_census recurses into child-graph nodes: a memset node nested one level down (as a
    nested capture or an embedded graph records it) is counted, so such a search loop stays eager."""
    import torch

    from mazero_amd._capi import check
    from mazero_amd._lib import load

    class MemsetParams(C.Structure):  # hipMemsetParams (hip_runtime_api.h)
        _fields_ = [("dst", C.c_void_p), ("elementSize", C.c_uint), ("height", C.c_size_t), ("pitch", C.c_size_t),
                    ("value", C.c_uint), ("width", C.c_size_t)]

    lib = load()
    hip = C.CDLL("libamdhip64.so.7")
    buf = torch.zeros(64, dtype=torch.int32, device="cuda")
    child, parent, node, cnode = C.c_void_p(), C.c_void_p(), C.c_void_p(), C.c_void_p()
    assert hip.hipGraphCreate(C.byref(child), 0) == 0
    assert hip.hipGraphCreate(C.byref(parent), 0) == 0
    prm = MemsetParams(buf.data_ptr(), 4, 1, 0, 0, 64)
    assert hip.hipGraphAddMemsetNode(C.byref(node), child, None, C.c_size_t(0), C.byref(prm)) == 0
    assert hip.hipGraphAddChildGraphNode(C.byref(cnode), parent, None, C.c_size_t(0), child) == 0
    total, memsets = C.c_int(0), C.c_int(0)
    check(lib, lib.mz_graph_census(parent, C.byref(total), C.byref(memsets)), "graph_census")
    assert (total.value, memsets.value) == (2, 1)
    hip.hipGraphDestroy(parent)
    hip.hipGraphDestroy(child)


# ------------------------------------------------------------------------------------------------
# Device root preprocessing (mz_root_glue)
# ------------------------------------------------------------------------------------------------
def _round_d2h_restated(d: np.ndarray) -> np.ndarray:
    """mzdriver.hip round_d2h, line by line on uint64 bit patterns: float64 -> float16 with one
    rounding (ties to even).  Returns the float16 bit patterns."""
    b = np.asarray(d, np.float64).view(np.uint64)
    out = np.empty(b.shape, np.uint16)
    for i, v in enumerate(b.reshape(-1).tolist()):
        sign = (v >> 48) & 0x8000
        ex = (v >> 52) & 0x7FF
        mant = v & 0xFFFFFFFFFFFFF
        if ex == 0x7FF:
            h = sign | 0x7C00 | (0x200 if mant else 0)
        elif ex == 0:
            h = sign
        else:
            e = ex - 1023 + 15
            m = (1 << 52) | mant
            shift = 42 if e >= 1 else 42 + (1 - e)
            if shift >= 64:
                h = sign
            else:
                q = m >> shift
                rem, half = m & ((1 << shift) - 1), 1 << (shift - 1)
                if rem > half or (rem == half and (q & 1)):
                    q += 1
                if e >= 1:
                    if q == (1 << 11):
                        q >>= 1
                        e += 1
                    h = (sign | 0x7C00) if e >= 31 else (sign | (e << 10) | (q & 0x3FF))
                else:
                    h = sign | q
        out.reshape(-1)[i] = h
    return out


def test_double_to_half_rounding_restatement():
    """The kernel's float64 -> float16 rounding equals numpy's astype(float16) (one rounding), on
    random values over half's whole range, its subnormals, the overflow boundary and exact ties."""
    rng = np.random.default_rng(0)
    xs = [
        rng.standard_normal(20000) * 10.0 ** rng.integers(-9, 6, 20000),
        rng.random(5000) * 2.0 ** -14,                     # half subnormals
        65504.0 + rng.random(3000) * 40.0,                  # overflow boundary (65520 rounds to inf)
        (np.arange(-2048, 2048) + 0.5) * 2.0 ** -10,        # ties at many binades
        (np.arange(1, 2000) + 0.5) * 2.0 ** -24,            # subnormal ties
        np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1e-300, -1e-300, 2.0 ** -25, 3 * 2.0 ** -26, 1e-4, 6e-5]),
    ]
    for x in xs:
        x = x.astype(np.float64)
        got = _round_d2h_restated(x)
        exp = x.astype(np.float16).view(np.uint16)
        nan = np.isnan(x)
        np.testing.assert_array_equal(got[~nan], exp[~nan])
        assert np.all((got[nan] & 0x7C00) == 0x7C00) and np.all(got[nan] & 0x3FF)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["float32", "float16"])
@pytest.mark.parametrize("A", [3, 9, 15, 36, 64])
def test_root_glue_matches_host_root_inputs(dtype, A):
    """mz_root_glue against the host root preprocessing (SampledMCTS.root_inputs, the reference's
    numpy expressions, pinned to the reference driver by the driver_*.npz fixtures), bit for bit:
    legal masks as int64 and bool with zeros, none; noise on and off; extreme logits."""
    import torch

    from mazero_amd._capi import MZ_DT_F16, MZ_DT_F32, check
    from mazero_amd.mcts_sampled import SampledMCTS
    from mazero_amd.nets import NetworkOutput, SearchConfig

    B, N, cur = 300, 3, 1
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(A)
    tb = _handle(B, A)
    cfg = SearchConfig(action_space_size=A)
    for legal_kind in ("none", "int64", "bool"):
        for noise in (True, False):
            logits = (rng.standard_normal((B, N, A)) * rng.choice([0.1, 1, 4, 30], size=(B, 1, 1))).astype(dtype)
            logits[:5, cur, 1 % A] = 60.0  # one dominant logit
            legal = None
            if legal_kind != "none":
                legal = (rng.random((B, N, A)) >= 0.3).astype(np.int64)
                legal[..., 0] = np.where(legal.sum(-1) == 0, 1, legal[..., 0])
                if legal_kind == "bool":
                    legal = legal.astype(bool)
            out = NetworkOutput(torch.zeros(B, 4, device=dev), rng.standard_normal((B, 1)).astype(np.float32),
                                rng.standard_normal((B, 1)).astype(np.float32), logits)
            seed = int(rng.integers(1 << 30))
            m_host, m_dev = SampledMCTS(cfg, np.random.RandomState(seed)), SampledMCTS(cfg, np.random.RandomState(seed))
            (rr, rv, rp, rb, eps, rn), seed_h = m_host.root_inputs(out, cur, legal, noise, 1.0)
            arrays, mode, eps_d, seed_d = m_dev.root_raw(out, cur, legal, noise)
            assert seed_d == seed_h and eps_d == eps and mode == (MZ_DT_F16 if dtype == "float16" else MZ_DT_F32,
                                                                  legal is not None)
            t = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in arrays.items()}
            probs, beta, nz = (torch.empty(B, A, device=dev) for _ in range(3))
            tb._sync_stream()
            lg = t.get("legal")
            rc = tb._lib.mz_root_glue(tb._h, C.c_void_p(t["logits"].data_ptr()), mode[0], A, 0,
                                      None if lg is None else C.c_void_p(lg.data_ptr()), A,
                                      C.c_void_p(t["noise"].data_ptr()), float(eps_d), 1.0,
                                      C.c_void_p(probs.data_ptr()), C.c_void_p(beta.data_ptr()),
                                      C.c_void_p(nz.data_ptr()))
            check(tb._lib, rc, "root_glue")
            where = f"{dtype} A={A} legal={legal_kind} noise={noise}"
            for got, exp, name in ((probs, rp, "probs"), (beta, rb, "beta"), (nz, rn, "noises")):
                np.testing.assert_array_equal(got.cpu().numpy().view(np.uint32), exp.reshape(B, A).view(np.uint32),
                                              err_msg=f"{name} {where}")
            np.testing.assert_array_equal(arrays["rewards"], rr)
            np.testing.assert_array_equal(arrays["values"], rv)


def test_wide_action_space_refused_at_construction():
    """the device driver glue takes one lane per action (A <= 64); SampledMCTS
    refuses a wider action space in its constructor, before any search launches (CPU: no device
    call is made), while the drop-in Tree_batch takes A <= 255."""
    from mazero_amd.mcts_sampled import MAX_GLUE_ACTIONS, SampledMCTS
    from mazero_amd.nets import SearchConfig

    with pytest.raises(RuntimeError, match="action_space_size 65"):
        SampledMCTS(SearchConfig(action_space_size=MAX_GLUE_ACTIONS + 1))
    SampledMCTS(SearchConfig(action_space_size=MAX_GLUE_ACTIONS))
