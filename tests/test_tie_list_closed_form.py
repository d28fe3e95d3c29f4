"""The selection's tie list in closed form, as the kernels compute it, against the reference's
sequential arg-max (select_child, cnode.cpp:355-370):

    max = FLOAT_MIN; for i: if max < s_i: max = s_i, list = [i]  elif s_i >= max - 1e-6: list += [i]

k_tree's level walk and its precomputed tie lists for nodes of up to eight children
(tree_select_prep, mzmcts.hip) use instead: M = the maximum, r = its first index,
list = [r] + [i > r : s_i >= M - 1e-6]; when M <= FLOAT_MIN, list = [i : s_i >= FLOAT_MIN].
This checks the identity in float32 over random, tied, signed-zero, FLOAT_MIN-adjacent, infinite
and NaN scores (host logic only; the kernels themselves are pinned by the -m gpu parity tests)."""
import numpy as np

F = np.float32
FLOAT_MIN = F(-1000000.0)
EPS = F(0.000001)


def sequential(s):
    mx, lst = FLOAT_MIN, []
    for i, v in enumerate(s):
        if mx < v:
            mx, lst = v, [i]
        elif v >= F(mx - EPS):
            lst.append(i)
    return lst


def closed_form(s):
    finite = [v for v in s if not np.isnan(v)]
    M = max(finite) if finite else F(np.nan)  # fmaxf: a NaN operand yields the other
    if M > FLOAT_MIN:
        r = next(i for i, v in enumerate(s) if v == M)
        thr = F(M - EPS)
        return [r] + [i for i in range(r + 1, len(s)) if s[i] >= thr]
    return [i for i, v in enumerate(s) if v >= FLOAT_MIN]


def test_closed_form_equals_sequential():
    rng = np.random.default_rng(7)
    specials = np.array([0.0, -0.0, 1.0, 1.0 + 5e-7, 1.0 - 5e-7, -1e6, -999999.94, -2e6, np.inf, -np.inf, np.nan],
                        dtype=F)
    for trial in range(20000):
        n = int(rng.integers(1, 9))
        kind = trial % 4
        if kind == 0:
            s = rng.random(n, dtype=F)
        elif kind == 1:  # ties and near-ties around a common value
            s = (F(0.5) + rng.integers(-2, 3, n).astype(F) * F(4e-7)).astype(F)
        elif kind == 2:
            s = rng.choice(specials, n)
        else:
            s = np.where(rng.random(n) < 0.5, rng.choice(specials, n), rng.random(n, dtype=F)).astype(F)
        s = [F(v) for v in s]
        assert closed_form(s) == sequential(s), s
