"""Seeded random small search configurations shared by the fuzz parity tests: the GPU against
the CPU port (tests/test_gpu_parity.py) and the port against the reference ctree
(tests/test_oracle.py), so the two comparisons cover the same cases."""
from __future__ import annotations

import numpy as np


def fuzz_configs(seed: int, n: int):
    """Seeded random small configurations across the kernels' classes and the search knobs (A up to
    255: past 64 actions the wide expansion and k_hbm)."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        A = int(rng.choice([1, 2, 3, 5, 9, 11, 15, 16, 17, 36, 63, 64, 65, 130, 255]))
        K = int(rng.choice([1, 1, 2, 3, 5, 8, 10, 33, 64, 70]))
        S = int(rng.integers(1, 61))
        B = int(rng.integers(1, 49))
        knobs = dict(discount=float(rng.choice([0.997, 0.9, 1.0])), rho=float(rng.choice([0.75, 0.5, 0.0])),
                     lam=float(rng.choice([0.8, 1.0, 0.5])), delta_lb=float(rng.choice([0.01, 0.1])),
                     pb_c_init=float(rng.choice([1.25, 2.5])), pb_c_base=float(rng.choice([19652.0, 500.0])))
        lz = float(rng.choice([0.0, 0.3])) if A >= 2 else 0.0
        ties = bool(rng.random() < 0.15)
        eps = float(rng.choice([0.0, 0.25]))
        out.append((B, A, K, S, knobs, lz, ties, eps, int(rng.integers(1 << 30))))
    return out


def fuzz_configs_large(seed: int, n: int):
    """Seeded random configurations at SMAC-like sizes (S 60-300, B 64-512): the larger layout
    classes of the chain and tree kernels and the general kernel."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        A = int(rng.choice([5, 9, 11, 14, 17, 36, 64, 100]))
        K = int(rng.choice([1, 1, 2, 3, 5, 8, 10, 16]))
        S = int(rng.integers(60, 301))
        B = int(rng.integers(64, 513))
        knobs = dict(discount=float(rng.choice([0.997, 0.99])), rho=float(rng.choice([0.75, 0.5])),
                     lam=float(rng.choice([0.8, 1.0])), delta_lb=0.01, pb_c_init=1.25, pb_c_base=19652.0)
        lz = float(rng.choice([0.0, 0.3]))
        eps = float(rng.choice([0.0, 0.25]))
        out.append((B, A, K, S, knobs, lz, False, eps, int(rng.integers(1 << 30))))
    return out
