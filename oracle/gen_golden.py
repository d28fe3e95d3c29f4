"""ORACLE — TEST INFRASTRUCTURE ONLY.  Records the golden vectors under tests/golden/.

Runs in the build container (it needs oracle/_ref/libmzref.so, the reference ctree compiled from
/root/reference by oracle/Makefile) and writes:

  tests/golden/trace_<name>.npz     every Tree_batch call of one synthetic search: the inputs
                                    (root prepare + per-simulation network outputs + tree seed +
                                    knobs) and the reference's outputs (selection idx/action per
                                    simulation, root value and marginal visit counts after every
                                    simulation, all final readbacks)
  tests/golden/kat_libstdcxx.json   libstdc++ mt19937 / discrete_distribution known answers
                                    (oracle/kat_libstdcxx.cpp) + glibc logf pUCT table entries
  tests/golden/full_<name>.npz      (--full) searches at the BASELINE sizes: the generator seed and
                                    the SHA-256 of the inputs it yields (synthetic.inputs_digest;
                                    the inputs themselves are regenerated, not stored), the
                                    reference's selection idx/action of every simulation and all
                                    final readbacks

Usage:  make -C oracle && python oracle/gen_golden.py [--full] [--only name,name]
"""
from __future__ import annotations

import ctypes as C
import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)

from mazero_amd import _capi  # noqa: E402
from mazero_amd.cytree import Tree_batch  # noqa: E402
from mazero_amd.synthetic import (DEFAULTS, inputs_digest, make_deep_window_inputs, make_search_inputs,  # noqa: E402
                                  run_search)

GOLDEN = os.path.join(ROOT, "tests", "golden")

# name: (B, A, K, S, noise_eps, legal_zero_frac, ties, knob overrides)
CONFIGS = {
    "matrix_k1": (8, 3, 1, 25, 0.25, 0.0, False, {}),
    "matrix_k5": (8, 3, 5, 25, 0.25, 0.0, False, {}),
    "3m_k1": (16, 9, 1, 50, 0.25, 0.0, False, {}),
    "3m_k5": (16, 9, 5, 50, 0.25, 0.0, False, {}),
    "3m_k10_legal": (16, 9, 10, 50, 0.25, 0.3, False, {}),
    "3s5z_k5_nonoise": (8, 15, 5, 50, 0.0, 0.0, False, {}),
    "3s5z_k10_legal": (8, 15, 10, 40, 0.25, 0.3, False, {}),
    "ties_a3_k10": (8, 3, 10, 30, 0.25, 0.0, True, {}),
    "ties_a9_k5": (8, 9, 5, 50, 0.0, 0.0, True, {}),
    "a1_k3": (4, 1, 3, 10, 0.25, 0.0, False, {}),
    "k_gt_a": (8, 3, 20, 20, 0.25, 0.0, False, {}),
    "deep_k1_s100": (4, 9, 1, 100, 0.25, 0.0, False, {}),
    "27m_k5_s70": (4, 36, 5, 70, 0.25, 0.3, False, {}),
    "27m_k40": (4, 36, 40, 30, 0.25, 0.0, False, {}),
    "knobs_rho03": (8, 9, 5, 50, 0.25, 0.0, False, dict(rho=0.3, lam=0.9, delta_lb=0.05)),
    "knobs_rho0": (8, 9, 3, 40, 0.25, 0.0, False, dict(rho=0.0, lam=1.0, discount=0.99)),
    # pools whose LDS image exceeds a CU's 160 KB (round 5: k_hbm; refused at construction before)
    "big_a64_k70_s60": (3, 64, 70, 60, 0.25, 0.3, False, {}),
    "big_27m_k16_s200": (2, 36, 16, 200, 0.25, 0.0, False, {}),
    # action spaces past one lane per action (round 5: expand_wide, k_hbm; refused before)
    "wide_a100_k5": (4, 100, 5, 40, 0.25, 0.3, False, {}),
    "wide_a255_k300": (2, 255, 300, 12, 0.25, 0.0, False, {}),
    # one deep path per tree with a tie at its bottom (synthetic.make_deep_window_inputs, round 6):
    # selections and next-expansion words past k_tree's 256-word LDS window of the engine stream;
    # 383 nodes (k_tree<384>) and 603 (k_tree<1024>, the level walk)
    "deep_window_k64_s190": (8, 2, 64, 190, 0.0, 0.0, "deep", {}),
    "deep_window_k64_s300": (4, 2, 64, 300, 0.0, 0.0, "deep", {}),
}


# BASELINE.json sizes: name: (B, A, K, S, noise_eps, legal_zero_frac, ties)
FULL = {
    "3m_k1": (256, 9, 1, 50, 0.25, 0.0, False),
    "3m_k5": (256, 9, 5, 50, 0.25, 0.0, False),
    "3m_k10": (256, 9, 10, 50, 0.25, 0.0, False),
    "3m_k5_ties": (256, 9, 5, 50, 0.25, 0.0, True),
    "2s3z_k1": (1024, 11, 1, 50, 0.25, 0.0, False),
    "2s3z_k5": (1024, 11, 5, 50, 0.25, 0.0, False),
    "3s5z_k5": (512, 15, 5, 100, 0.25, 0.0, False),
    "3s5z_k10": (512, 15, 10, 100, 0.25, 0.0, False),
    "3s5z_k5_legal30": (512, 15, 5, 100, 0.25, 0.3, False),
    "27m_k1": (256, 36, 1, 200, 0.25, 0.0, False),
    "27m_k5": (256, 36, 5, 200, 0.25, 0.0, False),
}


def full_inputs(name, seed):
    B, A, K, S, eps, lz, ties = FULL[name]
    return make_search_inputs(np.random.default_rng(seed), B, A, S, noise_eps=eps, legal_zero_frac=lz, ties=ties), K


def record_full(lib, name, seed):
    inp, K = full_inputs(name, seed)
    tb = Tree_batch(inp.B, 1, inp.A, K, inp.S, DEFAULTS["delta_lb"], inp.seed, DEFAULTS["rho"], DEFAULTS["lam"],
                    lib=lib)
    out = run_search(tb, inp, K, per_sim=False)
    arrays = dict(
        cfg=np.array([inp.B, inp.A, K, inp.S, inp.seed], np.int64),
        gen_seed=np.array([seed], np.int64),
        gen_args=np.array(FULL[name][4:7], np.float64),  # noise_eps, legal_zero_frac, ties
        inputs_sha256=np.frombuffer(bytes.fromhex(inputs_digest(inp)), np.uint8),
    )
    for k, v in out.items():
        arrays["out_" + k] = v
    path = os.path.join(GOLDEN, f"full_{name}.npz")
    np.savez_compressed(path, **arrays)
    return path


def record(lib, name, cfg, seed):
    B, A, K, S, eps, lz, ties, over = cfg
    knobs = dict(DEFAULTS)
    knobs.update(over)
    rng = np.random.default_rng(seed)
    if ties == "deep":
        inp = make_deep_window_inputs(rng, B, S, A)
    else:
        inp = make_search_inputs(rng, B, A, S, noise_eps=eps, legal_zero_frac=lz, ties=ties)
    tb = Tree_batch(B, 1, A, K, S, knobs["delta_lb"], inp.seed, knobs["rho"], knobs["lam"], lib=lib)
    out = run_search(tb, inp, K, knobs)
    arrays = dict(
        cfg=np.array([B, A, K, S, inp.seed], np.int64),
        knobs=np.array(
            [knobs[k] for k in ("pb_c_base", "pb_c_init", "discount", "delta_lb", "rho", "lam")] + [eps], np.float64
        ),
        in_root_reward=inp.root_reward,
        in_root_value=inp.root_value,
        in_root_policy=inp.root_policy,
        in_root_beta=inp.root_beta,
        in_root_noise=inp.root_noise,
        in_reward=inp.reward,
        in_value=inp.value,
        in_policy=inp.policy,
        in_beta=inp.beta,
    )
    for k, v in out.items():
        arrays["out_" + k] = v
    path = os.path.join(GOLDEN, f"trace_{name}.npz")
    np.savez_compressed(path, **arrays)
    return path


def kat():
    exe = os.path.join(HERE, "_build", "kat_libstdcxx")
    data = json.loads(subprocess.check_output([exe]).decode())
    libm = C.CDLL("libm.so.6")
    libm.logf.restype = C.c_float
    libm.logf.argtypes = [C.c_float]
    table = []
    for c2, c1 in ((19652.0, 1.25), (1.0, 0.5), (500.0, 2.0)):
        c2f, c1f = np.float32(c2), np.float32(c1)
        for n in (0, 1, 2, 7, 49, 50, 51, 199, 200, 1000):
            x = np.float32(np.float32(n) + c2f)
            x = np.float32(x + np.float32(1.0))
            x = np.float32(x / c2f)
            v = np.float32(np.float32(libm.logf(float(x))) + c1f)
            table.append([c2, c1, n, int(np.float32(v).view(np.uint32))])
    data["pbc_logf_bits"] = table
    with open(os.path.join(GOLDEN, "kat_libstdcxx.json"), "w") as f:
        json.dump(data, f)


def main():
    os.makedirs(GOLDEN, exist_ok=True)
    lib = _capi.bind(C.CDLL(os.path.join(HERE, "_ref", "libmzref.so")))
    assert lib.mz_backend() == b"reference-ctree"
    if "--full" in sys.argv:
        for i, name in enumerate(FULL):
            p = record_full(lib, name, seed=5000 + i)
            print("wrote", os.path.relpath(p, ROOT), os.path.getsize(p), "bytes", flush=True)
        return
    only = sys.argv[sys.argv.index("--only") + 1].split(",") if "--only" in sys.argv else None
    for i, (name, cfg) in enumerate(CONFIGS.items()):
        if only is not None and name not in only:
            continue
        p = record(lib, name, cfg, seed=1000 + i)
        print("wrote", os.path.relpath(p, ROOT), os.path.getsize(p), "bytes")
    if only is None:
        kat()
        print("wrote tests/golden/kat_libstdcxx.json")


if __name__ == "__main__":
    main()
