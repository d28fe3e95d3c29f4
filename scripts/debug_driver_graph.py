"""Diagnostic (not product): tests/test_driver.py::test_graph_replay_after_eager_launches with
per-agent reporting.  Graph searches (capture + replays), optional eager searches, then one
self-play step whose graph replays are compared with eager searches of the same inputs.

    python scripts/debug_driver_graph.py [n_graph_steps] [n_eager_steps] [final_steps]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import mazero_amd  # noqa: E402,F401
import torch  # noqa: E402

from mazero_amd.mcts_sampled import SampledMCTS  # noqa: E402
from mazero_amd.nets import SearchConfig, make_net, make_root_batch  # noqa: E402


FIELDS = ("kind", "bad", "eb|sel<<1", "t", "tot", "cur", "D", "herr", "tot_l2", "cur_l2", "D_l2", "P", "PS", "BA",
          "pk", "K", "hsx", "disc", "pe", "ne", "prm_P", "prm_PS", "prm_B", "prm_K", "ka_lo", "ka_hi", "kmem_base_lo",
          "kmem_base_hi", "base_lo", "base_hi", "err", "reward_lo")


def dump_records():
    """MZ_ARGCHECK builds: the device-side records of inconsistent launches (kind 1: on entry,
    kind 2/3: wave 0/1 set an error) and the kErrPath site bits."""
    import ctypes as C
    from mazero_amd._lib import load
    lib = load()
    try:
        fn = lib.mz_debug_dump
    except AttributeError:
        return
    buf = (C.c_uint * (2 + 64 * 32))()
    fn(buf, len(buf))
    n, sites = buf[0], buf[1]
    print(f"argcheck: {n} records, kErrPath sites {sites:#x}", flush=True)
    from mazero_amd import mcts_sampled
    peek = getattr(lib, "mz_debug_peek", None)
    if peek is not None:
        for tb in list(mcts_sampled._TREES.values()):
            words = (C.c_uint * 2048)()
            lay = (C.c_ulonglong * 8)()
            peek(tb._h, words, 2048, lay)
            print("arena base %#x err %#x seed %#x lp %#x T %#x hdr %#x stats %#x" % tuple(lay[:7]), flush=True)
            nz = [(i, words[i]) for i in range(2048) if words[i]]
            print(f"  nonzero words from err on ({len(nz)}): " +
                  " ".join(f"+{4 * i}:{v:#x}" for i, v in nz[:96]), flush=True)
    for r in range(min(n, 64)):
        w = buf[2 + 32 * r: 2 + 32 * (r + 1)]
        print("  " + " ".join(f"{k}={v:#x}" if k.endswith(("lo", "hi", "BA", "pk")) else f"{k}={v}"
                              for k, v in zip(FIELDS, w)), flush=True)


def main():
    n_graph = int(sys.argv[1]) if len(sys.argv) > 1 else 7
    n_eager = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    n_final = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    print("env:", {k: v for k, v in os.environ.items() if k.startswith(("DEBUG_CLR", "MZ_"))}, flush=True)
    N, A, B, S = 3, 9, 256, 50
    dev = torch.device("cuda", 0)
    cfg = SearchConfig(action_space_size=A, num_simulations=S, sampled_action_times=1)
    net = make_net(N, A, seed=0, device=dev)
    roots = [make_root_batch(net, B, 64, seed=10 + i, device=dev, legal_zero_frac=0.2) for i in range(3)]
    for n_steps, use_graph in ((n_graph, True), (n_eager, False)):
        m = SampledMCTS(cfg, np.random.RandomState(0), use_graph=use_graph)
        for i in range(n_steps):
            out, legal = roots[i % 3]
            acts = np.zeros((B, N), np.int32)
            for agent in range(N):
                try:
                    r = m.batch_search(net, out, agent, acts[:, :agent].copy() if agent else None, N, legal,
                                       device=dev, add_noise=True)
                except RuntimeError as e:
                    print(f"phase graph={use_graph} step {i} agent {agent}: {e}", flush=True)
                    dump_records()
                    return 3
                acts[:, agent] = [int(a[np.argmax(v), 0]) for a, v in zip(r.sampled_actions, r.sampled_visit_count)]
    bad = 0
    if os.environ.get("DBG_TEST_FINAL") == "1":  # the regression test's own final step
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        from consume import eps_greedy_given, select_action
        ur = np.random.default_rng(1)
        u_eps, u_cat = ur.random((N, B)).astype(np.float32), ur.random((N, B))
        rs_d = np.random.default_rng(3)
        drv = SampledMCTS(cfg, rs_d)
        out, legal = roots[0]
        acts = np.full((B, N), -1, np.int32)
        for agent in range(N):
            fac = acts[:, :agent].copy() if agent else None
            try:
                got = drv.batch_search(net, out, agent, fac, N, legal, device=dev, add_noise=True)
                print(f"test-final agent {agent}: ok", flush=True)
            except RuntimeError as e:
                print(f"test-final agent {agent}: ERR {e}; factor range "
                      f"{None if fac is None else (int(fac.min()), int(fac.max()))}", flush=True)
                dump_records()
                return 1
            for i in range(B):
                pos, _ = select_action(got.sampled_visit_count[i], 1.0, False, rs_d)
                acts[i, agent] = eps_greedy_given(got.sampled_actions[i][pos, 0], legal[i, agent], 0.1,
                                                  u_eps[agent, i], u_cat[agent, i])
        return 0
    for f in range(n_final):
        out, legal = roots[f % 3]
        acts = np.zeros((B, N), np.int32)
        for agent in range(N):
            fac = acts[:, :agent].copy() if agent else None
            res = {}
            for use_graph in (True, False):
                m = SampledMCTS(cfg, np.random.RandomState(100 + f), use_graph=use_graph)
                try:
                    r = m.batch_search(net, out, agent, fac, N, legal, device=dev, add_noise=True)
                    res[use_graph] = (r.value.copy(), [v.copy() for v in r.sampled_visit_count])
                except RuntimeError as e:
                    res[use_graph] = str(e)
            g, e = res[True], res[False]
            if isinstance(g, str) or isinstance(e, str):
                print(f"final {f} agent {agent}: graph={'ERR ' + g if isinstance(g, str) else 'ok'} "
                      f"eager={'ERR ' + e if isinstance(e, str) else 'ok'}", flush=True)
                bad += 1
                continue
            same = np.array_equal(g[0].view(np.uint32), e[0].view(np.uint32)) and all(
                np.array_equal(a, b) for a, b in zip(g[1], e[1]))
            print(f"final {f} agent {agent}: graph vs eager {'same' if same else 'DIFFER'}", flush=True)
            bad += 0 if same else 1
    dump_records()
    print(f"done: {bad} bad", flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
