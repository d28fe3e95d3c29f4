"""Headline benchmark: MCTS simulations/s of the MAZero sampled-MCTS hot path on MI355X.

BASELINE.json metric: "MCTS simulations/sec (whole node), SMAC 3m, 256 roots x 50 sims".
One step = one environment step of the self-play loop: the 3 agents of SMAC 3m are searched one
after another (core/selfplay_worker.py:196-211), each search = prepare + 50 simulations over 256
roots, i.e. 38,400 root-simulations per step per GPU.

Per search the device executes exactly what mazero_amd.mcts_sampled runs around the network:
  k_prepare (RNG stream + root expansion)  ->  selection of simulation 0
  49 x k_step<expand+backup, select, gather>  ->  k_step<expand+backup>  ->  k_readback
with the network replaced by synthetic device-resident outputs (softmax(N(0,1))
policy = beta, reward 0.1*N(0,1), value N(0,1), Dirichlet(0.3) root noise, hidden-state pool
[51, 256, 3*128] fp32 that the fused kernel gathers from).  The whole step (3 searches) is
captured once in a HIP graph and replayed.

Multi-GPU (torchrun, one process per GPU): roots are independent (cnode.cpp:633-641), so every
rank searches its own 256 roots (global root offset rank*256, seeds random_seed*2333+global index)
with no collective on the data path -> "scaling": "weak".  The barrier / max-over-ranks timing uses
torch.distributed (RCCL).

Also reported (rank 0, N=1 only):
  roofline      dominant kernel k_step<true,true> (fused simulation step): algorithmic bytes per
                launch (SURVEY §8d formula over the kernel's own counters) / its average duration,
                measured with HIP events on the launch stream around a graph of one search's 49
                back-to-back fused launches; traffic = rocprofv3 FETCH_SIZE+WRITE_SIZE per launch
                from profiles/pmc_latest.json (scripts/pmc_summary.py) for the same workload
  cpu_baseline  the reference C++ ctree (oracle/_ref/libmzref.so, compiled from the reference
                sources) -- or the CPU port when that is absent -- on the same synthetic inputs,
                one host core, timing only the tree calls, over a bounded sample (~10 s)
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
import mazero_amd  # noqa: E402,F401  (HIP runtime settings, before anything initialises HIP)

CONFIGS = {  # name: (agents N, actions A) -- smac_maps.py:17-133, n_actions = 6 + n_enemies
    "3m": (3, 9),
    "2s3z": (5, 11),
    "3s5z_vs_3s6z": (8, 15),
    "27m_vs_30m": (27, 36),
}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--map", default="3m", choices=sorted(CONFIGS))
    ap.add_argument("--roots", type=int, default=256, help="roots per GPU")
    ap.add_argument("--sims", type=int, default=50)
    ap.add_argument("--sampled-times", type=int, default=1, help="K (core/config.py:86 default 1)")
    ap.add_argument("--strong", action="store_true", help="split --roots over the GPUs instead of per GPU")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--seed", type=int, default=0)
    return ap.parse_args(argv)


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    from mazero_amd._lib import load
    from mazero_amd.cytree import Tree_batch
    from mazero_amd.synthetic import DEFAULTS, HIDDEN_PER_AGENT, make_search_inputs

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    lib = load()

    N, A = CONFIGS[args.map]
    S, K = args.sims, args.sampled_times
    B = args.roots // world if args.strong else args.roots
    root_offset = rank * B
    H = N * HIDDEN_PER_AGENT
    d = DEFAULTS
    c2, c1, g = d["pb_c_base"], d["pb_c_init"], d["discount"]

    # ---- synthetic inputs, one set per agent search, resident in HBM ----
    rng = np.random.default_rng(args.seed * 1000 + rank)
    host_inputs = [make_search_inputs(rng, B, A, S) for _ in range(N)]

    def dev_t(a):
        return torch.from_numpy(np.ascontiguousarray(a)).to(dev)

    searches = []
    for inp in host_inputs:
        tb = Tree_batch(B, 1, A, K, S, d["delta_lb"], inp.seed, d["rho"], d["lam"], root_offset=root_offset, lib=lib)
        # one allocation per search for the network outputs ([S, B | B | B*A | B*A]) and one for
        # the selection outputs: every distinct allocation a kernel touches costs a translation miss
        net = dev_t(np.concatenate([inp.reward.reshape(S, -1), inp.value.reshape(S, -1), inp.policy.reshape(S, -1),
                                    inp.beta.reshape(S, -1)], axis=1))
        sel = torch.empty(3, B, dtype=torch.int32, device=dev)
        searches.append(dict(
            tb=tb,
            rr=dev_t(inp.root_reward), rv=dev_t(inp.root_value), rp=dev_t(inp.root_policy),
            rb=dev_t(inp.root_beta), rn=dev_t(inp.root_noise), eps=inp.noise_eps,
            r=net[:, :B], v=net[:, B:2 * B], p=net[:, 2 * B:2 * B + B * A], b=net[:, 2 * B + B * A:],
            pool=torch.randn(S + 1, B, H, device=dev),
            leaf=torch.empty(B, H, device=dev),
            idx=sel[0], idy=sel[1], act=sel[2].view(B, 1),
            values=torch.empty(B, device=dev),
            visits=torch.empty(B, 1, A, dtype=torch.int32, device=dev),
        ))

    fused_events = []

    def one_search(sd, timed_events=None):
        tb = sd["tb"]
        out = (sd["idx"], sd["idy"], sd["act"])
        tb.prepare(sd["rr"], sd["rv"], sd["rp"], sd["rb"], K, sd["eps"], sd["rn"])
        tb.batch_selection_device(c2, c1, g, out=out)
        for s in range(S):
            if s + 1 < S:
                if timed_events is not None:
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    e0.record()
                tb.expansion_backup_selection_device(s + 1, g, K, sd["r"][s], sd["v"][s], sd["p"][s], sd["b"][s],
                                                     c2, c1, out=out, pool=sd["pool"], gather_out=sd["leaf"])
                if timed_events is not None:
                    e1.record()
                    timed_events.append((e0, e1))
            else:
                tb.batch_expansion_and_backup(s + 1, g, K, sd["r"][s], sd["v"][s], sd["p"][s], sd["b"][s])
        # search outputs stay on the device (mcts_sampled.py:176-191)
        lib.mz_get_roots_values(tb._h, C.c_void_p(sd["values"].data_ptr()), 1)
        lib.mz_get_roots_marginal_visit_count(tb._h, C.c_void_p(sd["visits"].data_ptr()), 1)

    def env_step():
        for sd in searches:  # agents searched sequentially (selfplay_worker.py:196-211)
            one_search(sd)

    # warm-up (also builds the pUCT tables, so nothing host->device happens inside the graph)
    stream = torch.cuda.Stream()
    torch.cuda.synchronize()
    with torch.cuda.stream(stream):
        for _ in range(max(1, args.warmup)):
            env_step()
    torch.cuda.synchronize()

    graph = None
    if not args.no_graph:
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=stream):
            env_step()
        torch.cuda.synchronize()
        for _ in range(max(1, args.warmup)):
            graph.replay()
        torch.cuda.synchronize()
    for sd in searches:
        sd["tb"].synchronize()  # surfaces any deferred device-side error before timing
    stats0 = [sd["tb"].stats() for sd in searches]

    # ---- timed region ----
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(stream):
        for _ in range(args.steps):
            if graph is not None:
                graph.replay()
            else:
                env_step()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
        tt = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    for sd in searches:
        sd["tb"].synchronize()
    stats1 = [sd["tb"].stats() for sd in searches]

    sims_per_rank = B * S * N * args.steps
    value = sims_per_rank * world / elapsed
    ms_per_step = elapsed / args.steps * 1e3

    # ---- roofline of the dominant kernel (rank 0) ----
    roofline = None
    if rank == 0:
        st = {k: sum(s1[k] - s0[k] for s0, s1 in zip(stats0, stats1)) for k in stats1[0]}
        launches_fused = N * (S - 1) * args.steps
        # SURVEY.md §8(d) per-simulation algorithmic bytes, over the kernel's own counters
        sel_b = 20 * st["path_edges"] + 20 * st["scored"] + 16 * st["selects"]
        exp_b = st["expands"] * (8 * A + 8 * K + 12) + 40 * st["new_children"]
        bak_b = 48 * st["backup_nodes"]
        gat_b = 2 * H * 4 * launches_fused * B
        # the fused kernel does all of it except the prepare-time expansion and the first selection
        # and the last (non-fused) expansion of each search: attribute proportionally
        frac_fused = (S - 1) / (S + 1)
        bytes_fused = (sel_b + exp_b + bak_b) * frac_fused + gat_b
        bytes_per_launch = bytes_fused / launches_fused
        # Average duration of the fused kernel, measured with HIP events on the launch stream: a
        # graph holding one search's S-1 fused launches (back to back, as in the timed region) is
        # replayed after an eager prepare + first selection; (e1 - e0) / (S - 1) per replay.
        sd0 = searches[0]
        tb0 = sd0["tb"]
        out0 = (sd0["idx"], sd0["idy"], sd0["act"])
        steps_graph = torch.cuda.CUDAGraph()
        with torch.cuda.stream(stream):
            tb0.prepare(sd0["rr"], sd0["rv"], sd0["rp"], sd0["rb"], K, sd0["eps"], sd0["rn"])
            tb0.batch_selection_device(c2, c1, g, out=out0)
        torch.cuda.synchronize()
        with torch.cuda.graph(steps_graph, stream=stream):
            for s in range(S - 1):
                tb0.expansion_backup_selection_device(s + 1, g, K, sd0["r"][s], sd0["v"][s], sd0["p"][s], sd0["b"][s],
                                                      c2, c1, out=out0, pool=sd0["pool"], gather_out=sd0["leaf"])
        durs = []
        with torch.cuda.stream(stream):
            for rep in range(6):
                tb0.prepare(sd0["rr"], sd0["rv"], sd0["rp"], sd0["rb"], K, sd0["eps"], sd0["rn"])
                tb0.batch_selection_device(c2, c1, g, out=out0)
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record()
                steps_graph.replay()
                e1.record()
                e1.synchronize()
                if rep > 0:
                    durs.append(e0.elapsed_time(e1) * 1e-3 / (S - 1))
        torch.cuda.synchronize()
        tb0.synchronize()
        avg = float(np.median(durs))
        achieved = bytes_per_launch / avg / 1e9
        roofline = dict(
            kernel="k_step<true,true> (fused expand+backup+select+gather)",
            bound="hbm",
            achieved=round(achieved, 3),
            peak=8000.0,
            unit="GB/s",
            frac=round(achieved / 8000.0, 6),
            traffic=pmc_traffic(args),
            bytes_per_launch=round(bytes_per_launch, 1),
            avg_launch_us=round(avg * 1e6, 3),
            mean_path_len=round(st["path_edges"] / max(1, st["selects"]), 3),
        )
        if os.environ.get("MZ_STAMPS") == "1" and st.get("stamped", 0) > 0:
            # diagnostic build: average shader cycles per fused launch and tree, per phase
            roofline["phase_cycles"] = {k[4:]: round(st[k] / st["stamped"], 1) for k in st if k.startswith("cyc_")}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(host_inputs, B, A, K, S, N, args.cpu_seconds)

    if rank == 0:
        line = {
            "metric": "MCTS simulations/sec (whole node), SMAC 3m, 256 roots×50 sims, 1/2/4/8 GPUs"
            if args.map == "3m" else f"MCTS simulations/sec (whole node), SMAC {args.map}",
            "value": round(value, 1),
            "unit": "simulations/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "strong" if args.strong else "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (device-resident network outputs + hidden-state pool, SURVEY §8d)",
            "config": {
                "workload": f"SMAC {args.map} self-play search: {N} sequential agent searches x {B} roots/GPU x {S} sims",
                "map": args.map,
                "agents": N,
                "actions": A,
                "roots_per_gpu": B,
                "roots_total": B * world,
                "sims": S,
                "sampled_times": K,
                "hidden": H,
                "graph": graph is not None,
                "parallelism": f"roots sharded over {world} GPU(s), no collective on the data path",
            },
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def workload_key(args):
    return f"{args.map}:B{args.roots}:S{args.sims}:K{args.sampled_times}"


def pmc_traffic(args):
    """HBM bytes per launch of the fused kernel from the committed rocprofv3 PMC summary of the same
    workload (profiles/pmc_latest.json, written by scripts/pmc_summary.py from separate
    FETCH_SIZE and WRITE_SIZE passes), or None when there is none for this configuration."""
    path = os.path.join(ROOT, "profiles", "pmc_latest.json")
    try:
        with open(path) as f:
            pm = json.load(f)
    except (OSError, ValueError):
        return None
    key = workload_key(args)
    ent = pm.get("workloads", {}).get(key)
    if not ent:
        return None
    return ent.get("fused_bytes_per_launch")


def cpu_baseline(host_inputs, B, A, K, S, N, budget_s):
    """The reference CPU ctree (or the CPU port), one host core, tree calls only, same inputs;
    plus the same on up to 16 host cores at once ("multi_core", informational)."""
    from mazero_amd import _capi
    from mazero_amd.cytree import Tree_batch
    from mazero_amd.synthetic import DEFAULTS

    ref = os.path.join(ROOT, "oracle", "_ref", "libmzref.so")
    port = os.path.join(ROOT, "oracle", "_build", "libmzport.so")
    if os.path.exists(ref):
        path, kind = ref, "reference"
    elif os.path.exists(port):
        path, kind = port, "port"
    else:
        return None
    lib = _capi.bind(C.CDLL(path))
    d = DEFAULTS
    c2, c1, g = d["pb_c_base"], d["pb_c_init"], d["discount"]
    sims = 0
    tree_time = 0.0
    steps = 0
    while tree_time < budget_s:
        for inp in host_inputs:  # one env step = N sequential searches
            tb = Tree_batch(B, 1, A, K, S, d["delta_lb"], inp.seed, d["rho"], d["lam"], lib=lib)
            t0 = time.perf_counter()
            tb.prepare(inp.root_reward, inp.root_value, inp.root_policy, inp.root_beta, K, inp.noise_eps,
                       inp.root_noise)
            for s in range(S):
                tb.batch_selection(c2, c1, g)
                tb.batch_expansion_and_backup(s + 1, g, K, inp.reward[s], inp.value[s], inp.policy[s], inp.beta[s])
            tb.get_roots_values()
            tb.get_roots_marginal_visit_count()
            tree_time += time.perf_counter() - t0
            sims += B * S
        steps += 1
    # (ii) SURVEY §8(d): the same searches on several host cores at once -- independent tree
    # batches, one per thread (the reference ctree releases the GIL inside its ctypes calls), as
    # many threads as this process's CPU share allows, at most 16 (the GPU box's share per GPU)
    def worker(budget, out, k):
        n_sims, t_run, t0w = 0, 0.0, time.perf_counter()
        while time.perf_counter() - t0w < budget:
            for inp in host_inputs:
                tb = Tree_batch(B, 1, A, K, S, d["delta_lb"], inp.seed, d["rho"], d["lam"], lib=lib)
                ts = time.perf_counter()
                tb.prepare(inp.root_reward, inp.root_value, inp.root_policy, inp.root_beta, K, inp.noise_eps,
                           inp.root_noise)
                for s in range(S):
                    tb.batch_selection(c2, c1, g)
                    tb.batch_expansion_and_backup(s + 1, g, K, inp.reward[s], inp.value[s], inp.policy[s],
                                                  inp.beta[s])
                tb.get_roots_values()
                tb.get_roots_marginal_visit_count()
                t_run += time.perf_counter() - ts
                n_sims += B * S
        out[k] = (n_sims, t_run)

    import threading
    try:
        share = len(os.sched_getaffinity(0))
    except AttributeError:
        share = os.cpu_count() or 1
    n_thr = max(1, min(16, share))
    res = [None] * n_thr
    t0 = time.perf_counter()
    thr = [threading.Thread(target=worker, args=(budget_s / 2, res, k)) for k in range(n_thr)]
    for x in thr:
        x.start()
    for x in thr:
        x.join()
    wall = time.perf_counter() - t0
    multi = {"value": round(sum(r[0] for r in res) / wall, 1), "threads": n_thr,
             "sample": f"{sum(r[0] for r in res)} sims in {wall:.1f} s wall, one independent tree batch per thread"}
    cpu_model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu_model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {
        "value": round(sims / tree_time, 1),
        "unit": "simulations/s",
        "cores": 1,
        "kind": kind,
        "sample": f"{steps} env steps x {N} searches x {B} roots x {S} sims (K={K}) = {sims} sims, "
                  f"{tree_time:.1f} s of tree calls on 1 core of '{cpu_model}' (nproc {os.cpu_count()})",
        "multi_core": multi,
    }


if __name__ == "__main__":
    main()
