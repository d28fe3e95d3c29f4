"""Headline benchmark: MCTS simulations/s of the MAZero sampled-MCTS hot path on MI355X.

BASELINE.json metric: "MCTS simulations/sec (whole node), SMAC 3m, 256 roots x 50 sims".
One step = one environment step of the self-play loop: the 3 agents of SMAC 3m are searched one
after another (core/selfplay_worker.py:196-211), each search = prepare + 50 simulations over 256
roots, i.e. 38,400 root-simulations per step per GPU.

Per search the device executes exactly what mazero_amd.mcts_sampled runs around the network:
  k_prepare (RNG stream + root expansion + the selection of simulation 0)
  49 x fused <expand+backup, select, gather>  ->  1 x <expand+backup>  ->  one k_readback
where the fused kernel is k_chain3 (K = 1, pools <= 256 nodes), k_chain (K = 1, larger pools), k_tree
(2 <= K <= 64, pools <= 1024 nodes) or k_step
(as the library reports it, mz_fused_kernel)
with the network replaced by synthetic device-resident outputs (softmax(N(0,1))
policy = beta, reward 0.1*N(0,1), value N(0,1), Dirichlet(0.3) root noise, hidden-state pool
[51, 256, 3*128] fp32 that the fused kernel gathers from).  The whole step (3 searches) is
captured once in a HIP graph and replayed.

Multi-GPU: one process per GPU.  Under torchrun (WORLD_SIZE set) every process is one rank;
`python bench.py --gpus N` without torchrun starts the N ranks itself (torch.distributed.run, before
anything touches the GPU) and n_gpus is the job's world size.  Roots are independent
(cnode.cpp:633-641), so ranks share no data-path collective:
  weak   (headline, "scaling": "weak")  every rank searches its own --roots (256) roots: the node's
         self-play, one shard of environments per GPU as the reference runs one data worker per
         GPU, each with its own 256-root searches; value = all ranks' simulations / the slowest
         rank's time (the "whole node" of the metric);
  strong (N > 1, reported beside it as "strong_scaling")  the --roots roots of ONE batch split over
         the ranks: rank r searches rows [lo, hi) of the global batch (global root offset lo, tree
         seeds random_seed*2333 + global index).  Bounded near 1.1x at 8 GPUs by the chain of
         147 dependent launches per env step (profiles/round6/strong_proxy.json).
`--strong` swaps the two.  The barrier / max-over-ranks clock uses torch.distributed (RCCL).

Also reported (rank 0, N=1 only):
  roofline      dominant kernel = the fused simulation step (49 of 52 launches): algorithmic bytes per
                launch (SURVEY §8d formula over the kernel's own counters) / its average duration,
                measured with HIP events on the launch stream around a graph of one search's 49
                back-to-back fused launches; traffic = rocprofv3 FETCH_SIZE+WRITE_SIZE per launch
                from profiles/pmc_latest.json (scripts/pmc_summary.py) for the same workload,
                2 x FETCH_SIZE + WRITE_SIZE (the guide's gfx950 correction; raw beside it)
  cpu_baseline  the reference C++ ctree (oracle/_ref/libmzref.so, compiled from the reference
                sources) -- or the CPU port when that is absent -- on the same synthetic inputs,
                one host core, timing only the tree calls, over a bounded sample (~10 s); plus
                "multi_core": one process per host core (up to --cpu-procs), roots sharded
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
    "matrix": (2, 3),  # BASELINE config #1: config/matrix 2-agent matrix game (matgame.py:16,27-60)
    "3m": (3, 9),
    "2s3z": (5, 11),
    "3s5z_vs_3s6z": (8, 15),
    "27m_vs_30m": (27, 36),
}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one process per GPU); without torchrun's WORLD_SIZE, N > 1 spawns them")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--map", default="3m", choices=sorted(CONFIGS))
    ap.add_argument("--roots", type=int, default=256, help="roots per GPU (weak scaling) / in total (strong)")
    ap.add_argument("--sims", type=int, default=50)
    ap.add_argument("--sampled-times", type=int, default=1, help="K (core/config.py:86 default 1)")
    ap.add_argument("--strong", action="store_true",
                    help="N > 1: headline value from the strong-scaling leg (--roots roots split over the GPUs) "
                         "instead of the weak one (--roots roots on every GPU)")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-procs", type=int, default=16,
                    help="processes of the multi-core CPU baseline (at most this process's CPU share)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--dropin", action="store_true",
                    help="time the tree-level drop-in instead: the reference driver's host loop "
                         "(mcts_sampled.py:114-172, numpy in and out of every Tree_batch call) on mazero_amd.cytree")
    ap.add_argument("--broadcast-every", type=int, default=0, metavar="N",
                    help="BASELINE config #5's weight broadcast: every N env steps inside the timed loop, rank 0 "
                         "publishes a new checkpoint and every rank runs WeightBroadcaster.sync() of the "
                         "--broadcast-map network's flat weights (selfplay_worker.py:371-375); 0 = off")
    ap.add_argument("--broadcast-map", default="27m_vs_30m", choices=sorted(CONFIGS),
                    help="the map whose network's weights the broadcast carries (config #5: 27m_vs_30m)")
    ap.add_argument("--backend", default="hip", choices=("hip", "port"),
                    help="'port': every rank searches on the host with the CPU port over gloo -- a CPU "
                         "test of the launcher / sharding / clock plumbing only, never a measurement")
    return ap.parse_args(argv)


def launch(args) -> int:
    """`--gpus N` without torchrun: start N ranks under torch.distributed.run (one process per GPU)
    and return its exit status.  Nothing here touches the GPU, so the ranks start clean."""
    import socket
    import subprocess

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *sys.argv[1:]]
    return subprocess.call(cmd, env=dict(os.environ))


class HipLeg:
    """One rank's searches on its GPU: N sequential agent searches over B roots (global root
    offset `root_offset`), inputs and network outputs resident in HBM, the whole env step captured
    in one HIP graph."""

    def __init__(self, args, host_inputs, root_offset, lib, dev, stream):
        import torch

        from mazero_amd.cytree import Tree_batch
        from mazero_amd.synthetic import DEFAULTS, HIDDEN_PER_AGENT

        B = host_inputs[0].B
        self.args, self.B, self.lib, self.stream = args, B, lib, stream
        # the last expansion and the readback in one launch (an older experiment build may lack it)
        self.fused_rb = hasattr(lib, "mz_expand_backup_readback")
        N, A = CONFIGS[args.map]
        S, K = args.sims, args.sampled_times
        self.N, self.A, self.S, self.K, self.H = N, A, S, K, N * HIDDEN_PER_AGENT
        d = DEFAULTS
        self.c2, self.c1, self.g = d["pb_c_base"], d["pb_c_init"], d["discount"]
        # synthetic inputs, one set per agent search, for this rank's global root range
        self.host_inputs = host_inputs

        def dev_t(a):
            return torch.from_numpy(np.ascontiguousarray(a)).to(dev)

        self.searches = []
        for inp in self.host_inputs:
            tb = Tree_batch(B, 1, A, K, S, d["delta_lb"], inp.seed, d["rho"], d["lam"], root_offset=root_offset,
                            lib=lib)
            # one allocation per search for the network outputs ([S, B | B | B*A | B*A]) and one for
            # the selection outputs: every distinct allocation a kernel touches costs a translation miss
            net = dev_t(np.concatenate([inp.reward.reshape(S, -1), inp.value.reshape(S, -1),
                                        inp.policy.reshape(S, -1), inp.beta.reshape(S, -1)], axis=1))
            sel = torch.empty(3, B, dtype=torch.int32, device=dev)
            self.searches.append(dict(
                tb=tb,
                rr=dev_t(inp.root_reward), rv=dev_t(inp.root_value), rp=dev_t(inp.root_policy),
                rb=dev_t(inp.root_beta), rn=dev_t(inp.root_noise), eps=inp.noise_eps,
                r=net[:, :B], v=net[:, B:2 * B], p=net[:, 2 * B:2 * B + B * A], b=net[:, 2 * B + B * A:],
                pool=torch.randn(S + 1, B, self.H, device=dev),
                leaf=torch.empty(B, self.H, device=dev),
                idx=sel[0], idy=sel[1], act=sel[2].view(B, 1),
                values=torch.empty(B, device=dev),
                visits=torch.empty(B, 1, A, dtype=torch.int32, device=dev),
            ))
        self.graph = None

    def one_search(self, sd):
        S, K, c2, c1, g = self.S, self.K, self.c2, self.c1, self.g
        tb = sd["tb"]
        out = (sd["idx"], sd["idy"], sd["act"])
        tb.prepare_selection_device(sd["rr"], sd["rv"], sd["rp"], sd["rb"], K, sd["eps"], sd["rn"], c2, c1, g, out=out)
        for s in range(S):
            if s + 1 < S:
                tb.expansion_backup_selection_device(s + 1, g, K, sd["r"][s], sd["v"][s], sd["p"][s], sd["b"][s],
                                                     c2, c1, out=out, pool=sd["pool"], gather_out=sd["leaf"])
            elif self.fused_rb:
                # the last expansion writes the search outputs too (mz_expand_backup_readback): they stay on
                # the device (mcts_sampled.py:176-191)
                tb.expansion_backup_readback_device(s + 1, g, K, sd["r"][s], sd["v"][s], sd["p"][s], sd["b"][s],
                                                    readback_discount=g,
                                                    out=dict(values=sd["values"], marginal_visit_count=sd["visits"]))
            else:
                tb.batch_expansion_and_backup(s + 1, g, K, sd["r"][s], sd["v"][s], sd["p"][s], sd["b"][s])
        if not self.fused_rb:  # search outputs stay on the device (mcts_sampled.py:176-191): one readback launch
            tb.get_roots_device(g, values=sd["values"], marginal_visit_count=sd["visits"])

    def env_step(self):
        for sd in self.searches:  # agents searched sequentially (selfplay_worker.py:196-211)
            self.one_search(sd)

    def prepare(self):
        """Warm-up (also builds the pUCT tables, so nothing host->device happens inside the graph),
        then the graph of one env step."""
        import torch

        torch.cuda.synchronize()
        with torch.cuda.stream(self.stream):
            for _ in range(max(1, self.args.warmup)):
                self.env_step()
        torch.cuda.synchronize()
        if not self.args.no_graph:
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph, stream=self.stream):
                self.env_step()
            torch.cuda.synchronize()
            for _ in range(max(1, self.args.warmup)):
                self.graph.replay()
            torch.cuda.synchronize()
        self.check()

    def check(self):
        for sd in self.searches:
            sd["tb"].synchronize()  # surfaces any deferred device-side error

    def stats(self):
        return [sd["tb"].stats() for sd in self.searches]

    def run(self, steps, before_step=None):
        import torch

        with torch.cuda.stream(self.stream):
            for i in range(steps):
                if before_step is not None:
                    before_step(i)
                if self.graph is not None:
                    self.graph.replay()
                else:
                    self.env_step()

    def roofline(self, stats0, stats1, steps):
        """Algorithmic bytes per launch of the fused kernel over its measured average duration."""
        import torch

        N, A, K, S, B, H = self.N, self.A, self.K, self.S, self.B, self.H
        c2, c1, g = self.c2, self.c1, self.g
        st = {k: sum(s1[k] - s0[k] for s0, s1 in zip(stats0, stats1)) for k in stats1[0]}
        launches_fused = N * (S - 1) * steps
        # SURVEY.md §8(d) per-simulation algorithmic bytes, over the kernel's own counters
        sel_b = 20 * st["path_edges"] + 20 * st["scored"] + 16 * st["selects"]
        exp_b = st["expands"] * (8 * A + 8 * K + 12) + 40 * st["new_children"]
        bak_b = 48 * st["backup_nodes"]
        gat_b = 2 * H * 4 * launches_fused * B
        # the fused kernel does all of it except the prepare-time expansion and the first selection
        # and the last (non-fused) expansion of each search: attribute proportionally
        frac_fused = (S - 1) / (S + 1)
        bytes_per_launch = ((sel_b + exp_b + bak_b) * frac_fused + gat_b) / launches_fused
        # Average duration of the fused kernel, measured with HIP events on the launch stream: a
        # graph holding one search's S-1 fused launches (back to back, as in the timed region) is
        # replayed after an eager prepare + first selection; (e1 - e0) / (S - 1) per replay.
        sd0 = self.searches[0]
        tb0 = sd0["tb"]
        out0 = (sd0["idx"], sd0["idy"], sd0["act"])
        steps_graph = torch.cuda.CUDAGraph()
        with torch.cuda.stream(self.stream):
            tb0.prepare(sd0["rr"], sd0["rv"], sd0["rp"], sd0["rb"], K, sd0["eps"], sd0["rn"])
            tb0.batch_selection_device(c2, c1, g, out=out0)
        torch.cuda.synchronize()
        with torch.cuda.graph(steps_graph, stream=self.stream):
            for s in range(S - 1):
                tb0.expansion_backup_selection_device(s + 1, g, K, sd0["r"][s], sd0["v"][s], sd0["p"][s], sd0["b"][s],
                                                      c2, c1, out=out0, pool=sd0["pool"], gather_out=sd0["leaf"])
        durs = []
        spans = getattr(self.lib, "mz_debug_spans", None)  # diagnostic builds (MZ_SPANS / MZ_STAMPS) only
        if spans is not None:
            spans.argtypes, spans.restype = [C.c_void_p, C.c_int, C.c_int, C.c_int], C.c_int
        with torch.cuda.stream(self.stream):
            for rep in range(6):
                tb0.prepare(sd0["rr"], sd0["rv"], sd0["rp"], sd0["rb"], K, sd0["eps"], sd0["rn"])
                tb0.batch_selection_device(c2, c1, g, out=out0)
                if spans is not None and rep == 5:
                    torch.cuda.synchronize()
                    spans(None, 0, 0, 1)
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
        span = launch_spans(spans, S, self.B) if spans is not None else None
        achieved = bytes_per_launch / avg / 1e9
        pmc = pmc_traffic(self.args)
        r = dict(
            kernel=fused_kernel_name(tb0),
            bound="hbm",
            achieved=round(achieved, 3),
            peak=8000.0,
            unit="GB/s",
            frac=round(achieved / 8000.0, 6),
            traffic=None if pmc is None else pmc.get("fused_bytes_per_launch_corrected"),
            traffic_raw=None if pmc is None else pmc.get("fused_bytes_per_launch"),
            traffic_note="rocprofv3 PMC, bytes per fused launch: 2 x FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md "
                         "§HBM gfx950 correction); traffic_raw = FETCH_SIZE + WRITE_SIZE",
            bytes_per_launch=round(bytes_per_launch, 1),
            avg_launch_us=round(avg * 1e6, 3),
            mean_path_len=round(st["path_edges"] / max(1, st["selects"]), 3),
        )
        if "mm_moved" in st and K > 1:
            # back-propagations after which the min/max normaliser moved (every internal node's
            # select_child outcome can change then), per tree and per launch: a launch's duration is
            # its slowest tree's, so the launch with no moved tree is what an incremental rescore needs
            backups = max(1, st["expands"] - N * steps * B)  # (minus the prepares' root expansions)
            p_move = st["mm_moved"] / backups
            r["normaliser_moved_per_backup"] = round(p_move, 4)
            r["launches_without_a_moved_tree"] = float(f"{(1.0 - p_move) ** B:.3e}")
        if span is not None:
            r["launch_span"] = span
        if os.environ.get("MZ_STAMPS") == "1" and st.get("stamped", 0) > 0:
            # diagnostic build: average shader cycles per fused launch and tree, per phase
            r["phase_cycles"] = {k[4:]: round(st[k] / st["stamped"], 1) for k in st if k.startswith("cyc_")}
        return r


def launch_spans(spans, S, B):
    """Diagnostic builds (MZ_SPANS / MZ_STAMPS): the last replay's fused launches (slots hsx = 1 ..
    S-1) on the chip-wide 100 MHz clock -- body = a launch's earliest wave start to its latest wave
    end (every wave role that records one), gap = one launch's latest wave end to the next launch's
    earliest wave start (mz_debug_spans); body + gap = the back-to-back period the HIP events
    measure.  wave_us: each role's mean end after its workgroup's start."""
    slots, trees = min(S, 256), min(B, 1024)
    buf = (C.c_ulonglong * (4 * slots * trees))()
    spans(C.cast(buf, C.c_void_p), slots, trees, 0)
    raw = np.array(buf[:], dtype=np.uint64).reshape(slots, trees, 4)[1:slots]
    info = np.where(raw >= np.uint64(1 << 63), raw & np.uint64((1 << 63) - 1), np.uint64(0))  # k_tree: tree shapes
    t = np.where(raw >= np.uint64(1 << 63), 0, raw).astype(np.float64) * 10.0  # ns
    start = t[:, :, 0]
    ends = np.where(t[:, :, 1:] > 0, t[:, :, 1:], np.nan)
    t0, t1 = start.min(axis=1), np.nanmax(ends, axis=(1, 2))
    body = t1 - t0
    gap = t0[1:] - t1[:-1]
    wave = {f"w{k}": round(float(np.nanmean(ends[:, :, k] - start)) / 1e3, 3)
            for k in range(3) if np.isfinite(ends[:, :, k]).any()}
    # one workgroup's own span (its start to its last recorded wave end): the mean tree against the
    # slowest tree of each launch (the launch ends with its slowest workgroup) and the start spread
    own = np.nanmax(ends, axis=2) - start
    shape = {}
    if info[:, :, 2].any():  # k_tree: the trees' own spans by back-propagation depth D, the slowest tree's D
        D = (info[:, :, 2] & np.uint64(0xffff)).astype(np.int64)
        slow = np.nanargmax(own, axis=1)
        shape = dict(own_us_by_D={int(k): [round(float(np.nanmean(own[D == k])) / 1e3, 3), int((D == k).sum())]
                                  for k in np.unique(D)},
                     slowest_tree_D=np.bincount(D[np.arange(len(slow)), slow]).tolist(),
                     ntot_max=int(((info[:, :, 2] >> np.uint64(16)) & np.uint64(0xffff)).max()))
        # the trees after whose back-propagation the min/max normaliser moved (bit 48): every score
        # of such a tree changes, so an incremental rescore (only the path's parents) helps only the
        # others.  A launch ends with its slowest tree: the slowest moved tree per launch bounds what
        # skipping the rescore in every other tree could give
        mv = ((info[:, :, 2] >> np.uint64(48)) & np.uint64(1)).astype(bool)
        if mv.any():
            own_mv = np.where(mv, own, np.nan)
            own_st = np.where(mv, np.nan, own)
            shape["normaliser_moved"] = dict(
                trees_per_launch=round(float(mv.sum(axis=1).mean()), 1),
                slowest_tree_us=round(float(np.nanmean(np.nanmax(own, axis=1))) / 1e3, 3),
                slowest_moved_tree_us=round(float(np.nanmean(np.nanmax(own_mv, axis=1))) / 1e3, 3),
                slowest_unmoved_tree_us=round(float(np.nanmean(np.nanmax(own_st, axis=1))) / 1e3, 3),
                launches_whose_slowest_tree_moved=round(float(mv[np.arange(len(own)), np.nanargmax(own, axis=1)].mean()), 3))
        ph = info[:, :, 3]
        if ph.any():  # wave 0's phase ends by D: barrier (1) left, barrier (2) left, chase done, end (us)
            marks = [((ph >> np.uint64(16 * k)) & np.uint64(0xffff)).astype(np.float64) * 0.01 for k in range(3)]
            shape["w0_phases_us_by_D"] = {int(k): [round(float(m[D == k].mean()), 3) for m in marks] +
                                          [round(float(np.nanmean(own[D == k])) / 1e3, 3)] for k in np.unique(D)}
    return dict(**shape,clock="s_memrealtime (100 MHz)", launches=int(len(body)),
                tree_us_mean=round(float(np.nanmean(own)) / 1e3, 3),
                tree_us_slowest=round(float(np.nanmean(np.nanmax(own, axis=1))) / 1e3, 3),
                start_spread_us=round(float(np.mean(start.max(axis=1) - t0)) / 1e3, 3),
                body_us_mean=round(float(body.mean()) / 1e3, 3), body_us_median=round(float(np.median(body)) / 1e3, 3),
                gap_us_mean=round(float(gap.mean()) / 1e3, 3), gap_us_median=round(float(np.median(gap)) / 1e3, 3),
                period_us=round(float(t1[-1] - t0[0]) / 1e3 / len(body), 3), wave_us=wave)


def fused_kernel_name(tb) -> str:
    """The per-simulation fused kernel the library launches for this handle, as the library itself
    reports it (mz_fused_kernel: chosen at mz_create from the geometry and MZ_CHAIN_V2 /
    MZ_NO_CHAIN / MZ_NO_TREE)."""
    if not hasattr(tb._lib, "mz_fused_kernel"):  # (an older experiment build, MZ_LIB_OVERRIDE)
        return "unknown (library without mz_fused_kernel)"
    k = tb.fused_kernel()
    what = {"k_chain3": "K = 1 chains, three waves", "k_chain": "K = 1 chains, two waves",
            "k_tree": "eight waves", "k_step": "general kernel",
            "k_hbm": "HBM-resident general kernel, eight waves"}[k.split("<")[0]]
    return f"{k} ({what}: fused expand+backup+select+gather)"


class DropinLeg:
    """--dropin: what the INTEGRATION.md import swap gives a user of the reference driver -- its
    per-simulation Tree_batch calls unchanged (mcts_sampled.py:114-172: batch_selection, then
    batch_expansion_and_backup with numpy arrays), one env step = N sequential searches with
    prepare and the two root readbacks the CPU baseline times too, on the MI355X library through
    the host-memory path (every call copies its inputs in and its outputs out).  A measurement of
    the boundary, not of the kernels."""

    def __init__(self, args, host_inputs, root_offset, lib):
        from mazero_amd.synthetic import DEFAULTS

        self.args, self.B, self.root_offset, self.lib = args, host_inputs[0].B, root_offset, lib
        N, A = CONFIGS[args.map]
        self.N, self.A, self.S, self.K = N, A, args.sims, args.sampled_times
        self.d = DEFAULTS
        self.host_inputs = host_inputs
        self.graph = None

    def env_step(self):
        from mazero_amd.cytree import Tree_batch

        d, S, K = self.d, self.S, self.K
        c2, c1, g = d["pb_c_base"], d["pb_c_init"], d["discount"]
        for inp in self.host_inputs:
            tb = Tree_batch(self.B, 1, self.A, K, S, d["delta_lb"], inp.seed, d["rho"], d["lam"],
                            root_offset=self.root_offset, lib=self.lib)
            tb.prepare(inp.root_reward, inp.root_value, inp.root_policy, inp.root_beta, K, inp.noise_eps,
                       inp.root_noise)
            for s in range(S):
                tb.batch_selection(c2, c1, g)
                tb.batch_expansion_and_backup(s + 1, g, K, inp.reward[s], inp.value[s], inp.policy[s], inp.beta[s])
            tb.get_roots_values()
            tb.get_roots_marginal_visit_count()

    def prepare(self):
        for _ in range(max(1, self.args.warmup)):
            self.env_step()

    def check(self):
        pass

    def run(self, steps, before_step=None):
        for i in range(steps):
            if before_step is not None:
                before_step(i)
            self.env_step()


class PortLeg:
    """--backend port (CPU test of the multi-rank plumbing only): the same searches of this rank's
    roots on the host with the CPU port library."""

    def __init__(self, args, host_inputs, root_offset):
        from mazero_amd import _capi
        from mazero_amd.synthetic import DEFAULTS

        path = os.path.join(ROOT, "oracle", "_build", "libmzport.so")
        self.lib = _capi.bind(C.CDLL(path))
        self.args, self.B, self.root_offset = args, host_inputs[0].B, root_offset
        N, A = CONFIGS[args.map]
        self.N, self.A, self.S, self.K = N, A, args.sims, args.sampled_times
        self.d = DEFAULTS
        self.host_inputs = host_inputs
        self.graph = None
        self.values = None

    def env_step(self):
        from mazero_amd.cytree import Tree_batch
        from mazero_amd.synthetic import run_search

        d, out = self.d, []
        for inp in self.host_inputs:
            tb = Tree_batch(self.B, 1, self.A, self.K, self.S, d["delta_lb"], inp.seed, d["rho"], d["lam"],
                            root_offset=self.root_offset, lib=self.lib)
            run_search(tb, inp, self.K, record=False)
            out.append(tb.get_roots_values())
        self.values = out

    def prepare(self):
        self.env_step()

    def check(self):
        pass

    def run(self, steps, before_step=None):
        for i in range(steps):
            if before_step is not None:
                before_step(i)
            self.env_step()


class WeightSync:
    """--broadcast-every N (BASELINE config #5, "self-play shard + RCCL weight broadcast"): before
    every N-th env step of the timed loop rank 0 publishes a new checkpoint index and every rank runs
    WeightBroadcaster.sync() (mazero_amd/weights.py): the index, then the --broadcast-map network's
    flat weights (one message per dtype) over the job's collective (RCCL on GPUs, gloo for
    --backend port), replacing the reference's Ray pull before an env step
    (selfplay_worker.py:371-375, storage.py:68-80).  checkpoint_interval 1, so every sync moves the
    weights.  Each rank times its own syncs on the host, the collective completed
    (stream-synchronised); the search graphs run on their own stream, which waits for the weights
    before the next env step."""

    def __init__(self, args, dev, stream=None):
        import torch.distributed as dist

        from mazero_amd.nets import make_net
        from mazero_amd.weights import WeightBroadcaster

        N, A = CONFIGS[args.broadcast_map]
        self.every, self.dev, self.stream = args.broadcast_every, dev, stream
        self.rank = dist.get_rank()
        self.net = make_net(N, A, seed=11 + self.rank, device=dev)  # different weights on every rank
        self.wb = WeightBroadcaster(self.net, src=0)
        self.bytes = sum(t.numel() * t.element_size() for t in self.wb.flat.tensors())
        self.index, self.calls, self.secs = 0, 0, 0.0

    def __call__(self, step):
        if step % self.every:
            return
        import torch

        t0 = time.perf_counter()
        if self.rank == 0:
            self.index += 1
            self.wb.publish(self.index)
        got = self.wb.sync()
        if self.dev.type == "cuda":
            cur = torch.cuda.current_stream(self.dev)
            cur.synchronize()
        self.secs += time.perf_counter() - t0
        self.calls += 1
        if got != self.index and self.rank == 0:
            raise RuntimeError(f"weight broadcast: sync returned checkpoint {got}, published {self.index}")

    def reset(self):
        self.calls, self.secs = 0, 0.0

    def record(self):
        return dict(syncs=self.calls, ms_per_sync=round(self.secs / max(1, self.calls) * 1e3, 4),
                    checkpoint=int(self.wb.model_index), transfers=int(self.wb.syncs))


def trace_mark(dev, k):
    """MZ_TRACE_MARKS=1 (profiling runs only): a one-element int16 fill -- FillFunctor<short> in a
    rocprofv3 kernel trace -- just outside the timed region, so scripts/trace_window.py can cut the
    timed region's dispatches out of the trace.  Never inside the timed region."""
    if os.environ.get("MZ_TRACE_MARKS") != "1" or dev.type != "cuda":
        return
    import torch

    torch.full((1,), k, dtype=torch.int16, device=dev)


def timed(leg, steps, world, dist, sync, dev, before_step=None):
    """EXACTLY `steps` env steps between barrier + device synchronisation on both sides; the max
    over ranks of the wall time, and this rank's own.  `before_step(i)` (the weight broadcast of
    --broadcast-every) runs inside the timed region."""
    trace_mark(dev, 1)
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    leg.run(steps, before_step)
    sync()
    elapsed = time.perf_counter() - t0
    own = elapsed
    trace_mark(dev, 2)
    if world > 1:
        import torch

        dist.barrier()
        tt = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    leg.check()
    return elapsed, own


def rank_record(rank, local, dev, legs, steps):
    """What one rank ran on, for the N > 1 line: its device (index, name, PCI bus id) and its own
    ms per env step in each leg (the line's value uses the max over ranks)."""
    rec = dict(rank=rank, local_rank=local, device=str(dev))
    if dev.type == "cuda":
        import torch

        p = torch.cuda.get_device_properties(dev)
        rec["device_name"] = p.name
        bus = getattr(p, "pci_bus_id", None)
        if bus is not None:
            rec["pci_bus_id"] = int(bus)
    rec["ms_per_step"] = {k: round(v["own"] / steps * 1e3, 4) for k, v in legs.items()}
    bc = {k: v["broadcast"] for k, v in legs.items() if v.get("broadcast")}
    if bc:
        rec["weight_broadcast"] = bc
    return rec


def segv_maps():
    """MZ_SEGV_MAPS=<file> (profiler-crash diagnosis only): on SIGSEGV the faulting address, PC,
    thread and /proc/self/maps go to <file> (scripts/segv_maps.c), then the profiler's own handler
    runs; a run that completes writes the maps to <file>.exit at exit."""
    path = os.environ.get("MZ_SEGV_MAPS")
    if not path:
        return
    import atexit
    import ctypes

    so = os.path.join(os.path.dirname(os.path.abspath(__file__)), "scripts", "_segv_maps.so")
    lib = ctypes.CDLL(so)
    lib.mz_segv_maps_install(path.encode())
    atexit.register(lambda: lib.mz_segv_maps_snapshot((path + ".exit").encode()))


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch(args))
    segv_maps()
    import torch
    import torch.distributed as dist

    from mazero_amd.shard import shard_bounds, slice_inputs
    from mazero_amd.synthetic import make_search_inputs

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    hip = args.backend == "hip"
    if hip:
        torch.cuda.set_device(local if world > 1 else 0)
        dev = torch.device("cuda", torch.cuda.current_device())
    else:
        dev = torch.device("cpu")
    if world > 1:
        if hip:
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
        world = dist.get_world_size()
        rank = dist.get_rank()
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the job has {world} rank(s)")
    if args.broadcast_every < 0:
        raise SystemExit("bench.py: --broadcast-every must be >= 0")
    if args.broadcast_every and not dist.is_initialized():
        # one rank: a single-rank group, so that the broadcast runs the same collective code path
        import socket

        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        kw = dict(device_id=dev) if hip else {}
        dist.init_process_group("nccl" if hip else "gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0,
                                world_size=1, **kw)
    sync = torch.cuda.synchronize if hip else (lambda: None)
    N, A = CONFIGS[args.map]
    S, K = args.sims, args.sampled_times

    if hip:
        from mazero_amd._lib import load

        lib = load()
        stream = torch.cuda.Stream()

        def make_leg(inputs, off):
            if args.dropin:
                return DropinLeg(args, inputs, off, lib)
            return HipLeg(args, inputs, off, lib, dev, stream)
    else:
        def make_leg(inputs, off):
            return PortLeg(args, inputs, off)

    # weak scaling (headline): every rank owns --roots roots of its own (global root offset rank * roots)
    # strong scaling: the --roots roots of one global batch split over the ranks, rank r searching
    #   rows [lo, hi) of every agent search's inputs (global root offset lo)
    # (one leg at world size 1, where the two are the same job)
    legs = {}
    order = ["strong", "weak"] if args.strong else ["weak", "strong"]
    if world == 1:
        order = order[:1]
    for kind in order:
        if kind == "weak":
            B, off, total = args.roots, rank * args.roots, args.roots * world
            rng = np.random.default_rng(args.seed * 1000 + rank)
            inputs = [make_search_inputs(rng, B, A, S) for _ in range(N)]
        else:
            lo, hi = shard_bounds(args.roots, world, rank)
            B, off, total = hi - lo, lo, args.roots
            rng = np.random.default_rng(args.seed * 1000)
            inputs = [make_search_inputs(rng, args.roots, A, S) for _ in range(N)]
            if world > 1:
                inputs = [slice_inputs(inp, lo, hi) for inp in inputs]
        leg = make_leg(inputs, off)
        leg.prepare()
        wsync = None
        if args.broadcast_every:
            wsync = WeightSync(args, dev, stream if hip else None)
            wsync(0)  # (warm-up: the first sync allocates the collective's buffers)
            wsync.reset()
        st0 = leg.stats() if hip and rank == 0 and not args.dropin else None
        elapsed, own = timed(leg, args.steps, world, dist, sync, dev, wsync)
        st1 = leg.stats() if hip and rank == 0 and not args.dropin else None
        legs[kind] = dict(kind=kind, leg=leg, B=B, total=total, elapsed=elapsed, own=own, st0=st0, st1=st1,
                          broadcast=None if wsync is None else wsync.record(), wsync=wsync)
    # N > 1: every rank's device and its own step time, gathered to rank 0, and the collective's
    # view of the job (the line checks itself against the launcher's world size)
    ranks = None
    if world > 1:
        recs = [None] * world
        dist.all_gather_object(recs, rank_record(rank, local, dev, legs, args.steps))
        ranks = dict(world_size=dist.get_world_size(), backend=str(dist.get_backend()), per_rank=recs,
                     distinct_devices=len({(r["device"], r.get("pci_bus_id")) for r in recs}))

    main_kind = order[0]
    m = legs[main_kind]
    value = m["total"] * S * N * args.steps / m["elapsed"]
    roofline = None
    if hip and rank == 0 and not args.dropin:
        roofline = m["leg"].roofline(m["st0"], m["st1"], args.steps)
    cpu = None
    if hip and rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(m["leg"].host_inputs, m["B"], A, K, S, N, args.cpu_seconds, args.cpu_procs,
                           ptree=args.map == "matrix")

    if rank == 0:
        other = {}
        for kind, lg in legs.items():
            if kind == main_kind:
                continue
            other[f"{kind}_scaling"] = dict(
                value=round(lg["total"] * S * N * args.steps / lg["elapsed"], 1),
                unit="simulations/s",
                ms_per_step=round(lg["elapsed"] / args.steps * 1e3, 4),
                roots_total=lg["total"],
                roots_per_gpu=lg["B"],
                steps=args.steps,
            )
        if args.map == "3m" and args.roots == 256 and S == 50:
            # (the per-search workload of BASELINE.json's metric on every GPU for the weak leg, split over
            # the GPUs for the strong one; config.roots_total / roots_per_gpu say which)
            metric = "MCTS simulations/sec (whole node), SMAC 3m, 256 roots×50 sims, 1/2/4/8 GPUs"
        else:
            metric = (f"MCTS simulations/sec (whole node), SMAC {args.map}, {args.roots} roots×{S} sims"
                      + (" per GPU" if main_kind == "weak" and world > 1 else ""))
        if args.dropin:
            metric = (f"MCTS simulations/sec, tree-level drop-in (reference driver loop on mazero_amd.cytree, "
                      f"host numpy arrays), SMAC {args.map}, {m['total']} roots×{S} sims")
        line = {
            "metric": metric,
            "value": round(value, 1),
            "unit": "simulations/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(m["elapsed"] / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": main_kind,
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (device-resident network outputs + hidden-state pool, SURVEY §8d)" if hip
            else "synthetic; --backend port: CPU port on every rank (plumbing test, not a measurement)",
            "config": {
                "workload": f"SMAC {args.map} self-play search: {N} sequential agent searches x {m['B']} roots/GPU "
                            f"x {S} sims",
                "map": args.map,
                "agents": N,
                "actions": A,
                "roots_per_gpu": m["B"],
                "roots_total": m["total"],
                "sims": S,
                "sampled_times": K,
                "hidden": N * 128,
                "graph": hip and not args.no_graph and not args.dropin,
                "dropin": bool(args.dropin),
                "backend": args.backend,
                "parallelism": (f"{world} GPU(s), {m['B']} roots each, no collective on the data path"
                                if main_kind == "weak" else
                                f"{m['total']} roots sharded over {world} GPU(s), no collective on the data path"),
            },
            **other,
            **({"ranks": ranks} if ranks is not None else {}),
            **({"weight_broadcast": weight_broadcast_line(args, m, ranks)} if args.broadcast_every else {}),
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


def weight_broadcast_line(args, m, ranks):
    """The --broadcast-every fields of the line: what moved and each rank's own time per sync in the
    headline leg (rank 0's own beside them)."""
    rec = dict(every_steps=args.broadcast_every, network=f"{args.broadcast_map} MuZero-shaped (mazero_amd.nets)",
               bytes=m["wsync"].bytes, src_rank=0, checkpoint_interval=1, **m["broadcast"])
    if ranks is not None:
        rec["per_rank_ms_per_sync"] = [r.get("weight_broadcast", {}).get(m["kind"], {}).get("ms_per_sync")
                                       for r in ranks["per_rank"]]
    return rec


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
    return pm.get("workloads", {}).get(workload_key(args)) or None


def _cpu_worker(path, shards, B, A, K, S, budget_s, start, q):
    """One host process of the multi-core CPU baseline: this process's root shard of every agent
    search, searched with the CPU tree library until the budget is spent (tree calls only)."""
    from mazero_amd import _capi
    from mazero_amd.cytree import Tree_batch
    from mazero_amd.synthetic import DEFAULTS

    lib = _capi.bind(C.CDLL(path))
    d = DEFAULTS
    c2, c1, g = d["pb_c_base"], d["pb_c_init"], d["discount"]
    start.wait()
    n_sims, t_run, t0 = 0, 0.0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        for inp in shards:
            tb = Tree_batch(inp.B, 1, A, K, S, d["delta_lb"], inp.seed, d["rho"], d["lam"], lib=lib)
            ts = time.perf_counter()
            tb.prepare(inp.root_reward, inp.root_value, inp.root_policy, inp.root_beta, K, inp.noise_eps,
                       inp.root_noise)
            for s in range(S):
                tb.batch_selection(c2, c1, g)
                tb.batch_expansion_and_backup(s + 1, g, K, inp.reward[s], inp.value[s], inp.policy[s], inp.beta[s])
            tb.get_roots_values()
            tb.get_roots_marginal_visit_count()
            t_run += time.perf_counter() - ts
            n_sims += inp.B * S
    q.put((n_sims, t_run, time.perf_counter() - t0))


def ptree_baseline(host_inputs, B, A, K, S, N, budget_s):
    """BASELINE config #1's "pure-Python ptree" (oracle/ptree.py: the reference ships no Python tree,
    SURVEY §0): the same env steps through the pure-Python restatement of the ctree, one core, tree
    calls only."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import ptree

    from mazero_amd.synthetic import DEFAULTS

    d = DEFAULTS
    c2, c1, g = d["pb_c_base"], d["pb_c_init"], d["discount"]
    sims, t_run, steps = 0, 0.0, 0
    while t_run < budget_s:
        for inp in host_inputs:
            tb = ptree.Tree_batch(B, 1, A, K, S, d["delta_lb"], inp.seed, d["rho"], d["lam"])
            t0 = time.perf_counter()
            tb.prepare(inp.root_reward, inp.root_value, inp.root_policy, inp.root_beta, K, inp.noise_eps,
                       inp.root_noise)
            for s in range(S):
                tb.batch_selection(c2, c1, g)
                tb.batch_expansion_and_backup(s + 1, g, K, inp.reward[s], inp.value[s], inp.policy[s], inp.beta[s])
            tb.get_roots_values()
            tb.get_roots_marginal_visit_count()
            t_run += time.perf_counter() - t0
            sims += B * S
        steps += 1
    return {"value": round(sims / t_run, 1), "unit": "simulations/s", "cores": 1, "kind": "port",
            "sample": f"{steps} env steps x {N} searches x {B} roots x {S} sims (K={K}) = {sims} sims, "
                      f"{t_run:.1f} s of tree calls, pure-Python ptree (oracle/ptree.py)"}


def physical_cores():
    """Physical cores of the host (distinct (physical id, core id) pairs in /proc/cpuinfo), or None."""
    try:
        pairs, phys_id = set(), None
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("physical id"):
                    phys_id = line.split(":", 1)[1].strip()
                elif line.startswith("core id"):
                    pairs.add((phys_id, line.split(":", 1)[1].strip()))
        return len(pairs) or None
    except OSError:
        return None


def cpu_quota():
    """This process's CPU bandwidth limit from its cgroup (v2 cpu.max, else v1 cfs quota/period):
    {"cpus": quota / period or None when unlimited, "source": file, "raw": its content}, or None."""
    cands = ["/sys/fs/cgroup/cpu.max"]
    try:  # the process's own cgroup path (v2 "0::/path", v1 "...:cpu,cpuacct:/path")
        with open("/proc/self/cgroup") as f:
            for line in f:
                parts = line.strip().split(":", 2)
                if len(parts) == 3 and parts[0] == "0":
                    cands.insert(0, "/sys/fs/cgroup" + parts[2].rstrip("/") + "/cpu.max")
                elif len(parts) == 3 and "cpu" in parts[1].split(","):
                    cands.append(("/sys/fs/cgroup/cpu,cpuacct" + parts[2].rstrip("/"), "v1"))
    except OSError:
        pass
    cands += [("/sys/fs/cgroup/cpu,cpuacct", "v1"), ("/sys/fs/cgroup/cpu", "v1")]
    for c in cands:
        try:
            if isinstance(c, tuple):
                with open(c[0] + "/cpu.cfs_quota_us") as f:
                    q = int(f.read().strip())
                with open(c[0] + "/cpu.cfs_period_us") as f:
                    per = int(f.read().strip())
                return {"cpus": round(q / per, 3) if q > 0 else None, "source": c[0] + "/cpu.cfs_{quota,period}_us",
                        "raw": f"{q} {per}"}
            with open(c) as f:
                raw = f.read().strip()
            q, per = raw.split()[:2]
            return {"cpus": None if q == "max" else round(int(q) / int(per), 3), "source": c, "raw": raw}
        except (OSError, ValueError):
            continue
    return None


def cpu_baseline(host_inputs, B, A, K, S, N, budget_s, procs=16, ptree=False):
    """The reference CPU ctree (or the CPU port), one host core, tree calls only, same inputs; plus
    SURVEY §8(d)(ii): the same env steps on several host cores at once, one process per core with
    the roots sharded over the processes ("multi_core"); plus, for BASELINE config #1 (`ptree`),
    the pure-Python ptree on the same env steps."""
    import multiprocessing as mp

    from mazero_amd import _capi
    from mazero_amd.cytree import Tree_batch
    from mazero_amd.shard import shard_bounds, slice_inputs
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
    # (ii) one process per core, the roots of every search sharded over the processes (each
    # process's trees are seeded locally: the work per tree is the same as in the sharded batch)
    try:
        share = sorted(os.sched_getaffinity(0))
    except AttributeError:
        share = list(range(os.cpu_count() or 1))
    # the CPU time this job may use: the affinity mask lists every CPU of the host on a GPU box, the
    # cgroup's bandwidth quota is what bounds it (one GPU's share of the node)
    quota = cpu_quota()
    q_cpus = int(quota["cpus"]) if quota and quota["cpus"] else None
    n_proc = max(1, min(procs, len(share), B, q_cpus or procs))
    ctx = mp.get_context("spawn")  # a fresh interpreter per worker (this process may hold the GPU)
    start, q = ctx.Event(), ctx.Queue()
    workers = []
    for k in range(n_proc):
        lo, hi = shard_bounds(B, n_proc, k)
        shards = [slice_inputs(inp, lo, hi) for inp in host_inputs]
        w = ctx.Process(target=_cpu_worker, args=(path, shards, B, A, K, S, budget_s / 2, start, q), daemon=True)
        w.start()
        workers.append(w)
    time.sleep(0.5)
    start.set()
    res = [q.get(timeout=budget_s * 4 + 60) for _ in workers]
    for w in workers:
        w.join(timeout=30)
    wall = max(r[2] for r in res)
    total = sum(r[0] for r in res)
    multi = {"value": round(total / wall, 1), "processes": n_proc, "cores": n_proc, "cgroup_cpu_quota": quota,
             "sample": f"{total} sims in {wall:.1f} s wall: {n_proc} processes, each searching its shard of "
                       f"the {B} roots of every agent search ({kind} ctree)"}
    # the whole host: a GPU box grants this job one GPU's share of the node's CPUs (16), so every
    # physical core cannot be measured there; the projection scales the measured per-process rate
    phys = physical_cores()
    if phys:
        multi["whole_host_projection"] = {
            "value": round(total / wall / n_proc * phys, 1), "cores": phys,
            "basis": f"measured rate per process at {n_proc} processes x {phys} physical cores (linear: an upper "
                     f"bound on the reference ctree's whole-host throughput); not measured: this job's cgroup "
                     f"grants {quota['cpus'] if quota else 'an unknown number of'} CPUs of bandwidth "
                     f"({quota['source'] + ' = ' + quota['raw'] if quota else 'no cgroup limit file found'}), "
                     f"while the affinity mask lists {len(share)}"}
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
        "cpu_model": cpu_model,
        "sample": f"{steps} env steps x {N} searches x {B} roots x {S} sims (K={K}) = {sims} sims, "
                  f"{tree_time:.1f} s of tree calls on 1 core of '{cpu_model}' (nproc {os.cpu_count()}, "
                  f"this process's share {len(share)})",
        "multi_core": multi,
        **({"ptree": ptree_baseline(host_inputs, B, A, K, S, N, budget_s / 2)} if ptree else {}),
    }


if __name__ == "__main__":
    main()
