"""Reconcile bench.py's roofline numbers with rocprofv3 (scripts/profile_configs.sh output).

    python scripts/reconcile.py gpurun_out/prof --out gpurun_out/prof/summary.json

Per configuration directory (bench.json, traced.json, trace/*kernel_stats.csv, PMC summary):
  frac              bench.json's roofline.frac: algorithmic bytes per fused launch / the fused
                    kernel's average duration from HIP events (no profiler attached)
  traced_event_us   the same HIP-event measurement inside the run traced by rocprofv3
  rocprof_mean_us   rocprofv3's mean duration of the fused kernel in that same run
  agree             traced_event_us / rocprof_mean_us: the two clocks measure the same thing
  profiler_slowdown traced_event_us / bench avg_launch_us: what the kernel tracing itself costs
  frac_rocprof      bytes per launch / rocprof_mean_us / 8 TB/s: frac recomputed from the committed
                    profile's own per-dispatch durations (taken under the profiler)
  step_sum_ms       rocprof_mean_us x the fused launches of one env step, against bench.json's
                    ms_per_step (the fused kernel alone must fit in the measured step)
  traffic           PMC bytes per fused launch, 2 x FETCH_SIZE + WRITE_SIZE (raw beside it), and
                    its ratio to the algorithmic bytes
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os


def last_json(path):
    with open(path) as f:
        lines = [x for x in f if x.startswith("{")]
    return json.loads(lines[-1])


def fused_stats(trace_dir):
    files = glob.glob(os.path.join(trace_dir, "**", "*kernel_stats.csv"), recursive=True)
    for f in files:
        for r in csv.DictReader(open(f)):
            nm = r["Name"]
            if (("k_chain<" in nm or "k_tree<" in nm) and ", true>" in nm) or ("k_chain3<" in nm and ", true," in nm) \
                    or "k_step<true, true" in nm or "k_hbm<true, true" in nm:
                return dict(calls=int(r["Calls"]), mean_ns=float(r["AverageNs"]), min_ns=float(r["MinNs"]),
                            max_ns=float(r["MaxNs"]), total_ns=float(r["TotalDurationNs"]))
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--out", required=True)
    ap.add_argument("--pmc", default=None, help="pmc_latest.json (default: <root>/../pmc_latest.json)")
    args = ap.parse_args()
    pmc_path = args.pmc or os.path.join(os.path.dirname(os.path.abspath(args.root)), "pmc_latest.json")
    pmc = json.load(open(pmc_path)).get("workloads", {}) if os.path.exists(pmc_path) else {}
    out = {}
    for d in sorted(glob.glob(os.path.join(args.root, "*", ""))):
        name = os.path.basename(os.path.dirname(d))
        try:
            b = last_json(os.path.join(d, "bench.json"))
            t = last_json(os.path.join(d, "traced.json"))
        except (OSError, IndexError, ValueError):
            continue
        rb, rt = b["roofline"], t["roofline"]
        fs = fused_stats(os.path.join(d, "trace"))
        c = b["config"]
        key = f"{c['map']}:B{c['roots_per_gpu']}:S{c['sims']}:K{c['sampled_times']}"
        e = dict(
            workload=key,
            value=b["value"],
            ms_per_step=b["ms_per_step"],
            bytes_per_launch=rb["bytes_per_launch"],
            avg_launch_us=rb["avg_launch_us"],
            frac=rb["frac"],
            traced_value=t["value"],
            traced_event_us=rt["avg_launch_us"],
        )
        if fs:
            slow = rt["avg_launch_us"] / rb["avg_launch_us"]
            e.update(
                rocprof_calls=fs["calls"],
                rocprof_mean_us=round(fs["mean_ns"] / 1e3, 3),
                agree=round(rt["avg_launch_us"] / (fs["mean_ns"] / 1e3), 4),
                profiler_slowdown=round(slow, 4),
                frac_rocprof=round(rb["bytes_per_launch"] / (fs["mean_ns"] / 1e3) / 1e3 / 8000.0, 6),
                frac_rocprof_over_frac=round(rb["bytes_per_launch"] / (fs["mean_ns"] / 1e3) / 1e3 / 8000.0
                                             / rb["frac"], 4),
                step_sum_ms=round(fs["mean_ns"] * c["agents"] * (c["sims"] - 1) / 1e6, 4),
            )
        p = pmc.get(key)
        if p and p.get("fused_bytes_per_launch"):
            e.update(
                traffic=p.get("fused_bytes_per_launch_corrected"),
                traffic_raw=p["fused_bytes_per_launch"],
                traffic_over_algorithmic=round(p.get("fused_bytes_per_launch_corrected") / rb["bytes_per_launch"], 3),
            )
        out[name] = e
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    json.dump(out, open(args.out, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
