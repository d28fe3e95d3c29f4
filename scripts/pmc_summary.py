"""Summarise rocprofv3 --pmc passes of bench.py into profiles/pmc_latest.json.

    python scripts/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write --bench-args '' \\
        --out profiles/pmc_latest.json

FETCH_SIZE / WRITE_SIZE are kilobytes per dispatch (TCC_EA0_RDREQ / _WRREQ based).  Per
MI355X_MICROARCH.md §HBM, FETCH_SIZE reads half the bytes of a wide (16 B/lane) coalesced stream
and other widths are uncalibrated; both are recorded per launch: `fused_bytes_per_launch` is the
raw FETCH_SIZE + WRITE_SIZE in bytes, `fused_bytes_per_launch_corrected` = 2 x FETCH_SIZE +
WRITE_SIZE (the guide's correction, what bench.py reports as roofline.traffic).
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import json
import os
import re
import shlex
import sys


def read(dirname, counter):
    files = glob.glob(os.path.join(dirname, "*counter_collection.csv"))
    per = collections.defaultdict(list)
    for f in files:
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                per[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in per.items()}, {k: len(v) for k, v in per.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--bench-args", default="", help="the bench.py arguments of the profiled run")
    ap.add_argument("--out", default="profiles/pmc_latest.json")
    args = ap.parse_args()
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
    import bench
    key = bench.workload_key(bench.parse(shlex.split(args.bench_args)))
    fetch, nf = read(args.fetch_dir, "FETCH_SIZE")
    write, nw = read(args.write_dir, "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        short = k.replace("void ", "").replace("(anonymous namespace)::", "")
        short = re.sub(r"\(.*$", "", short).replace(" ", "")
        kernels[short] = dict(fetch_kb=fetch.get(k), write_kb=write.get(k), dispatches=max(nf.get(k, 0), nw.get(k, 0)))
    def is_fused(k):  # the per-simulation fused kernel: k_chain3 / k_chain / k_tree with selection, or k_step<true,true>
        return ((k.startswith("k_chain<") or k.startswith("k_tree<")) and k.endswith(",true>")) or \
            (k.startswith("k_chain3<") and ",true," in k) or k.startswith("k_step<true,true") or \
            k.startswith("k_hbm<true,true")
    fused = next((v for k, v in kernels.items() if is_fused(k)), {})
    out = {}
    if os.path.exists(args.out):
        out = json.load(open(args.out))
    out.setdefault("workloads", {})[key] = dict(
        kernels=kernels,
        fused_bytes_per_launch=None if not fused else round((fused["fetch_kb"] + fused["write_kb"]) * 1024),
        fused_bytes_per_launch_corrected=None if not fused else round((2 * fused["fetch_kb"] + fused["write_kb"]) * 1024),
        note="FETCH_SIZE/WRITE_SIZE in KB per dispatch, means over all dispatches of the profiled run",
    )
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    json.dump(out, open(args.out, "w"), indent=1)
    print(json.dumps(out["workloads"][key], indent=1))


if __name__ == "__main__":
    main()
