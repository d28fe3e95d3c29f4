"""Cut bench.py's timed region out of a rocprofv3 kernel trace and summarise it.

    MZ_TRACE_MARKS=1 rocprofv3 --kernel-trace --stats --output-format csv -d DIR -o run -- python3 bench.py ...
    python scripts/trace_window.py DIR --bench traced.json [--out window.json]

With MZ_TRACE_MARKS=1, bench.py launches a one-element int16 fill (FillFunctor<short>) just before
the barrier + synchronize that opens the timed region and just after the synchronize that closes
it.  Every dispatch between the two marks belongs to the timed region: the env steps' graph
replays and nothing else (no eager warm-up, no roofline replays).  Per kernel: dispatch count,
mean / median / min / max duration; for the whole window: the span from the first dispatch's start
to the last one's end, the sum of the dispatch durations and the gaps between consecutive
dispatches.  With --bench (the same run's JSON line) the window is checked against the run's own
ms_per_step and the fused kernel's HIP-event duration.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os

import numpy as np


def short(name: str) -> str:
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0]


def load_trace(d: str):
    files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no kernel_trace.csv under {d}")
    rows = []
    for f in files:
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    return rows


def window(rows):
    marks = [i for i, r in enumerate(rows) if "FillFunctor<short>" in r[2]]
    if len(marks) < 2:
        raise SystemExit(f"expected two FillFunctor<short> marks, found {len(marks)} (MZ_TRACE_MARKS=1?)")
    return rows[marks[0] + 1:marks[1]]


def summarise(win, steps=None):
    per = {}
    for s, e, n in win:
        per.setdefault(short(n), []).append(e - s)
    kernels = {}
    for n, ds in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        a = np.array(ds, dtype=np.float64)
        kernels[n] = dict(calls=len(ds), mean_ns=round(float(a.mean()), 1), median_ns=float(np.median(a)),
                          min_ns=float(a.min()), max_ns=float(a.max()), total_ns=float(a.sum()))
        if steps:
            kernels[n]["calls_per_step"] = len(ds) / steps
    st = np.array([r[0] for r in win], dtype=np.float64)
    en = np.array([r[1] for r in win], dtype=np.float64)
    gaps = st[1:] - en[:-1]
    out = dict(dispatches=len(win), span_ns=float(en.max() - st.min()), sum_durations_ns=float((en - st).sum()),
               gap_ns_mean=round(float(gaps.mean()), 1) if len(gaps) else None,
               gap_ns_median=float(np.median(gaps)) if len(gaps) else None, kernels=kernels)
    if steps:
        out["span_ms_per_step"] = round(out["span_ns"] / steps / 1e6, 4)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("--bench", help="the traced run's JSON line (bench.py stdout)")
    ap.add_argument("--out")
    a = ap.parse_args()
    b = None
    if a.bench:
        with open(a.bench) as f:
            b = json.loads([x for x in f if x.startswith("{")][-1])
    steps = b["steps"] if b else None
    res = summarise(window(load_trace(a.trace_dir)), steps)
    if b:
        fused = next((k for k in res["kernels"] if (("k_chain<" in k or "k_tree<" in k) and ", true>" in k)
                      or ("k_chain3<" in k and ", true," in k) or "k_hbm<true, true" in k), None)
        rb = b["roofline"]
        res["bench"] = dict(ms_per_step=b["ms_per_step"], value=b["value"], event_launch_us=rb["avg_launch_us"],
                            bytes_per_launch=rb["bytes_per_launch"], frac=rb["frac"])
        if fused:
            k = res["kernels"][fused]
            mean_us = k["mean_ns"] / 1e3
            res["fused"] = dict(kernel=fused, calls_per_step=k["calls_per_step"], mean_us=round(mean_us, 3),
                                mean_x_calls_ms=round(mean_us * k["calls_per_step"] / 1e3, 4),
                                fits_step=mean_us * k["calls_per_step"] / 1e3 <= b["ms_per_step"],
                                frac_from_trace=round(rb["bytes_per_launch"] / (mean_us * 1e-6) / 8e12, 6))
    txt = json.dumps(res, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main()
