"""Split the full search loop's GPU time per simulation into model, glue, tree and copies.

    MZ_TRACE_MARKS=1 rocprofv3 --kernel-trace --stats --output-format csv -d DIR -o search -- \
        python3 bench_search.py --device-only --steps S > line.json
    python scripts/search_split.py DIR --line line.json --out profiles/round4/bench_search_trace.json

The two FillFunctor<short> marks bracket bench_search.py's timed region (env steps of graph-replayed
searches, each followed by the host readback).  Every dispatch between them is classified by name:
  tree    the mz kernels of the tree library (k_prepare, k_chain*, k_tree, k_step, k_readback, ...)
  glue    the driver glue (k_policy_glue, k_joint_action, k_root_glue)
  copies  torch copy / fill kernels (the hidden-state pool copy, input uploads, dtype casts)
  model   everything else (the network's GEMMs, norms, activations, reductions)
Per simulation = the window's totals / (steps x agents x sims).  `span` is the window's wall time on
the device clock; span minus the dispatch durations is time the GPU had no kernel running (launch
boundaries, host work: root preprocessing, readbacks).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from trace_window import load_trace, short, window  # noqa: E402

TREE = ("k_prepare", "k_chain", "k_tree", "k_step", "k_readback", "k_copy_words", "k_set_word", "k_gather")
GLUE = ("k_policy_glue", "k_joint_action", "k_root_glue")
COPY_HINTS = ("copy", "Copy", "fill", "Fill", "cast", "Cast")


def category(name: str) -> str:
    n = short(name)
    base = n.split("<")[0].split("::")[-1]
    if base.startswith(TREE):
        return "tree"
    if base.startswith(GLUE):
        return "glue"
    if any(h in n for h in COPY_HINTS):
        return "copies"
    return "model"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("--line", required=True, help="bench_search.py --device-only's JSON line")
    ap.add_argument("--out")
    a = ap.parse_args()
    line = json.loads([x for x in open(a.line).read().splitlines() if x.startswith("{")][-1])
    win = window(load_trace(a.trace_dir))
    steps = int(line["steps"])
    import re

    m = re.search(r"\((\d+) agents x (\d+) roots x (\d+) sims", line["metric"])
    N, B, S = (int(x) for x in m.groups())
    sims = steps * N * S
    cats, kern = {}, {}
    for s, e, n in win:
        c = category(n)
        d = cats.setdefault(c, dict(dispatches=0, ns=0))
        d["dispatches"] += 1
        d["ns"] += e - s
        k = kern.setdefault(short(n), dict(category=c, dispatches=0, ns=0))
        k["dispatches"] += 1
        k["ns"] += e - s
    span = win[-1][1] - win[0][0]
    busy = sum(e - s for s, e, _ in win)
    out = dict(
        source="rocprofv3 --kernel-trace of bench_search.py --device-only (graph-replayed device loop), the timed "
               "region between the MZ_TRACE_MARKS fills",
        line=line, steps=steps, agents=N, roots=B, sims=S, simulations_per_root=sims,
        span_us_per_sim=round(span / sims / 1e3, 3), kernel_us_per_sim=round(busy / sims / 1e3, 3),
        idle_us_per_sim=round((span - busy) / sims / 1e3, 3),
        per_sim={c: dict(dispatches=round(v["dispatches"] / sims, 2), us=round(v["ns"] / sims / 1e3, 3))
                 for c, v in sorted(cats.items(), key=lambda kv: -kv[1]["ns"])},
        kernels={n: dict(category=v["category"], per_sim=round(v["dispatches"] / sims, 3),
                         us_per_sim=round(v["ns"] / sims / 1e3, 3), mean_us=round(v["ns"] / v["dispatches"] / 1e3, 3))
                 for n, v in sorted(kern.items(), key=lambda kv: -kv[1]["ns"])},
    )
    js = json.dumps(out, indent=1)
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            f.write(js + "\n")
    print(js)


if __name__ == "__main__":
    main()
