"""The documents against the committed measurements and the tree (CPU).

DESIGN.md / README.md / INTEGRATION.md / scripts/README.md quote numbers from `profiles/` and name
files of this repository.  These checks keep them from drifting: every repository file they name
exists, README's headline is the committed headline bench line, and DESIGN §5's configuration table
is the committed reconciliation (`profiles/round6/roofline_reconcile.json`)."""
from __future__ import annotations

import json
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DOCS = ["DESIGN.md", "README.md", "INTEGRATION.md", os.path.join("scripts", "README.md")]
ROUND = os.path.join(ROOT, "profiles", "round6")

# names of the reference's own sources (in /root/reference, cited by file:line) and of files a
# document says are gone
NOT_OURS = {"cnode.cpp", "utils.cpp", "cnode.h", "cytree.pyx", "ctree.pxd", "mazero_amd/_hipenv.py"}
# per-configuration files of profiles/<round>/<config>/
PER_CONFIG = {"bench.json", "traced.json", "pmc_summary.txt", "rocprof_kernel_stats.csv",
              "rocprof_timed_window.json"}


def _read(doc: str) -> str:
    with open(os.path.join(ROOT, doc)) as f:
        return f.read()


@pytest.mark.parametrize("doc", DOCS)
def test_named_files_exist(doc):
    text = _read(doc)
    names = set(re.findall(r"`([A-Za-z0-9_./-]+\.(?:py|sh|hip|json|jsonl|md|h|cpp|log|npz|txt|csv))`", text))
    missing = []
    for n in sorted(names):
        if n in NOT_OURS or n.startswith(("core/", "common_lib/", "config/")) or os.path.basename(n) in NOT_OURS:
            continue
        if n in PER_CONFIG:
            assert os.path.exists(os.path.join(ROUND, "3m_k1", n)), n
            continue
        cands = [n] + [os.path.join(d, n) for d in ("scripts", "mazero_amd", "mazero_amd/csrc", "oracle", "include",
                                                     "tests", "profiles/round6", "profiles/round6/ab", "profiles/round5", "profiles/round4", "profiles/round3",
                                                     "profiles")]
        if not any(os.path.exists(os.path.join(ROOT, c)) for c in cands):
            missing.append(n)
    assert not missing, f"{doc} names files that do not exist: {missing}"


def _bench(config: str) -> dict:
    with open(os.path.join(ROUND, config, "bench.json")) as f:
        return json.loads(f.readline())


def test_readme_headline_is_the_committed_line():
    b = _bench("3m_k1")
    m = re.search(r"\*\*([0-9.]+) M\s+simulations/s\*\*", _read("README.md"))
    assert m, "README's headline sentence"
    assert abs(float(m.group(1)) - b["value"] / 1e6) < 0.05
    cpu = b["cpu_baseline"]["value"]
    r = re.search(r"([0-9,]+)×\s+the reference ctree on one host core", _read("README.md"))
    assert r and abs(int(r.group(1).replace(",", "")) - b["value"] / cpu) <= 1


def test_design_table_is_the_committed_reconciliation():
    with open(os.path.join(ROUND, "roofline_reconcile.json")) as f:
        rec = json.load(f)
    rows = {}
    text = _read("DESIGN.md")
    sec = text[text.index("### Round 6 (`profiles/round6/`)"):text.index("### Round 5 (for the record")]
    for line in sec.splitlines():
        m = re.match(r"\| (3m|2s3z|3s5z_vs_3s6z|27m_vs_30m) (\d+)×(\d+) K=(\d+) \| ([0-9.]+) M \| [^|]+\| ([0-9.]+) µs \|",
                     line)
        if m:
            key = {"3m": "3m", "2s3z": "2s3z", "3s5z_vs_3s6z": "3s5z", "27m_vs_30m": "27m"}[m.group(1)] + f"_k{m.group(4)}"
            rows[key] = (float(m.group(5)), float(m.group(6)))
    assert set(rows) == set(rec), (sorted(rows), sorted(rec))
    for k, (msims, us) in rows.items():
        assert abs(msims - rec[k]["value"] / 1e6) < 0.05, k
        assert abs(us - rec[k]["avg_launch_us"]) < 0.006, k
