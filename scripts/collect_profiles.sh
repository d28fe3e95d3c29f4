#!/bin/bash
# Copy the judged pieces of a scripts/profile_configs.sh pass into profiles/<round>/<config>/
# (tracked): the bench line (plain and traced), the PMC summary and the rocprofv3 kernel stats;
# the pass's reconciliation entries are merged into profiles/<round>/roofline_reconcile.json (the
# configurations it did not profile keep their entries) and profiles/pmc_latest.json is refreshed.
# Usage: scripts/collect_profiles.sh round2
cd "$(dirname "$0")/.." || exit 2
dst=profiles/${1:?round name}
mkdir -p "$dst"
for d in gpurun_out/prof/*/; do
    c=$(basename "$d")
    [ -f "$d/bench.json" ] || continue
    mkdir -p "$dst/$c"
    grep -h '^{' "$d/bench.json" > "$dst/$c/bench.json"
    grep -h '^{' "$d/traced.json" > "$dst/$c/traced.json"
    cp "$d/pmc_summary.txt" "$dst/$c/pmc_summary.txt"
    cp "$d/trace/run_kernel_stats.csv" "$dst/$c/rocprof_kernel_stats.csv"
    [ -f "$d/window.json" ] && cp "$d/window.json" "$dst/$c/rocprof_timed_window.json"
done
python - "$dst/roofline_reconcile.json" gpurun_out/prof/summary.json <<'PY'
import json, os, sys
out, new = sys.argv[1], json.load(open(sys.argv[2]))
cur = json.load(open(out)) if os.path.exists(out) else {}
cur.update(new)
json.dump(dict(sorted(cur.items())), open(out, "w"), indent=1)
PY
cp gpurun_out/pmc_latest.json profiles/pmc_latest.json
ls "$dst"
