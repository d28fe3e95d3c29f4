#!/bin/bash
# Copy the judged pieces of a scripts/profile_configs.sh pass into profiles/<round>/ (tracked):
# per configuration the bench lines (plain and traced) and the rocprofv3 kernel stats, plus the
# PMC summary and the reconciliation.  Usage: scripts/collect_profiles.sh round2
cd "$(dirname "$0")/.." || exit 2
dst=profiles/${1:?round name}
mkdir -p "$dst"
python scripts/reconcile.py gpurun_out/prof --out "$dst/roofline_reconcile.json" > /dev/null || exit 1
cp gpurun_out/pmc_latest.json "$dst/pmc_summary.json"
for d in gpurun_out/prof/*/; do
    c=$(basename "$d")
    [ -f "$d/bench.json" ] || continue
    grep -h '^{' "$d/bench.json" > "$dst/bench_$c.json"
    grep -h '^{' "$d/traced.json" > "$dst/bench_traced_$c.json"
    cp "$d/trace/run_kernel_stats.csv" "$dst/rocprof_kernel_stats_$c.csv"
done
ls "$dst"
