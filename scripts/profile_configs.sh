#!/bin/bash
# Measurement pass over the BASELINE.json configurations that fit one GPU: for each one
#   bench.json         bench.py as the driver runs it (headline also with the CPU baseline)
#   traced.json        bench.py under rocprofv3 --kernel-trace --stats (its own HIP-event timing
#                      of the fused kernel, taken under the profiler)
#   trace/             the rocprofv3 kernel trace + stats of that run
#   window.json        that trace cut to the timed region (scripts/trace_window.py)
#   pmc_fetch/, pmc_write/   separate --pmc FETCH_SIZE / WRITE_SIZE passes
# then scripts/pmc_summary.py (-> gpurun_out/pmc_latest.json) and scripts/reconcile.py
# (-> gpurun_out/prof/summary.json).  CONFIGS="3m_k1 ..." selects a subset.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
R=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
declare -A ARGS=(
  [3m_k1]="--map 3m --roots 256 --sims 50 --sampled-times 1"
  [3m_k5]="--map 3m --roots 256 --sims 50 --sampled-times 5"
  [3m_k10]="--map 3m --roots 256 --sims 50 --sampled-times 10"
  [3s5z_k10]="--map 3s5z_vs_3s6z --roots 512 --sims 100 --sampled-times 10"
  [2s3z_k1]="--map 2s3z --roots 1024 --sims 50 --sampled-times 1"
  [3s5z_k5]="--map 3s5z_vs_3s6z --roots 512 --sims 100 --sampled-times 5"
  [27m_k1]="--map 27m_vs_30m --roots 256 --sims 200 --sampled-times 1"
  [27m_k5]="--map 27m_vs_30m --roots 256 --sims 200 --sampled-times 5"
  [27m_k16]="--map 27m_vs_30m --roots 256 --sims 200 --sampled-times 16"
)
CONFIGS=${CONFIGS:-"3m_k1 3m_k5 3m_k10 2s3z_k1 3s5z_k5 3s5z_k10 27m_k1 27m_k5 27m_k16"}
# the PMC passes run first, so the bench lines carry this build's traffic (bench.py reads
# profiles/pmc_latest.json; on the box that copy is refreshed after every configuration)
cp profiles/pmc_latest.json gpurun_out/pmc_latest.json 2>/dev/null
step() {  # log timeout cmd...
    local log=$1 to=$2; shift 2
    timeout -k 10 "$to" "$@" > "$log" 2> "$log.err"
    local rc=$?
    echo "  $(basename "$log") rc=$rc"
    [ $rc -ne 0 ] && { tail -5 "$log.err"; exit $rc; }
    return 0
}
for c in $CONFIGS; do
    a=${ARGS[$c]}
    d=gpurun_out/prof/$c
    mkdir -p "$d"
    echo "== $c ($a)"
    cpu="--no-cpu"; [ "$c" = 3m_k1 ] && cpu=""
    # (27m: 27 agent searches x 200 sims = 5,400 fused dispatches per env step; rocprofv3's PMC
    # collection crashed on the host at --steps 3, so those passes profile one step)
    # (27m K = 1 under --pmc with the env step captured as one graph of 5,481 kernel nodes: rocprofv3
    # segfaults a few seconds into the replay, inside librocprofiler-sdk on an HSA runtime thread,
    # profiles/round5/pmc_crash_27m_k1_graph_analysis.txt; the 27m PMC passes launch eagerly,
    # --no-graph, the same kernels)
    ps="--steps 3 --warmup 1"; case $c in 27m*) ps="--steps 1 --warmup 1 --no-graph";; esac
    step "$d/pmc_fetch.json" 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/$d/pmc_fetch" -o run -- \
        python3 "$R/bench.py" --no-cpu $ps $a
    step "$d/pmc_write.json" 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/$d/pmc_write" -o run -- \
        python3 "$R/bench.py" --no-cpu $ps $a
    step "$d/pmc_summary.txt" 120 python scripts/pmc_summary.py "$d/pmc_fetch" "$d/pmc_write" --bench-args "$a" \
        --out gpurun_out/pmc_latest.json
    cp gpurun_out/pmc_latest.json profiles/pmc_latest.json
    step "$d/bench.json" 300 python bench.py $a $cpu
    # (MZ_TRACE_MARKS: fill kernels just outside the timed region, so trace_window.py can cut it out)
    export MZ_TRACE_MARKS=1
    step "$d/traced.json" 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$d/trace" -o run -- \
        python3 "$R/bench.py" --no-cpu $a
    unset MZ_TRACE_MARKS
    python scripts/trace_window.py "$d/trace" --bench "$d/traced.json" --out "$d/window.json" > /dev/null || exit 3
    # keep the summaries: per-dispatch traces and counter dumps of the 27m workloads are > 64 MiB
    python scripts/reconcile.py gpurun_out/prof --out gpurun_out/prof/summary.json > /dev/null || exit $?
    find "$d" -name "*kernel_trace.csv" -o -name "*counter_collection.csv" | xargs -r rm -f
done
python scripts/reconcile.py gpurun_out/prof --out gpurun_out/prof/summary.json
