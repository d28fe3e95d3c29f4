#!/bin/bash
# Round-4 GPU-box pass.  STEPS (default "pytest bench"): any of
#   pytest   the whole -m gpu suite (PYTEST_ARGS to narrow it)
#   smoke    __graft_entry__.smoke()
#   bench    headline bench line (bench.py, defaults)
#   configs  bench.py --no-cpu over CONFIGS ("name:args;name:args", default: every K>1 config)
#   dropin   bench.py --dropin at 3m K=1 and K=5
#   ab       interleaved A/B against each ALTS build (default: the round-3 build)
#   stamps   MZ_STAMPS=1 phase cycles, K = 1 and K = 5
#   micro    scripts/_gridsize: launch period against grid and workgroup size
#   search   bench_search.py (full loop with a network) + a rocprofv3 kernel trace of it
# Every GPU step has its own time limit; any failure ends the script (no later GPU step runs).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS="${STEPS:-pytest bench}"
run() {  # name, limit, command...
    local name=$1 lim=$2
    shift 2
    echo "== $name: $*"
    timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    tail -3 "gpurun_out/$name.log"
    [ $rc -eq 0 ] || exit $rc
}
for st in $STEPS; do
    case $st in
        pytest) run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
                    --timeout-method thread ${PYTEST_ARGS} ;;
        smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
        bench) run bench 400 python bench.py ;;
        configs)
            IFS=';' read -ra CS <<< "${CONFIGS:-3m_k5:--sampled-times 5;3m_k10:--sampled-times 10;3s5z_k5:--map 3s5z_vs_3s6z --roots 512 --sims 100 --sampled-times 5;27m_k5:--map 27m_vs_30m --sims 200 --sampled-times 5}"
            for c in "${CS[@]}"; do
                run "cfg_${c%%:*}" 400 python bench.py --no-cpu ${c#*:}
            done ;;
        dropin)
            run dropin_k1 400 python bench.py --dropin --no-cpu --steps 10
            run dropin_k5 400 python bench.py --dropin --no-cpu --steps 10 --sampled-times 5
            run dropin_split 300 python scripts/dropin_split.py
            MZ_HOST_COPY=1 run dropin_split_copy 300 python scripts/dropin_split.py ;;
        ab)  # interleaved A/B of the product against each build in ALTS (default: the round-3 build)
            for alt in ${ALTS:-r3}; do
                ALT_TAG=$alt ALT=$PWD/mazero_amd/_build/variant_$alt.so run ab_$alt 900 bash scripts/ab_ktree.sh \
                    "${AB_CONFIGS:-3m_k1:--sampled-times 1;2s3z_k1:--map 2s3z --roots 1024;27m_k1:--map 27m_vs_30m --sims 200;3m_k5:--sampled-times 5;3m_k10:--sampled-times 10}"
                cat gpurun_out/ab_$alt.log
            done ;;
        stamps)  # per-phase cycles (MZ_STAMPS=1 diagnostic build) for K = 1 and K = 5
            MZ_STAMPS=1 run stamps_k1 300 python bench.py --no-cpu --steps 5
            MZ_STAMPS=1 run stamps_k5 300 python bench.py --no-cpu --steps 5 --sampled-times 5 ;;
        micro)  # launch period against grid / workgroup size (scripts/gridsize.hip, built beforehand)
            run gridsize 120 ./scripts/_gridsize ;;
        search)
            run search 600 python bench_search.py
            MZ_TRACE_MARKS=1 run search_trace 600 rocprofv3 --kernel-trace --stats --output-format csv \
                -d gpurun_out/search_prof -o search -- python3 bench_search.py --device-only --steps 3
            run search_split 60 python scripts/search_split.py gpurun_out/search_prof \
                --line gpurun_out/search_trace.log --out gpurun_out/bench_search_trace.json ;;
        *) echo "unknown step $st"; exit 2 ;;
    esac
done
exit 0
