#!/bin/bash
# Round-3 measurement pass (one GPU box).  STEPS selects: headline strong k10 spans trace search
# matrix dropin pytest spansv.
#   headline  bench.py at its defaults (3m 256x50 K=1, CPU legs included)
#   strong    the strong-scaling proxy: one rank's env step at B = 256/G roots (G = 8, 4, 2)
#   k10       K = 10: 3m 256x50, 3s5z_vs_3s6z 512x100
#   spans     MZ_STAMPS=1 build at 3m K=1 / K=5: per-phase cycles + launch body / boundary spans
#   trace     rocprofv3 --kernel-trace of the headline with MZ_TRACE_MARKS=1, cut to the timed
#             region by scripts/trace_window.py
#   search    bench_search.py (the full loop with a network)
#   matrix    BASELINE config #1: matrix 2-agent, 8 roots x 25 sims (CPU legs: reference ctree and the
#             pure-Python ptree)
#   dropin    the tree-level drop-in: the reference driver's host loop on mazero_amd.cytree
#   pytest    the GPU test suite
#   spansv    the spans-only build (scripts/build_variant.sh spans -DMZ_SPANS=1): launch body / boundary
#             at 3m K=1 / K=5 untraced, then 3m K=1 under rocprofv3 --kernel-trace (same build)
# Every GPU step has its own time limit; a fault / abort / timeout ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
R=$(pwd)
export TMPDIR=/tmp
O=gpurun_out/r3
mkdir -p $O
STEPS=${STEPS:-"headline strong k10 spans trace"}
step() {  # name timeout cmd...
    local name=$1 to=$2; shift 2
    timeout -k 10 "$to" "$@" > "$O/$name.json" 2> "$O/$name.err"
    local rc=$?
    echo "$name rc=$rc $(grep -o '"value": [0-9.]*' "$O/$name.json" | head -1)"
    if [ $rc -ne 0 ]; then tail -5 "$O/$name.err"; exit $rc; fi
}
for s in $STEPS; do
  case $s in
    headline) step headline 400 python bench.py ;;
    strong)   for b in 32 64 128 256; do step roots_$b 200 python bench.py --no-cpu --roots $b; done ;;
    k10)      step 3m_k10 200 python bench.py --no-cpu --sampled-times 10 &&
              step 3s5z_k10 300 python bench.py --no-cpu --map 3s5z_vs_3s6z --roots 512 --sims 100 --sampled-times 10 ;;
    spans)    export MZ_STAMPS=1
              step spans_3m_k1 200 python bench.py --no-cpu &&
              step spans_3m_k5 200 python bench.py --no-cpu --sampled-times 5
              unset MZ_STAMPS ;;
    trace)    export MZ_TRACE_MARKS=1
              step traced_3m_k1 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/trace_3m_k1" -o run -- \
                  python3 "$R/bench.py" --no-cpu
              unset MZ_TRACE_MARKS
              python scripts/trace_window.py $O/trace_3m_k1 --bench $O/traced_3m_k1.json --out $O/window_3m_k1.json > /dev/null || exit 3
              find $O/trace_3m_k1 -name "*kernel_trace.csv" -size +30M -delete ;;
    search)   step search 900 python bench_search.py ${SEARCH_ARGS} ;;
    matrix)   step matrix_k1 300 python bench.py --map matrix --roots 8 --sims 25 --sampled-times 1 --steps 50 --cpu-seconds 4 &&
              step matrix_k3 300 python bench.py --map matrix --roots 8 --sims 25 --sampled-times 3 --steps 50 --cpu-seconds 4 ;;
    memset)   # the runtime defect behind round 1's graph failure: default packet capture, then off
              timeout -k 10 200 python -u scripts/memset_graph_repro.py 600 6 > $O/memset_repro_default.log 2>&1
              echo "memset repro (default) rc=$?"; tail -3 $O/memset_repro_default.log
              DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 200 python -u scripts/memset_graph_repro.py 600 6 \
                  > $O/memset_repro_pc0.log 2>&1
              echo "memset repro (packet capture off) rc=$?"; tail -3 $O/memset_repro_pc0.log ;;
    dropin)   step dropin_3m_k1 300 python bench.py --dropin --steps 5 --warmup 1 --no-cpu &&
              step dropin_3m_k5 300 python bench.py --dropin --steps 5 --warmup 1 --no-cpu --sampled-times 5 ;;
    pytest)   timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
                  --timeout-method thread > $O/pytest_gpu.log 2>&1
              rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc ;;
    spansv)   export MZ_LIB_OVERRIDE=$R/mazero_amd/_build/variant_spans.so MZ_TRACE_MARKS=1
              step spansv_3m_k1 200 python bench.py --no-cpu &&
              step spansv_3m_k5 200 python bench.py --no-cpu --sampled-times 5 &&
              step spansv_traced_3m_k1 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/trace_spansv_3m_k1" \
                  -o run -- python3 "$R/bench.py" --no-cpu
              unset MZ_LIB_OVERRIDE MZ_TRACE_MARKS
              python scripts/trace_window.py $O/trace_spansv_3m_k1 --bench $O/spansv_traced_3m_k1.json \
                  --out $O/window_spansv_3m_k1.json > /dev/null || exit 3 ;;
  esac
done
