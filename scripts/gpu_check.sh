#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench, diagnostics.  Each GPU step has its own time
# limit; a step that faults / aborts / times out ends the script (exit status > 1), a plain test
# failure (status 1) does not.  Select steps with STEPS="pytest smoke bench stamps prof pmc".
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-"pytest smoke bench stamps prof"}
step() {  # name timeout cmd...
    local name=$1 to=$2; shift 2
    echo "=== $name" | tee -a gpurun_out/steps.log
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc" | tee -a gpurun_out/steps.log
    tail -4 "gpurun_out/$name.log"
    if [ $rc -gt 1 ]; then exit $rc; fi
    return 0
}
for s in $STEPS; do
  case $s in
    pytest) step pytest_gpu 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread ${PYTEST_ARGS} ;;
    smoke)  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)  step bench 600 python bench.py ${BENCH_ARGS} ;;
    search) step bench_search 900 python bench_search.py ${SEARCH_ARGS} ;;
    stamps) MZ_STAMPS=1 step bench_stamps 600 python bench.py --no-cpu ${BENCH_ARGS} ;;
    prof)   step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o bench -- python3 "$R/bench.py" --no-cpu --steps 10 ${BENCH_ARGS} ;;
    pmc)    step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/pmc_fetch" -o bench -- python3 "$R/bench.py" --no-cpu --steps 5 ${BENCH_ARGS} &&
            step pmc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/pmc_write" -o bench -- python3 "$R/bench.py" --no-cpu --steps 5 ${BENCH_ARGS} &&
            step pmc_summary 120 python scripts/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write --bench-args "${BENCH_ARGS}" --out gpurun_out/pmc_latest.json ;;
  esac
done
