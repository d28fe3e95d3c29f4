#!/bin/bash
# One GPU-box pass after a change: the Python memset repro with packet capture off (control), the
# whole GPU test suite, smoke, the headline bench.  Each step has its own limit; faults end it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 200 python -u scripts/memset_graph_repro.py 300 6 > gpurun_out/repro_py_pc0.log 2>&1; echo "py repro pc0 rc=$?"; tail -2 gpurun_out/repro_py_pc0.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log; [ $rc -gt 1 ] && exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/bench.log
exit $rc
