#!/bin/bash
# Round-5 box pass: the whole GPU test suite, smoke, the headline bench (as the driver runs them).
# Each step under its own limit; a failing step ends the pass.  Logs under gpurun_out/r5/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/r5; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -2 $O/smoke.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err; rc=$?; echo "bench rc=$rc"; cat $O/bench_default.json
exit $rc
