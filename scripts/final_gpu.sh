#!/bin/bash
# Round-end confirmation on one box: the GPU suite, a widened fuzz (MZ_FUZZ_CHUNKS), smoke() and the
# default bench line, each step under its own limit, stopping at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/final; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
  || { tail -20 $O/tests.log; exit 1; }
tail -2 $O/tests.log
MZ_FUZZ_CHUNKS=${SMALL:-60} timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 300 \
  --timeout-method thread -k "fuzz_small" > $O/fuzz_small.log 2>&1 || { tail -20 $O/fuzz_small.log; exit 1; }
tail -1 $O/fuzz_small.log
MZ_FUZZ_CHUNKS=${LARGE:-8} timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 300 \
  --timeout-method thread -k "fuzz_large" > $O/fuzz_large.log 2>&1 || { tail -20 $O/fuzz_large.log; exit 1; }
tail -1 $O/fuzz_large.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cat $O/bench.json
