#!/bin/bash
# Round-5 GPU test subsets: ./scripts/r5_tests.sh '<pytest -k expression>' [files...]
# Each pytest step under its own time limit; stops at the first failing step.
set -o pipefail
K="$1"; shift
FILES="${@:-tests/test_gpu_parity.py}"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest $FILES -v --timeout 300 --timeout-method thread -k "$K" > gpurun_out/r5_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r5_tests.log
exit $rc
