#!/bin/bash
# Kernel iteration pass: GPU parity suite, then bench configurations with the product build and with
# the previous kernels (MZ_NO_TREE=1), plus the stamped build.  Every GPU step has its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/tree_pytest.log 2>&1
  rc=$?; tail -4 gpurun_out/tree_pytest.log; [ $rc -ne 0 ] && exit $rc
fi
out=gpurun_out/tree_ab.jsonl; : > $out
CONFIGS=${CONFIGS:-"k1 k5 3s5z 27m5"}
for c in $CONFIGS; do
  case $c in
    k1) args="--sampled-times 1";;
    k5) args="--sampled-times 5";;
    3s5z) args="--map 3s5z_vs_3s6z --roots 512 --sims 100 --sampled-times 5";;
    27m5) args="--map 27m_vs_30m --roots 256 --sims 200 --sampled-times 5";;
    27m1) args="--map 27m_vs_30m --roots 256 --sims 200 --sampled-times 1";;
    2s3z) args="--map 2s3z --roots 1024 --sims 50 --sampled-times 1";;
  esac
  timeout -k 10 200 python bench.py --no-cpu $args >> $out 2>> gpurun_out/tree_ab.err || exit $?
  [ -n "$AB" ] && { MZ_NO_TREE=1 timeout -k 10 200 python bench.py --no-cpu $args >> $out 2>> gpurun_out/tree_ab.err || exit $?; }
  [ -n "$STAMPS" ] && { MZ_STAMPS=1 timeout -k 10 200 python bench.py --no-cpu $args >> $out 2>> gpurun_out/tree_ab.err || exit $?; }
  for v in $VARIANTS; do  # experiment builds: mazero_amd/_build/<name>.so
    MZ_LIB_OVERRIDE=mazero_amd/_build/$v.so timeout -k 10 200 python bench.py --no-cpu $args >> $out 2>> gpurun_out/tree_ab.err || exit $?
  done
done
python - $out <<'PY'
import json, sys
for line in open(sys.argv[1]):
    d = json.loads(line); r = d["roofline"]; c = d["config"]; pc = r.get("phase_cycles")
    print(c["map"], "K=%d" % c["sampled_times"], f"{d['value']/1e6:.2f}M", f"{d['ms_per_step']:.4f}ms", r["avg_launch_us"], "us",
          " ".join(f"{k}={v:.0f}" for k, v in pc.items() if v) if pc else "")
PY
