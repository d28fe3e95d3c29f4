#!/bin/bash
# k_tree iteration pass: GPU parity suite, then the K > 1 bench configurations with k_tree and
# with k_step (MZ_NO_TREE=1), plus the stamped build.  Every GPU step has its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/tree_pytest.log 2>&1
rc=$?; tail -4 gpurun_out/tree_pytest.log; [ $rc -ne 0 ] && exit $rc
out=gpurun_out/tree_ab.jsonl; : > $out
for args in ${CONFIGS:-"--sampled-times 5" "--map 3s5z_vs_3s6z --roots 512 --sims 100 --sampled-times 5" "--map 27m_vs_30m --roots 256 --sims 200 --sampled-times 5"}; do
  for v in 0 1; do
    MZ_NO_TREE=$v timeout -k 10 200 python bench.py --no-cpu $args >> $out 2>> gpurun_out/tree_ab.err || exit $?
  done
  MZ_STAMPS=1 timeout -k 10 200 python bench.py --no-cpu $args >> $out 2>> gpurun_out/tree_ab.err || exit $?
done
python - $out <<'PY'
import json, sys
for line in open(sys.argv[1]):
    d = json.loads(line); r = d["roofline"]; c = d["config"]; pc = r.get("phase_cycles")
    print(c["map"], "K=%d" % c["sampled_times"], f"{d['value']/1e6:.2f}M", r["avg_launch_us"], "us",
          " ".join(f"{k}={v:.0f}" for k, v in pc.items() if v) if pc else "")
PY
