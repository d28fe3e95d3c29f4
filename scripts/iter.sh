#!/bin/bash
# One kernel-iteration pass on the GPU box: tree-kernel parity tests, then the fused-kernel time at
# 3m K=1 / K=5 (normal build) and the per-phase cycle stamps (diagnostic build).  Every GPU step
# has its own time limit; a fault / abort / timeout ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
out=gpurun_out/iter.jsonl
: > "$out"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread > gpurun_out/iter_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/iter_pytest.log; [ $rc -ne 0 ] && exit $rc
for k in 1 5; do
    timeout -k 10 200 python bench.py --no-cpu --sampled-times $k >> "$out" 2> gpurun_out/iter_err.log || exit $?
    MZ_STAMPS=1 timeout -k 10 200 python bench.py --no-cpu --sampled-times $k >> "$out" 2>> gpurun_out/iter_err.log || exit $?
done
python - "$out" <<'EOF'
import json, sys
for line in open(sys.argv[1]):
    d = json.loads(line); r = d["roofline"]; pc = r.get("phase_cycles")
    print(f"K={d['config']['sampled_times']} {d['value']/1e6:.2f}M sims/s  launch {r['avg_launch_us']} us" +
          ("  " + " ".join(f"{k}={v:.0f}" for k, v in pc.items()) if pc else ""))
EOF
