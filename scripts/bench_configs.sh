#!/bin/bash
# bench.py over the BASELINE.json configurations that fit one GPU (one JSON line each).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
out=gpurun_out/bench_configs.jsonl
: > "$out"
run() {
    timeout -k 10 300 python bench.py "$@" >> "$out" 2> gpurun_out/bench_configs.err || exit $?
}
run --map 3m --roots 256 --sims 50 --sampled-times 1
run --map 3m --roots 256 --sims 50 --sampled-times 5
run --map 2s3z --roots 1024 --sims 50 --sampled-times 1
run --map 3s5z_vs_3s6z --roots 512 --sims 100 --sampled-times 5
run --map 27m_vs_30m --roots 256 --sims 200 --sampled-times 1
run --map 27m_vs_30m --roots 256 --sims 200 --sampled-times 5
