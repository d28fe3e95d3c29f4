#!/bin/bash
# Whole-step A/B of experiment builds: `bench.py --no-cpu` (ms per env step, HIP events over the
# graph replays) for each library in LIBS (paths; "prod" = the product build), interleaved REPS times.
#   LIBS="prod mazero_amd/_build/variant_x.so" bash scripts/ab_step.sh [bench args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/ab_step; mkdir -p $O
for rep in $(seq 1 ${REPS:-3}); do
  for lib in ${LIBS:-prod}; do
    tag=$(basename "$lib" .so)
    if [ "$lib" = prod ]; then
      timeout -k 10 200 python bench.py --no-cpu "$@" > $O/${tag}_$rep.json 2>/dev/null || exit 1
    else
      MZ_LIB_OVERRIDE=$PWD/$lib timeout -k 10 200 python bench.py --no-cpu "$@" > $O/${tag}_$rep.json 2>/dev/null || exit 1
    fi
    echo "rep$rep $tag ms_per_step $(grep -o '"ms_per_step": [0-9.]*' $O/${tag}_$rep.json | cut -d' ' -f2) launch_us $(grep -o '"avg_launch_us": [0-9.]*' $O/${tag}_$rep.json | cut -d' ' -f2)"
  done
done
