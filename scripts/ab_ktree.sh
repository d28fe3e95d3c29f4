#!/bin/bash
# A/B of the product library against an experiment build (default: mazero_amd/_build/variant_old.so),
# interleaved twice: fused-launch mean (HIP events) per run.  The configurations are
# "name:bench args;..." from the first argument, else AB_CONFIGS, else the K > 1 ones.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/ab${ALT_TAG:+_$ALT_TAG}; mkdir -p $O
ALT=${ALT:-$PWD/mazero_amd/_build/variant_old.so}
DEF="3m_k5:--sampled-times 5;3s5z_k5:--map 3s5z_vs_3s6z --roots 512 --sims 100 --sampled-times 5;3m_k10:--sampled-times 10"
CONFIGS=${1:-${AB_CONFIGS:-$DEF}}
IFS=';' read -ra CFGS <<< "$CONFIGS"
for rep in 1 2; do
  for cfg in "${CFGS[@]}"; do
    n=${cfg%%:*}; a=${cfg#*:}
    timeout -k 10 200 python bench.py --no-cpu $a > $O/new_${n}_$rep.json 2>/dev/null || exit 1
    MZ_LIB_OVERRIDE=$ALT timeout -k 10 200 python bench.py --no-cpu $a > $O/alt_${n}_$rep.json 2>/dev/null || exit 1
    echo "$n rep$rep new $(grep -o '"avg_launch_us": [0-9.]*' $O/new_${n}_$rep.json | cut -d' ' -f2) alt $(grep -o '"avg_launch_us": [0-9.]*' $O/alt_${n}_$rep.json | cut -d' ' -f2)"
  done
done
