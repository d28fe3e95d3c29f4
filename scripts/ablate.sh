#!/bin/bash
# Timing ablations (diagnostics only): bench.py's fused-kernel time with experiment builds that
# drop one part of the work (scripts/build_variant.sh NAME -DMZ_ABL_...).  Results are not valid
# searches; only the launch time is read.  VARIANTS="name ..." K="1 5".
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
out=gpurun_out/ablate.txt
: > "$out"
for k in ${K:-1 5}; do
  for v in base ${VARIANTS}; do
    if [ "$v" = base ]; then ov=""; else ov="mazero_amd/_build/variant_$v.so"; fi
    MZ_LIB_OVERRIDE=$ov timeout -k 10 120 python bench.py --no-cpu --steps 10 --sampled-times $k > gpurun_out/abl_$v.json 2> gpurun_out/abl_$v.err
    rc=$?
    if [ $rc -gt 1 ]; then echo "K=$k $v rc=$rc" >> "$out"; tail -3 gpurun_out/abl_$v.err; exit $rc; fi
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('K=$k', '$v', d['roofline']['avg_launch_us'], 'us')" gpurun_out/abl_$v.json >> "$out" 2>/dev/null || echo "K=$k $v rc=$rc (no result)" >> "$out"
  done
done
cat "$out"
