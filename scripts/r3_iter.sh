#!/bin/bash
# Chain-kernel iteration pass (one GPU box): GPU tests, then the headline-style bench of the new
# k_chain3 against k_chain (MZ_CHAIN_V2=1) at the K = 1 BASELINE configurations, the stamped build
# and the spans build.  STEPS selects: pytest ab ktree stamps spans.  A fault / abort / timeout ends it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
R=$(pwd)
export TMPDIR=/tmp
O=gpurun_out/it
mkdir -p $O
STEPS=${STEPS:-"pytest ab ktree stamps spans"}
summ() { python - "$@" <<'PY'
import json, sys
for f in sys.argv[1:]:
    try:
        d = json.loads([x for x in open(f) if x.startswith("{")][-1])
    except Exception as e:
        print(f, "no line", e); continue
    r = d["roofline"]; c = d["config"]
    print(f"{f.split('/')[-1]:28s} {c['map']:14s} K={c['sampled_times']} {d['value']/1e6:8.2f}M  {d['ms_per_step']:8.4f} ms  launch {r['avg_launch_us']} us",
          ("span " + json.dumps(r["launch_span"])) if r.get("launch_span") else "",
          ("\n   " + " ".join(f"{k}={v:.0f}" for k, v in r["phase_cycles"].items() if v)) if r.get("phase_cycles") else "")
PY
}
run() {  # name timeout args...
    local name=$1 to=$2; shift 2
    timeout -k 10 "$to" python bench.py --no-cpu "$@" > $O/$name.json 2> $O/$name.err
    local rc=$?; [ $rc -ne 0 ] && { echo "$name rc=$rc"; tail -5 $O/$name.err; exit $rc; }
    return 0
}
for s in $STEPS; do
  case $s in
    pytest) timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 \
                --timeout-method thread ${PYTEST_ARGS} > $O/pytest_gpu.log 2>&1
            rc=$?; echo "pytest rc=$rc"; tail -15 $O/pytest_gpu.log | grep -v "^$"; [ $rc -ne 0 ] && [ $rc -ne 5 ] && exit $rc; true ;;
    ab)     for cfg in "3m:--map 3m" "2s3z:--map 2s3z --roots 1024" "27m:--map 27m_vs_30m --sims 200"; do
                n=${cfg%%:*}; a=${cfg#*:}
                run ab_${n}_v3 300 $a
                MZ_CHAIN_V2=1 run ab_${n}_v2 300 $a
            done
            summ $O/ab_*.json ;;
    ktree)  for cfg in "3m_k5:--map 3m --sampled-times 5" "3s5z_k5:--map 3s5z_vs_3s6z --roots 512 --sims 100 --sampled-times 5" \
                       "27m_k5:--map 27m_vs_30m --sims 200 --sampled-times 5"; do
                n=${cfg%%:*}; a=${cfg#*:}
                run kt_${n} 300 $a
            done
            summ $O/kt_*.json ;;
    stamps) MZ_STAMPS=1 run stamps_3m 200; summ $O/stamps_3m.json ;;
    kspans) MZ_LIB_OVERRIDE=$R/mazero_amd/_build/variant_spans.so run kspans_3m_k5 200 --sampled-times 5
            MZ_LIB_OVERRIDE=$R/mazero_amd/_build/variant_spans.so run kspans_3s5z_k5 300 --map 3s5z_vs_3s6z --roots 512 --sims 100 --sampled-times 5
            MZ_STAMPS=1 run kstamps_3m_k5 200 --sampled-times 5
            summ $O/kspans_*.json $O/kstamps_3m_k5.json ;;
    spans)  MZ_LIB_OVERRIDE=$R/mazero_amd/_build/variant_spans.so run spans_3m 200
            MZ_LIB_OVERRIDE=$R/mazero_amd/_build/variant_spans.so MZ_CHAIN_V2=1 run spans_3m_v2 200
            summ $O/spans_3m.json $O/spans_3m_v2.json ;;
  esac
done
