#!/bin/bash
# Round-6 box pass: STEPS="tests ab stamps bench" (default "tests"), each step under its own limit,
# stopping at the first failing step.  Logs under gpurun_out/r6/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/r6; mkdir -p $O
STEPS=${STEPS:-tests}
for st in $STEPS; do
  case $st in
    tests)
      timeout -k 10 1050 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread ${PYK:+-k "$PYK"} \
        > $O/tests.log 2>&1; rc=$?; tail -15 $O/tests.log; [ $rc -ne 0 ] && exit $rc ;;
    ab)
      # interleaved A/B of the fused kernel (HIP-event mean per launch) against experiment builds
      for rep in 1 2; do
        for cfg in ${AB:-3m_k5 3m_k10 3s5z_k5 3s5z_k10 27m_k5}; do
          case $cfg in
            3m_k5) a="--sampled-times 5";; 3m_k10) a="--sampled-times 10";;
            3s5z_k5) a="--map 3s5z_vs_3s6z --roots 512 --sims 100 --sampled-times 5";;
            3s5z_k10) a="--map 3s5z_vs_3s6z --roots 512 --sims 100 --sampled-times 10";;
            27m_k5) a="--map 27m_vs_30m --roots 256 --sims 200 --sampled-times 5";;
            3m_k1) a="--sampled-times 1";; 2s3z_k1) a="--map 2s3z --roots 1024 --sims 50";;
            27m_k1) a="--map 27m_vs_30m --roots 256 --sims 200 --sampled-times 1";;
            27m_k16) a="--map 27m_vs_30m --roots 256 --sims 200 --sampled-times 16";;
          esac
          line="$cfg rep$rep"
          for v in prod ${ALTS:-r4 split}; do
            if [ $v = prod ]; then env=""; elif [ $v = no1024s ]; then env="MZ_NO_TREE_1024S=1"; else env="MZ_LIB_OVERRIDE=$PWD/mazero_amd/_build/variant_$v.so"; fi
            env $env timeout -k 10 200 python bench.py --no-cpu --steps 5 --warmup 2 $a > $O/ab_${cfg}_${v}_$rep.json 2> $O/ab.err || { tail -5 $O/ab.err; exit 1; }
            line="$line $v $(grep -o '"avg_launch_us": [0-9.]*' $O/ab_${cfg}_${v}_$rep.json | cut -d' ' -f2)/$(grep -o '"ms_per_step": [0-9.]*' $O/ab_${cfg}_${v}_$rep.json | head -1 | cut -d' ' -f2)"
          done
          echo "$line" | tee -a $O/ab.txt
        done
      done ;;
    stamps)
      for cfg in ${STAMPCFG:-3m_k5}; do
        case $cfg in
          3m_k1) a="--sampled-times 1";; 3m_k5) a="--sampled-times 5";; 3s5z_k10) a="--map 3s5z_vs_3s6z --roots 512 --sims 100 --sampled-times 10";;
          27m_k5) a="--map 27m_vs_30m --roots 256 --sims 200 --sampled-times 5";;
          27m_k16) a="--map 27m_vs_30m --roots 256 --sims 200 --sampled-times 16";;
        esac
        MZ_STAMPS=1 timeout -k 10 200 python bench.py --no-cpu --steps 3 --warmup 1 $a > $O/stamps_$cfg.json 2> $O/stamps.err || exit 1
      done ;;
    spans)
      # launch spans (MZ_SPANS build, scripts/build_variant.sh spans -DMZ_SPANS=1): per wave role
      for cfg in ${STAMPCFG:-3m_k1}; do
        case $cfg in
          3m_k1) a="--sampled-times 1";; 3m_k5) a="--sampled-times 5";; 2s3z_k1) a="--map 2s3z --roots 1024 --sims 50";;
          27m_k5) a="--map 27m_vs_30m --roots 256 --sims 200 --sampled-times 5";;
          3m_k10) a="--sampled-times 10";; 3s5z_k5) a="--map 3s5z_vs_3s6z --roots 512 --sims 100 --sampled-times 5";;
          3s5z_k10) a="--map 3s5z_vs_3s6z --roots 512 --sims 100 --sampled-times 10";;
          27m_k1) a="--map 27m_vs_30m --roots 256 --sims 200 --sampled-times 1";;
        esac
        for sv in ${SPANV:-spans}; do
          MZ_LIB_OVERRIDE=$PWD/mazero_amd/_build/variant_$sv.so timeout -k 10 200 python bench.py --no-cpu --steps 3 --warmup 1 $a \
            > $O/${sv}_$cfg.json 2> $O/spans.err || { tail -5 $O/spans.err; exit 1; }
        done
      done ;;
    segv)
      # the round-3/4 profiler abort: the 27m K = 1 --pmc pass over the env step's graph (5,481 kernel
      # nodes), with the fault's address, PC, thread and the process's mappings dumped by
      # scripts/segv_maps.c; the same pass eagerly first (its mappings at exit).  Last step of a call.
      a="--no-cpu --steps 1 --warmup 1 --map 27m_vs_30m --roots 256 --sims 200 --sampled-times 1"
      MZ_SEGV_MAPS=$PWD/$O/segv_eager.txt timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv \
        -d $PWD/$O/pmc_eager -o run -- python3 $PWD/bench.py $a --no-graph > $O/segv_eager.log 2>&1
      echo "eager pmc pass rc=$?"
      MZ_SEGV_MAPS=$PWD/$O/segv_graph.txt timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv \
        -d $PWD/$O/pmc_graph -o run -- python3 $PWD/bench.py $a > $O/segv_graph.log 2>&1
      echo "graph pmc pass rc=$?"
      head -5 $O/segv_graph.txt 2>/dev/null
      exit 0 ;;
    w0stamps)
      # wave 0's eight k_tree phases (variant builds with -DMZ_STAMPS=1 -DMZ_STAMPS_W0): cfg:variant pairs
      for pair in ${W0PAIRS:-3m_k5:w0prod 3m_k5:w0lev256}; do
        cfg=${pair%%:*}; v=${pair##*:}
        case $cfg in
          3m_k5) a="--sampled-times 5";; 3m_k10) a="--sampled-times 10";;
          3s5z_k5) a="--map 3s5z_vs_3s6z --roots 512 --sims 100 --sampled-times 5";;
          27m_k5) a="--map 27m_vs_30m --roots 256 --sims 200 --sampled-times 5";;
        esac
        MZ_STAMPS=1 MZ_LIB_OVERRIDE=$PWD/mazero_amd/_build/variant_$v.so timeout -k 10 200 python bench.py --no-cpu --steps 3 \
          --warmup 1 $a > $O/w0_${cfg}_$v.json 2> $O/w0.err || { tail -5 $O/w0.err; exit 1; }
        python -c "import json,sys; r=json.load(open('$O/w0_${cfg}_$v.json'))['roofline']; print('$cfg $v', r['avg_launch_us'], r.get('phase_cycles'))"
      done ;;
    mut)
      # the beyond-window test against a build whose wave 1 chases without the stream offset (the
      # round-5 bug, mazero_amd/_build/variant_mut_w1_oR.so): expected to FAIL; never ends the pass
      MZ_LIB_OVERRIDE=$PWD/mazero_amd/_build/variant_mut_w1_oR.so timeout -k 10 300 python -u -m pytest \
        tests/test_rng_window.py -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "B64_S190" \
        > $O/mut.log 2>&1; echo "mutation run rc=$? (1 = the test caught it)"; grep -E "Error|assert|passed|failed" $O/mut.log | head -8 ;;
    strong)
      # the strong-scaling proxy on this build: one rank's env step over 256/G roots
      for r in 256 128 64 32; do
        timeout -k 10 200 python bench.py --no-cpu --roots $r > $O/strong_$r.json 2> $O/strong.err || { tail -5 $O/strong.err; exit 1; }
        echo "roots $r: $(grep -o '"ms_per_step": [0-9.]*' $O/strong_$r.json | head -1) $(grep -o '"avg_launch_us": [0-9.]*' $O/strong_$r.json)"
      done ;;
    bcast)
      # config #5's weight broadcast in the timed loop (one rank: RCCL single-rank group)
      timeout -k 10 300 python bench.py --no-cpu --broadcast-every ${BEVERY:-1} ${BARGS:-} > $O/bcast.json 2> $O/bcast.err \
        || { tail -5 $O/bcast.err; exit 1; }; cat $O/bcast.json ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; tail -2 $O/smoke.log
      [ $rc -ne 0 ] && exit $rc ;;
    bench)
      timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err; rc=$?; cat $O/bench.json; [ $rc -ne 0 ] && exit $rc ;;
  esac
done
