# full GPU test suite, then fused-kernel timings over a few configurations
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
out=gpurun_out/iter.jsonl; : > $out
for args in "--sampled-times 1" "--sampled-times 5" "--map 27m_vs_30m --roots 256 --sims 200 --sampled-times 1" "--map 27m_vs_30m --roots 256 --sims 200 --sampled-times 5" "--map 3s5z_vs_3s6z --roots 512 --sims 100 --sampled-times 5"; do
  timeout -k 10 200 python bench.py --no-cpu $args >> $out 2> gpurun_out/iter.err || exit $?
done
python - $out <<'PY'
import json, sys
for line in open(sys.argv[1]):
    d = json.loads(line); r = d["roofline"]; c = d["config"]; pc = r.get("phase_cycles")
    print(c["map"], "K=%d" % c["sampled_times"], f"{d['value']/1e6:.2f}M sims/s", "launch", r["avg_launch_us"], "us",
          (" ".join(f"{k}={v:.0f}" for k, v in pc.items()) if pc else ""))
PY
for args in "--sampled-times 1" "--map 27m_vs_30m --roots 256 --sims 200 --sampled-times 1"; do
  MZ_STAMPS=1 timeout -k 10 200 python bench.py --no-cpu $args > gpurun_out/st.json 2>> gpurun_out/iter.err || exit $?
  python -c "
import json; d=json.loads(open('gpurun_out/st.json').read().strip().splitlines()[-1]); pc=d['roofline']['phase_cycles']
print('stamps', d['config']['map'], d['roofline']['avg_launch_us'], ' '.join(f'{k}={v:.0f}' for k,v in pc.items()))"
done
