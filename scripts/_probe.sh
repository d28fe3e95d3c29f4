mkdir -p gpurun_out
out=gpurun_out/probe.jsonl; : > $out
for args in "--sampled-times 5"; do
  MZ_STAMPS=1 MZ_LIB_OVERRIDE=mazero_amd/_build/variant_probe3.so timeout -k 10 200 python bench.py --no-cpu $args >> $out 2> gpurun_out/probe.err || exit $?
done
python - $out <<'PY'
import json, sys
for line in open(sys.argv[1]):
    d = json.loads(line); r = d["roofline"]; c = d["config"]; pc = r.get("phase_cycles") or {}
    print(c["map"], c["sampled_times"], f"{d['value']/1e6:.2f}M", r["avg_launch_us"], "path", r["mean_path_len"])
    print("   ", " ".join(f"{k}={v:.0f}" for k, v in pc.items()))
PY
