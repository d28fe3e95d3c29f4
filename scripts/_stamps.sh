# per-phase cycle stamps (diagnostic build) for a few configurations
mkdir -p gpurun_out
out=gpurun_out/stamps.jsonl; : > $out
for args in "--sampled-times 1" "--sampled-times 5" "--map 27m_vs_30m --roots 256 --sims 200 --sampled-times 1" "--map 3s5z_vs_3s6z --roots 512 --sims 100 --sampled-times 5"; do
  MZ_STAMPS=1 timeout -k 10 200 python bench.py --no-cpu $args >> $out 2> gpurun_out/stamps.err || exit $?
done
python - $out <<'PY'
import json, sys
for line in open(sys.argv[1]):
    d = json.loads(line); r = d["roofline"]; c = d["config"]; pc = r.get("phase_cycles") or {}
    print(c["map"], c["sampled_times"], f"{d['value']/1e6:.2f}M", r["avg_launch_us"], "path", r["mean_path_len"])
    print("   ", " ".join(f"{k}={v:.0f}" for k, v in pc.items()))
PY
