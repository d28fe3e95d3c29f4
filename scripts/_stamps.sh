# per-phase cycle stamps (diagnostic build) for the BASELINE configurations -> gpurun_out/stamps_*.json
mkdir -p gpurun_out
run() { name=$1; shift; MZ_STAMPS=1 timeout -k 10 200 python bench.py --no-cpu "$@" > gpurun_out/stamps_$name.json 2> gpurun_out/stamps.err || exit $?; }
run 3m_k1 --sampled-times 1
run 3m_k5 --sampled-times 5
run 27m_k1 --map 27m_vs_30m --roots 256 --sims 200 --sampled-times 1
run 27m_k5 --map 27m_vs_30m --roots 256 --sims 200 --sampled-times 5
run 3s5z_k5 --map 3s5z_vs_3s6z --roots 512 --sims 100 --sampled-times 5
for f in gpurun_out/stamps_*.json; do
  python -c "
import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); pc=d['roofline']['phase_cycles']
print('$f', d['roofline']['avg_launch_us'], ' '.join(f'{k}={v:.0f}' for k,v in pc.items()))"
done
