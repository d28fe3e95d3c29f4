# A/B timing of two library builds in one call (same box): VARIANT_A / VARIANT_B paths
mkdir -p gpurun_out
out=gpurun_out/ab.jsonl; : > $out
for rep in 1 2; do
for lib in $VARIANT_A $VARIANT_B; do
for args in "--sampled-times 1" "--sampled-times 5" "--map 27m_vs_30m --roots 256 --sims 200 --sampled-times 5" "--map 3s5z_vs_3s6z --roots 512 --sims 100 --sampled-times 5"; do
  MZ_LIB_OVERRIDE=$lib timeout -k 10 200 python bench.py --no-cpu $args > gpurun_out/ab1.json 2>> gpurun_out/ab.err || exit $?
  python -c "
import json; d=json.loads(open('gpurun_out/ab1.json').read().strip().splitlines()[-1]); c=d['config']
print('$lib'.split('/')[-1], c['map'], 'K=%d' % c['sampled_times'], d['roofline']['avg_launch_us'], round(d['value']/1e6, 2))"
done; done; done
