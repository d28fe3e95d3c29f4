mkdir -p gpurun_out
MZ_STAMPS=1 MZ_LIB_OVERRIDE=mazero_amd/_build/variant_probe3.so timeout -k 10 200 python bench.py --no-cpu --sampled-times 5 > gpurun_out/probe.jsonl 2> gpurun_out/probe.err || exit $?
python -c "
import json; d=json.loads(open('gpurun_out/probe.jsonl').read().strip().splitlines()[-1]); pc=d['roofline']['phase_cycles']
print('probe K=5', d['roofline']['avg_launch_us'], ' '.join(f'{k}={v:.0f}' for k,v in pc.items()))"
