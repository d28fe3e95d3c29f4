# full GPU test suite, then the fused-kernel timings and stamps at 3m K=1 / K=5 (scripts/iter.sh)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
bash scripts/iter.sh
MZ_STAMPS=1 MZ_LIB_OVERRIDE=mazero_amd/_build/variant_probe3.so timeout -k 10 200 python bench.py --no-cpu --sampled-times 5 > gpurun_out/probe.jsonl 2> gpurun_out/probe.err || exit $?
python -c "
import json; d=json.loads(open('gpurun_out/probe.jsonl').read().strip().splitlines()[-1]); pc=d['roofline']['phase_cycles']
print('probe K=5', d['roofline']['avg_launch_us'], ' '.join(f'{k}={v:.0f}' for k,v in pc.items()))"
