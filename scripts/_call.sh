cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_chain.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_chain.log; [ $rc -gt 1 ] && exit $rc
for v in 0 1; do MZ_NO_CHAIN=$v timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench_chain$v.json 2>&1 || exit $?; python -c "
import json; d=json.loads(open('gpurun_out/bench_chain$v.json').read().strip().splitlines()[-1]); print('NO_CHAIN=$v', round(d['value']/1e6,2), 'M', d['roofline']['avg_launch_us'], 'us')"; done
