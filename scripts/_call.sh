cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_workers.py tests/test_driver.py tests/test_consume.py tests/test_weights.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_w.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_w.log
