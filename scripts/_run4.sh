cd $GRAFT_REPO_ROOT
STEPS="pytest stamps" bash scripts/gpu_check.sh
MZ_STAMPS=1 timeout -k 10 300 python bench.py --no-cpu --sampled-times 5 > gpurun_out/stamps_k5.log 2>&1; tail -1 gpurun_out/stamps_k5.log
