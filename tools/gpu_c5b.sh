set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python bench.py --workload c5 --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/b_so5.log 2>&1 && \
timeout -k 10 600 python bench.py --workload c4 --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/b_so4.log 2>&1
echo rc=$?
