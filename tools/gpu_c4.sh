set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python bench.py --workload c3 --steps 2 --warmup 1 --digest --cpu-sample 0 > gpurun_out/b_so3.log 2>&1 && \
timeout -k 10 600 python bench.py --workload c4 --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/b_so4.log 2>&1
echo rc=$?
