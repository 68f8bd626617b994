set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python bench.py --workload c4 --steps 1 --warmup 1 --cpu-sample 0 --no-scan-once > gpurun_out/b_c4n.log 2>&1
echo rc=$?
