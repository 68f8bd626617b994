set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread -k "heavy or split or partition" tests > gpurun_out/t_c5.log 2>&1 || exit 1
timeout -k 10 500 python bench.py --workload c5 --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/b_c5.log 2>&1
echo rc=$?
