set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread -k "list or heavy or digest or clustered" tests > gpurun_out/t_lb.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --workload c3 --steps 2 --warmup 1 --digest --cpu-sample 0 > gpurun_out/b_lb3.log 2>&1 && \
timeout -k 10 300 python bench.py --cpu-sample 0 > gpurun_out/b_lb2.log 2>&1
echo rc=$?
