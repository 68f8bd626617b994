set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread -k "split_passes or partition or route" tests > gpurun_out/t_so.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --workload c3 --steps 2 --warmup 1 --digest --cpu-sample 0 > gpurun_out/b_so3.log 2>&1 && \
timeout -k 10 400 python bench.py --workload c3 --parts 6 --steps 1 --warmup 1 --digest --cpu-sample 0 > gpurun_out/b_so36.log 2>&1 && \
timeout -k 10 500 python bench.py --workload c5 --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/b_so5.log 2>&1
echo rc=$?
