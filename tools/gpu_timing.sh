set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread -k "timing or engine_selected or known or heavy" tests > gpurun_out/t_tm.log 2>&1 && \
timeout -k 10 300 python bench.py --cpu-sample 0 > gpurun_out/b_tm.log 2>&1 && \
timeout -k 10 300 python bench.py --workload c3 --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/b_tm3.log 2>&1
echo rc=$?
