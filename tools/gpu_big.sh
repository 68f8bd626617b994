# full GPU suite, then one step of each large per-GPU workload (C3, C4, C5 shares)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/t_all.log 2>&1 && \
timeout -k 10 300 python -u bench.py --workload c3 --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/b_c3.log 2>&1 && \
timeout -k 10 300 python -u bench.py --workload c5 --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/b_c5.log 2>&1 && \
timeout -k 10 300 python -u bench.py --workload c4 --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/b_c4.log 2>&1
echo rc=$?
