# two-phase heavy bins: binned parity, C2 bench, then the heavy C5 shares
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "binned" > gpurun_out/t_par.log 2>&1 && \
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --cpu-sample 0 > gpurun_out/b_c2.log 2>&1 && \
timeout -k 10 300 python -u bench.py --workload c5 --reads 32000000 --parts 2 --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/c5_32m_p2.log 2>&1 && \
timeout -k 10 170 python -u bench.py --workload c5 --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/b_c5.log 2>&1
echo rc=$?
