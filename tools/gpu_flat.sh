# heavy-bin flat lists: parity first, then C2 and C3 benches
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -m pytest tests -x -q -m gpu -k "heavy or partition or capacity or large or list or clustered" > gpurun_out/t_flat.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/b_c2.log 2>&1 && \
timeout -k 10 400 python bench.py --workload c3 --steps 2 --warmup 1 --digest --cpu-sample 0 > gpurun_out/b_c3_p4.log 2>&1 && \
KB_BIN_FLAT_L=3 timeout -k 10 400 python bench.py --workload c3 --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/b_c3_f3.log 2>&1
echo rc=$?
