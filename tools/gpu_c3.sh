# partitioned passes: parity at small size, then C3 (100M x 150 bp) at two
# partition counts whose kb_digest sums must agree
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -m pytest tests -x -q -m gpu -k "partition or digest" > gpurun_out/t_c3.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/b_c2.log 2>&1 && \
timeout -k 10 400 python bench.py --workload c3 --steps 3 --warmup 1 --digest > gpurun_out/b_c3_p4.log 2>&1 && \
timeout -k 10 400 python bench.py --workload c3 --parts 6 --steps 2 --warmup 1 --digest --cpu-sample 0 > gpurun_out/b_c3_p6.log 2>&1
echo rc=$?
