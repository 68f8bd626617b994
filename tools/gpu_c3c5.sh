# C3 (digest must match DESIGN.md section 9) and C5 per-GPU share
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python bench.py --workload c3 --steps 2 --warmup 1 --digest --cpu-sample 0 > gpurun_out/b_c3.log 2>&1 && \
timeout -k 10 500 python bench.py --workload c5 --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/b_c5.log 2>&1
echo rc=$?
