# routed (multi-GPU path over a 1-rank RCCL group) vs direct, and its kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 python bench.py --steps 10 --warmup 3 --cpu-sample 0 > gpurun_out/b_direct.log 2>&1 && \
timeout -k 10 200 python bench.py --routed --steps 10 --warmup 3 --cpu-sample 0 > gpurun_out/b_routed.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_routed -o kt -- python3 bench.py --routed --steps 10 --warmup 3 --cpu-sample 0 > gpurun_out/prof_routed.log 2>&1
echo rc=$?
