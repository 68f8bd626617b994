# full GPU suite (stops at the first failure), then the default bench
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/t_all.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/b_full.log 2>&1
echo rc=$?
