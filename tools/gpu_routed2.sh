# routed-path parity (route/shard tests), then routed bench + kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread -k "route or shard or dist or rehears" tests > gpurun_out/t_route.log 2>&1 && \
timeout -k 10 200 python bench.py --routed --steps 10 --warmup 3 --cpu-sample 0 > gpurun_out/b_routed.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_routed -o kt -- python3 bench.py --routed --steps 10 --warmup 3 --cpu-sample 0 > gpurun_out/prof_routed.log 2>&1
echo rc=$?
