# pipelined routed path: rehearsal test (stepwise + pipelined), routed bench with and without pipelining
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread -k "rehears or route or shard or learned" tests > gpurun_out/t_pipe.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --routed --steps 10 --warmup 3 --cpu-sample 0 --no-pipeline > gpurun_out/b_r0.log 2>&1 && \
timeout -k 10 200 python bench.py --routed --steps 10 --warmup 3 --cpu-sample 0 > gpurun_out/b_r1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pipe_kt -o kt -- python3 bench.py --routed --steps 4 --warmup 2 --cpu-sample 0 > gpurun_out/pipe_kt.log 2>&1
echo rc=$?
