# Round profile set for profiles/: kernel trace stats, HBM traffic (FETCH_SIZE and
# WRITE_SIZE in separate --pmc passes, no tracing alongside), the default bench,
# and the routed path (1-rank RCCL group) bench + kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > gpurun_out/t_all.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kt -o kt -- python3 bench.py --steps 10 --warmup 3 --cpu-sample 0 > gpurun_out/prof_kt.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_f -o pmc -- python3 bench.py --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/pmc_f.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_w -o pmc -- python3 bench.py --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/pmc_w.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_routed -o kt -- python3 bench.py --routed --steps 10 --warmup 3 --cpu-sample 0 > gpurun_out/prof_routed.log 2>&1 && \
timeout -k 10 200 python3 bench.py --routed --steps 10 --warmup 3 --cpu-sample 0 > gpurun_out/b_routed.log 2>&1 && \
timeout -k 10 600 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
echo rc=$?
