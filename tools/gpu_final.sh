# smoke, default bench, routed bench
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && \
timeout -k 10 200 python bench.py --routed --steps 10 --warmup 3 --cpu-sample 0 > gpurun_out/b_routed.log 2>&1
echo rc=$?
