# r04 final evidence 8 (the round's last build): GPU suite, smoke, default
# bench line, C3 leg with digest, C2 and C3 kernel traces + stats
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4f10; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input"
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 600 --timeout-method thread tests > $O/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > $O/c2_bench.json 2> $O/c2_bench.err || exit 1
timeout -k 10 400 python -u bench.py --cpu-sample 0 --workload c3 --steps 2 --warmup 2 --digest > $O/c3.json 2> $O/c3.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 bench.py $NOX --steps 20 --warmup 3 > $O/kt.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_c3 -o kt -- python3 bench.py $NOX --workload c3 --steps 2 --warmup 2 > $O/kt_c3.log 2>&1 || exit 1
echo rc=$?
