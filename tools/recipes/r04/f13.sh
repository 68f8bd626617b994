# r04 final evidence 11: the final tree with long lists = over 64 ids -- GPU suite, smoke, default
# bench line, C3 leg with digest
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4f13; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 600 --timeout-method thread tests > $O/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > $O/c2_bench.json 2> $O/c2_bench.err || exit 1
timeout -k 10 400 python -u bench.py --cpu-sample 0 --workload c3 --steps 2 --warmup 1 --digest > $O/c3.json 2> $O/c3.err || exit 1
echo rc=$?
