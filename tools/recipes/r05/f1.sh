# r05 final evidence 1: the whole GPU suite; smoke; the default bench line;
# C2 kernel trace + stats; C2 FETCH_SIZE / WRITE_SIZE passes (traffic.json)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5f1; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input"
timeout -k 10 1000 python -u -m pytest -x -v -m gpu --timeout 600 --timeout-method thread tests > $O/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > $O/c2_bench.json 2> $O/c2_bench.err || exit 1
echo rc=$?
