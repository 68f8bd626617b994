# r05 g1: the partition-restart race: the skew stress on
# the fixed diagnostic build and on round 4's single-word build (must fail),
# then the parity suite and one default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5g1; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/test_gpu_race.py > $O/race.txt 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_parity.py > $O/parity.txt 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > $O/c2_bench.json 2> $O/c2_bench.err || exit 1
echo done
