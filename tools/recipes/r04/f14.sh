# r04 final check of the committed tree: smoke, ranked / capacity parity, C2
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4f14; mkdir -p $O
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_capacity.py -m gpu -k "ranked or large_lists or clustered_long or c3 or dropin" > $O/tests.txt 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --cpu-sample 0 --no-capacity --no-host-input --steps 20 --warmup 5 > $O/c2.json 2> $O/c2.err || exit 1
echo rc=$?
