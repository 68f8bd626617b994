# r06 g3: bench.py at N = 2 as a gloo rehearsal (two ranks on one GPU): the
# C2 leg and the new C4 / C5 as-specified legs at 1/400 of their reads; then a
# short default N = 1 line (no CPU leg) to check nothing else moved
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6g3; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -m gpu --timeout 500 --timeout-method thread tests/test_gpu_dist.py \
    -k "capacity_rehearsal" > $O/rehearsal.txt 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --steps 10 --warmup 2 --cpu-sample 0 --no-host-input > $O/c2_bench.json 2> $O/c2_bench.err || exit 1
echo done
