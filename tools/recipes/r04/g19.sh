# r04 g19: chunked two-sweep receiver conversion (one reservation per bucket
# and chunk): dist + superkmer parity, C3 / C5 / routed C2 benches
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4g19; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dist.py tests/test_gpu_parity.py -m gpu > $O/tests.txt 2>&1 && \
timeout -k 10 300 python -u bench.py $NOX --workload c3 --steps 2 --warmup 1 --digest > $O/c3.json 2> $O/c3.err && \
timeout -k 10 300 python -u bench.py $NOX --routed --steps 20 --warmup 3 > $O/routed.json 2> $O/routed.err && \
timeout -k 10 500 python -u bench.py $NOX --workload c5 --steps 2 --warmup 2 --digest > $O/c5.json 2> $O/c5.err
echo rc=$?
