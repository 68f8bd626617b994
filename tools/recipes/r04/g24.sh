# r04 g24: LDS-staged receiver conversion (KB_CONVERT_STAGED, default on):
# dist + parity + capacity tests, C3 / C5 / routed C2 A/B (staged vs lane per
# record), digests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4g24; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input"
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_dist.py tests/test_gpu_parity.py tests/test_gpu_capacity.py -m gpu > $O/tests.txt 2>&1 && \
timeout -k 10 300 python -u bench.py $NOX --workload c3 --steps 2 --warmup 1 --digest > $O/c3.json 2> $O/c3.err && \
KB_CONVERT_STAGED=0 timeout -k 10 300 python -u bench.py $NOX --workload c3 --steps 2 --warmup 1 --digest > $O/c3_lane.json 2> $O/c3_lane.err && \
timeout -k 10 300 python -u bench.py $NOX --routed --steps 20 --warmup 3 > $O/routed.json 2> $O/routed.err && \
KB_CONVERT_STAGED=0 timeout -k 10 300 python -u bench.py $NOX --routed --steps 20 --warmup 3 > $O/routed_lane.json 2> $O/routed_lane.err && \
timeout -k 10 500 python -u bench.py $NOX --workload c5 --steps 2 --warmup 2 --digest > $O/c5.json 2> $O/c5.err
echo rc=$?
