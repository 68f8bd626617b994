# r05 g36: the receiver conversion in 1024-thread blocks (8192 records per
# block trip, ~4x the records per bucket range; KB_CONVERT_THREADS=1024):
# dist parity with it, C3 alternating 256 / 1024 on the same build
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5g36; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input"
KB_CONVERT_THREADS=1024 timeout -k 10 800 python -u -m pytest -x -q -m gpu --timeout 600 --timeout-method thread tests/test_gpu_dist.py tests/test_gpu_capacity.py > $O/tests.txt 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 300 python -u bench.py $NOX --workload c3 --steps 2 --warmup 1 --digest > $O/c3_t256_$i.json 2> $O/c3_t256_$i.err || exit 1
  KB_CONVERT_THREADS=1024 timeout -k 10 300 python -u bench.py $NOX --workload c3 --steps 2 --warmup 1 --digest > $O/c3_t1024_$i.json 2> $O/c3_t1024_$i.err || exit 1
done
echo done
