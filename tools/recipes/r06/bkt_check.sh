# r06: bucket_kernel at 1024 threads -- parity and capacity suites,
# C3 with its digest, the default C2 line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/bkt_check; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_capacity.py tests/test_gpu_scale.py > $O/tests.txt 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --cpu-sample 0 --workload c3 --steps 3 --warmup 1 --digest > $O/c3.json 2> $O/c3.err || exit 1
timeout -k 10 300 python -u bench.py --cpu-sample 0 --no-capacity --no-host-input --steps 20 --warmup 3 > $O/c2.json 2> $O/c2.err || exit 1
echo done
