# r06: parity + distributed suites on the batched row loads; then A/B of the
# K <= 63 bucket_kernel at 4 records in flight (bk4u4) against 2, C5 share
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/rows_bk4; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_dist.py > $O/tests.txt 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 400 python -u bench.py --cpu-sample 0 --workload c5 --steps 2 --warmup 1 > $O/c5_base$i.json 2>> $O/err.txt || exit 1
  KB_LIB_PATH=genome-assembly_amd/lib/bk4u4/libkbin.so timeout -k 10 400 python -u bench.py --cpu-sample 0 --workload c5 --steps 2 --warmup 1 > $O/c5_u4_$i.json 2>> $O/err.txt || exit 1
done
echo done
