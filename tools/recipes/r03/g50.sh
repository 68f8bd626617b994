# round 3b: bucket_kernel reads each 24-B record with one 16-B and one 8-B load
# (lib/ld2) vs HEAD, alternating; bucket-path parity with lib/ld2
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3d1; mkdir -p $O
KB_LIB_PATH=genome-assembly_amd/lib/ld2/libkbin.so timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_dist.py -k "balanced or edge_inputs or random or partitioned or receiver or route or virtual or large" > $O/test_ld2.txt 2>&1 || exit 1
NOX="--cpu-sample 0 --no-capacity --no-host-input --steps 30 --warmup 5"
for i in 1 2 3; do
  KB_LIB_PATH=genome-assembly_amd/lib/ld2/libkbin.so timeout -k 10 200 python -u bench.py $NOX > $O/ld2_$i.json 2> $O/ld2_$i.err || exit 1
  timeout -k 10 200 python -u bench.py $NOX > $O/cur_$i.json 2> $O/cur_$i.err || exit 1
done
echo rc=$?
