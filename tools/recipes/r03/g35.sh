# round 3b: K <= 31 bin-ordered records in 32-B rows (bucket_kernel's two
# stores per record into one row) + e_hi left zero for one-word keys, vs HEAD
# bfe7876 (pairs + word 1 arrays); then the -m gpu suite
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3b8; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "radix or balanced or edge_inputs or heavy or split or offset" > $O/test_quick.txt 2>&1 || exit 1
NOX="--cpu-sample 0 --no-capacity --no-host-input --steps 30 --warmup 5"
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py $NOX > $O/new$i.json 2> $O/new$i.err || exit 1
  KB_LIB_PATH=genome-assembly_amd/lib/ab_old/libkbin.so timeout -k 10 200 python -u bench.py $NOX > $O/old$i.json 2> $O/old$i.err || exit 1
done
timeout -k 10 1500 python -u -m pytest -x -q -m gpu --timeout 900 --timeout-method thread tests > $O/gpu_tests.txt 2>&1 || exit 1
echo rc=$?
