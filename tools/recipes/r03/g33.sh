# round 3b: (header, word 0) pair record layout (16-B placement stores) vs
# HEAD 35c61e3 (lib/ab_old); C5 share vs the same; then the -m gpu suite
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3b6; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "two_word or radix or balanced or edge_inputs or heavy" > $O/test_quick.txt 2>&1 || exit 1
NOX="--cpu-sample 0 --no-capacity --no-host-input --steps 30 --warmup 5"
for i in 1 2; do
  timeout -k 10 200 python -u bench.py $NOX > $O/new$i.json 2> $O/new$i.err || exit 1
  KB_LIB_PATH=genome-assembly_amd/lib/ab_old/libkbin.so timeout -k 10 200 python -u bench.py $NOX > $O/old$i.json 2> $O/old$i.err || exit 1
done
timeout -k 10 300 python -u bench.py --cpu-sample 0 --workload c5 --steps 2 --warmup 1 --digest > $O/c5_new.json 2> $O/c5_new.err || exit 1
KB_LIB_PATH=genome-assembly_amd/lib/ab_old/libkbin.so timeout -k 10 300 python -u bench.py --cpu-sample 0 --workload c5 --steps 2 --warmup 1 --digest > $O/c5_old.json 2> $O/c5_old.err || exit 1
timeout -k 10 1500 python -u -m pytest -x -q -m gpu --timeout 900 --timeout-method thread tests > $O/gpu_tests.txt 2>&1 || exit 1
echo rc=$?
