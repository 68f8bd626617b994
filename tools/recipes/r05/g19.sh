# r05 g19: the table zeroed with 16-B LDS stores: parity subset, C2 and C3
# alternating against lib/ab_prev (the previous commit)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5g19; mkdir -p $O
T="python -u -m pytest -x -q -m gpu --timeout 900 --timeout-method thread"
NOX="--cpu-sample 0 --no-capacity --no-host-input"
timeout -k 10 900 $T tests/test_gpu_parity.py tests/test_gpu_race.py > $O/parity.txt 2>&1 || exit 1
for i in 1 2; do
  KB_LIB_PATH=genome-assembly_amd/lib/ab_prev/libkbin.so timeout -k 10 300 python -u bench.py $NOX --steps 30 --warmup 5 > $O/c2_prev_$i.json 2> $O/c2_prev_$i.err || exit 1
  timeout -k 10 300 python -u bench.py $NOX --steps 30 --warmup 5 > $O/c2_new_$i.json 2> $O/c2_new_$i.err || exit 1
done
for i in 1 2; do
  KB_LIB_PATH=genome-assembly_amd/lib/ab_prev/libkbin.so timeout -k 10 300 python -u bench.py $NOX --workload c3 --steps 2 --warmup 1 --digest > $O/c3_prev_$i.json 2> $O/c3_prev_$i.err || exit 1
  timeout -k 10 300 python -u bench.py $NOX --workload c3 --steps 2 --warmup 1 --digest > $O/c3_new_$i.json 2> $O/c3_new_$i.err || exit 1
done
echo done
