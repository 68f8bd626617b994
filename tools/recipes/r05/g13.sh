# r05 g13: ranked bins stage 4 B per occurrence (slot + 1 << 16 | rank) instead
# of 4 + 2 B: parity (parity, race, capacity suites), C3 alternating against
# lib/ab_prev with the digest asserted, C3 prof counters
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5g13; mkdir -p $O
T="python -u -m pytest -x -q -m gpu --timeout 900 --timeout-method thread"
NOX="--cpu-sample 0 --no-capacity --no-host-input"
timeout -k 10 1000 $T tests/test_gpu_parity.py tests/test_gpu_race.py tests/test_gpu_capacity.py > $O/parity.txt 2>&1 || exit 1
for i in 1 2; do
  KB_LIB_PATH=genome-assembly_amd/lib/ab_prev/libkbin.so timeout -k 10 300 python -u bench.py $NOX --workload c3 --steps 2 --warmup 1 --digest > $O/c3_prev_$i.json 2> $O/c3_prev_$i.err || exit 1
  timeout -k 10 300 python -u bench.py $NOX --workload c3 --steps 2 --warmup 1 --digest > $O/c3_new_$i.json 2> $O/c3_new_$i.err || exit 1
done
KB_LIB_PATH=genome-assembly_amd/lib/prof/libkbin.so timeout -k 10 400 python -u bench.py $NOX --workload c3 --steps 1 --warmup 2 > $O/c3_prof.json 2> $O/c3_prof.err || exit 1
echo done
