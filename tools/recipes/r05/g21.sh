# r05 g21: ranked bins' rank -> ordinal map written through an LDS inverse
# (coalesced rord stores): ranked parity (race, capacity), C3 alternating
# against lib/ab_prev, then the prof build's record re-expansion counters by
# bin kind with the pass's bin table (KB_DIAG_BINS)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5g21; mkdir -p $O
T="python -u -m pytest -x -q -m gpu --timeout 900 --timeout-method thread"
NOX="--cpu-sample 0 --no-capacity --no-host-input"
timeout -k 10 900 $T tests/test_gpu_race.py tests/test_gpu_capacity.py > $O/parity.txt 2>&1 || exit 1
for i in 1 2; do
  KB_LIB_PATH=genome-assembly_amd/lib/ab_prev/libkbin.so timeout -k 10 300 python -u bench.py $NOX --workload c3 --steps 2 --warmup 1 --digest > $O/c3_prev_$i.json 2> $O/c3_prev_$i.err || exit 1
  timeout -k 10 300 python -u bench.py $NOX --workload c3 --steps 2 --warmup 1 --digest > $O/c3_new_$i.json 2> $O/c3_new_$i.err || exit 1
done
KB_DIAG_BINS=$O/c3_bins.txt KB_LIB_PATH=genome-assembly_amd/lib/prof/libkbin.so timeout -k 10 400 python -u bench.py $NOX --workload c3 --steps 1 --warmup 2 > $O/c3_prof.json 2> $O/c3_prof.err || exit 1
echo done
