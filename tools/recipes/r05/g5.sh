# r05 g5: ranked kernel back to by-value args (C3 A/B vs lib/ab_old), the C5
# share with sub-bins to depth 5 (parity tests + bench A/B with digest), C4
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5g5; mkdir -p $O
T="python -u -m pytest -x -v -m gpu --timeout 900 --timeout-method thread"
NOX="--cpu-sample 0 --no-capacity --no-host-input"
timeout -k 10 600 $T tests/test_gpu_parity.py -k "ranked or large_lists or clustered" > $O/ranked.txt 2>&1 || exit 1
timeout -k 10 300 python -u bench.py $NOX --workload c3 --steps 2 --warmup 1 > $O/c3_new.json 2> $O/c3_new.err || exit 1
KB_LIB_PATH=genome-assembly_amd/lib/ab_old/libkbin.so timeout -k 10 300 python -u bench.py $NOX --workload c3 --steps 2 --warmup 1 > $O/c3_old.json 2> $O/c3_old.err || exit 1
timeout -k 10 900 $T tests/test_gpu_capacity.py -k "c5" > $O/c5tests.txt 2>&1 || exit 1
timeout -k 10 500 python -u bench.py --cpu-sample 0 --workload c5 --steps 2 --warmup 2 --digest > $O/c5_new.json 2> $O/c5_new.err || exit 1
KB_LIB_PATH=genome-assembly_amd/lib/ab_old/libkbin.so timeout -k 10 500 python -u bench.py --cpu-sample 0 --workload c5 --steps 2 --warmup 2 --digest > $O/c5_old.json 2> $O/c5_old.err || exit 1
echo done
