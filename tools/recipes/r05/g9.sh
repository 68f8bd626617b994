# r05 g9: bin kernels through a pointer with global-typed fields (no FLAT
# ops), ranked included: parity subset, then C2 (alternating) / C3 / C5 / C4
# against lib/ab_old (round 4's by-value kernels)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5g9; mkdir -p $O
T="python -u -m pytest -x -q -m gpu --timeout 900 --timeout-method thread"
NOX="--cpu-sample 0 --no-capacity --no-host-input"
timeout -k 10 900 $T tests/test_gpu_parity.py tests/test_gpu_race.py > $O/parity.txt 2>&1 || exit 1
for i in 1 2; do
  KB_LIB_PATH=genome-assembly_amd/lib/ab_old/libkbin.so timeout -k 10 300 python -u bench.py $NOX --steps 30 --warmup 5 > $O/c2_old_$i.json 2> $O/c2_old_$i.err || exit 1
  timeout -k 10 300 python -u bench.py $NOX --steps 30 --warmup 5 > $O/c2_new_$i.json 2> $O/c2_new_$i.err || exit 1
done
timeout -k 10 300 python -u bench.py $NOX --workload c3 --steps 2 --warmup 1 --digest > $O/c3_new.json 2> $O/c3_new.err || exit 1
KB_LIB_PATH=genome-assembly_amd/lib/ab_old/libkbin.so timeout -k 10 300 python -u bench.py $NOX --workload c3 --steps 2 --warmup 1 > $O/c3_old.json 2> $O/c3_old.err || exit 1
timeout -k 10 500 python -u bench.py --cpu-sample 0 --workload c5 --steps 2 --warmup 2 --digest > $O/c5_new.json 2> $O/c5_new.err || exit 1
timeout -k 10 400 python -u bench.py --cpu-sample 0 --workload c4 --steps 2 --warmup 1 --digest > $O/c4_new.json 2> $O/c4_new.err || exit 1
echo done
