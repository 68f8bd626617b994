# r05 g18: light bins stage 4 B per occurrence too (slot + 1 << 16 | record
# index; ordinals by record index in LDS for the windows, KB_BIN_PACK):
# parity suites, C2 alternating against lib/ab_prev and KB_BIN_PACK=0, C3
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5g18; mkdir -p $O
T="python -u -m pytest -x -q -m gpu --timeout 900 --timeout-method thread"
NOX="--cpu-sample 0 --no-capacity --no-host-input"
timeout -k 10 1000 $T tests/test_gpu_parity.py tests/test_gpu_race.py tests/test_gpu_capacity.py > $O/parity.txt 2>&1 || exit 1
for i in 1 2; do
  KB_LIB_PATH=genome-assembly_amd/lib/ab_prev/libkbin.so timeout -k 10 300 python -u bench.py $NOX --steps 30 --warmup 5 > $O/c2_prev_$i.json 2> $O/c2_prev_$i.err || exit 1
  timeout -k 10 300 python -u bench.py $NOX --steps 30 --warmup 5 > $O/c2_new_$i.json 2> $O/c2_new_$i.err || exit 1
  KB_BIN_PACK=0 timeout -k 10 300 python -u bench.py $NOX --steps 30 --warmup 5 > $O/c2_nopack_$i.json 2> $O/c2_nopack_$i.err || exit 1
done
timeout -k 10 300 python -u bench.py $NOX --workload c3 --steps 2 --warmup 1 --digest > $O/c3_new.json 2> $O/c3_new.err || exit 1
KB_LIB_PATH=genome-assembly_amd/lib/prof/libkbin.so timeout -k 10 300 python -u bench.py $NOX --steps 5 --warmup 2 > $O/c2_prof.json 2> $O/c2_prof.err || exit 1
echo done
