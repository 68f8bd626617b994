# r05 g3: race stress + parity + dist (async group sender) on the new build
# (bin kernels read BinArgs through a pointer, branch-free register sorts);
# C2 and routed A/B alternating against lib/ab_old (args by value, sync send);
# generator twin, C2 oracle digest, repeated C3 regime test; C3 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5g3; mkdir -p $O
T="python -u -m pytest -x -v -m gpu --timeout 900 --timeout-method thread"
NOX="--cpu-sample 0 --no-capacity --no-host-input"
timeout -k 10 600 $T tests/test_gpu_race.py > $O/race.txt 2>&1 || exit 1
timeout -k 10 900 $T tests/test_gpu_parity.py > $O/parity.txt 2>&1 || exit 1
timeout -k 10 900 $T tests/test_gpu_dist.py > $O/dist.txt 2>&1 || exit 1
for i in 1 2; do
  KB_LIB_PATH=genome-assembly_amd/lib/ab_old/libkbin.so timeout -k 10 300 python -u bench.py $NOX --steps 30 --warmup 5 > $O/c2_old_$i.json 2> $O/c2_old_$i.err || exit 1
  timeout -k 10 300 python -u bench.py $NOX --steps 30 --warmup 5 > $O/c2_new_$i.json 2> $O/c2_new_$i.err || exit 1
done
timeout -k 10 300 python -u bench.py $NOX --routed --steps 30 --warmup 5 > $O/routed_new.json 2> $O/routed_new.err || exit 1
timeout -k 10 600 $T tests/test_gpu_scale.py -k "generator_twin or oracle_digest" > $O/twin.txt 2>&1 || exit 1
timeout -k 10 900 $T tests/test_gpu_capacity.py -k repeated > $O/c3rep.txt 2>&1 || exit 1
KB_LIB_PATH=genome-assembly_amd/lib/ab_old/libkbin.so timeout -k 10 300 python -u bench.py $NOX --workload c3 --steps 2 --warmup 1 > $O/c3_old.json 2> $O/c3_old.err || exit 1
timeout -k 10 300 python -u bench.py $NOX --workload c3 --steps 2 --warmup 1 > $O/c3_new.json 2> $O/c3_new.err || exit 1
echo done
