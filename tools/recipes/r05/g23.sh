# r05 g23 (rerun as g25 with the b-1 edge split): the edge split by its pre-context (BM_EDGE): C3 with the digest, C2,
# C5 and C4 shares, alternating against lib/ab_prev (the previous commit)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5g23; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input"
P=genome-assembly_amd/lib/ab_prev/libkbin.so
for i in 1 2; do
  KB_LIB_PATH=$P timeout -k 10 300 python -u bench.py $NOX --workload c3 --steps 2 --warmup 1 --digest > $O/c3_prev_$i.json 2> $O/c3_prev_$i.err || exit 1
  timeout -k 10 300 python -u bench.py $NOX --workload c3 --steps 2 --warmup 1 --digest > $O/c3_new_$i.json 2> $O/c3_new_$i.err || exit 1
done
for i in 1 2; do
  KB_LIB_PATH=$P timeout -k 10 300 python -u bench.py $NOX --steps 30 --warmup 5 > $O/c2_prev_$i.json 2> $O/c2_prev_$i.err || exit 1
  timeout -k 10 300 python -u bench.py $NOX --steps 30 --warmup 5 > $O/c2_new_$i.json 2> $O/c2_new_$i.err || exit 1
done
for w in c5 c4; do
  KB_LIB_PATH=$P timeout -k 10 300 python -u bench.py $NOX --workload $w --steps 2 --warmup 1 --digest > $O/${w}_prev.json 2> $O/${w}_prev.err || exit 1
  timeout -k 10 300 python -u bench.py $NOX --workload $w --steps 2 --warmup 1 --digest > $O/${w}_new.json 2> $O/${w}_new.err || exit 1
done
echo done
