# r06 A/B: two-word records in flight per thread in the 1024-thread bucket
# ordering (KB_BK_U4: 4 shipped, tuned at 512 threads) -- C5 share, digest-compared
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/ab_bk4; mkdir -p $O
L=genome-assembly_amd/lib
C5="--cpu-sample 0 --workload c5 --steps 2 --warmup 1 --digest"
for i in 1 2; do
  timeout -k 10 400 python -u bench.py $C5 > $O/u4_$i.json 2>> $O/err.txt || exit 1
  for u in 6 8; do
    KB_LIB_PATH=$L/bk4u$u/libkbin.so timeout -k 10 400 python -u bench.py $C5 > $O/u${u}_$i.json 2>> $O/err.txt || exit 1
  done
done
echo done
