# r06 A/B: bucket_kernel records in flight per thread (K <= 31): 4 (default)
# against 2, 6, 8; C2 bench alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/ab_bku; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input --steps 20 --warmup 3"
L=genome-assembly_amd/lib
for i in 1 2; do
  timeout -k 10 300 python -u bench.py $NOX > $O/u4_$i.json 2>> $O/err.txt || exit 1
  for u in 2 6 8; do
    KB_LIB_PATH=$L/bku$u/libkbin.so timeout -k 10 300 python -u bench.py $NOX > $O/u${u}_$i.json 2>> $O/err.txt || exit 1
  done
done
echo done
