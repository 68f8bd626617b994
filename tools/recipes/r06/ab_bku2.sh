# r06 A/B: records in flight at 1024-thread bucket workgroups: 8 (default) vs 4, 12
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/ab_bku2; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input --steps 20 --warmup 3"
L=genome-assembly_amd/lib
for i in 1 2; do
  timeout -k 10 300 python -u bench.py $NOX > $O/u8_$i.json 2>> $O/err.txt || exit 1
  for u in 4 12; do
    KB_LIB_PATH=$L/bku$u/libkbin.so timeout -k 10 300 python -u bench.py $NOX > $O/u${u}_$i.json 2>> $O/err.txt || exit 1
  done
done
echo done
