# r06 A/B: records in flight at 1024-thread bucket workgroups, C3 (digest) and
# C2: 8 (default) vs 12 vs 16
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/ab_bku3; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input --steps 20 --warmup 3"
L=genome-assembly_amd/lib
timeout -k 10 400 python -u bench.py --cpu-sample 0 --workload c3 --steps 3 --warmup 1 --digest > $O/c3_u8.json 2>> $O/err.txt || exit 1
KB_LIB_PATH=$L/bku12/libkbin.so timeout -k 10 400 python -u bench.py --cpu-sample 0 --workload c3 --steps 3 --warmup 1 --digest > $O/c3_u12.json 2>> $O/err.txt || exit 1
for i in 1 2; do
  timeout -k 10 300 python -u bench.py $NOX > $O/u8_$i.json 2>> $O/err.txt || exit 1
  for u in 12 16; do
    KB_LIB_PATH=$L/bku$u/libkbin.so timeout -k 10 300 python -u bench.py $NOX > $O/u${u}_$i.json 2>> $O/err.txt || exit 1
  done
done
echo done
