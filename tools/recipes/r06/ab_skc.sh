# r06 A/B: the record pass's count loop with 2 (default), 4, 8 records (and
# their bucket-map loads) per trip; C2 alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/ab_skc; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input --steps 20 --warmup 3"
L=genome-assembly_amd/lib
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py $NOX > $O/c2_$i.json 2>> $O/err.txt || exit 1
  for c in 4 8; do
    KB_LIB_PATH=$L/skc$c/libkbin.so timeout -k 10 300 python -u bench.py $NOX > $O/c${c}_$i.json 2>> $O/err.txt || exit 1
  done
done
echo done
