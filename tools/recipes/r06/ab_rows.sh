# r06 A/B: the record pass's row loads eight in flight per lane (new) against
# one at a time (base), C2 bench alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/ab_rows; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input --steps 20 --warmup 3"
for i in 1 2 3; do
  KB_LIB_PATH=genome-assembly_amd/lib/base/libkbin.so timeout -k 10 300 python -u bench.py $NOX > $O/base$i.json 2>> $O/err.txt || exit 1
  timeout -k 10 300 python -u bench.py $NOX > $O/new$i.json 2>> $O/err.txt || exit 1
done
echo done
