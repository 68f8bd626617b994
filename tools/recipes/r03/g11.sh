set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3j; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input"
for f in 50 80 120 160 240; do
  KB_BIN_SUB_FILL_PCT=$f timeout -k 10 120 python -u bench.py $NOX --steps 20 --warmup 5 > $O/c2_f$f.json 2> $O/c2_f$f.err || exit 1
  KB_BIN_SUB_FILL_PCT=$f timeout -k 10 200 python -u bench.py $NOX --reads 8000000 --genome 40000000 --parts 8 --steps 3 --warmup 2 > $O/zs8_f$f.json 2> $O/zs8_f$f.err || exit 1
done
echo rc=$?
