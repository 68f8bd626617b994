# r04 g31: the long-list regime's sub-bin fill at C3: 30 / 50 / 60 % against
# the default 40 %
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4g31; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input"
timeout -k 10 300 python -u bench.py $NOX --workload c3 --steps 2 --warmup 2 > $O/c3_40.json 2> $O/c3_40.err || exit 1
for f in 30 50 60; do
  KB_BIN_SUB_FILL_PCT=$f timeout -k 10 300 python -u bench.py $NOX --workload c3 --steps 2 --warmup 2 --digest > $O/c3_$f.json 2> $O/c3_$f.err || exit 1
done
timeout -k 10 300 python -u bench.py $NOX --workload c3 --steps 2 --warmup 2 > $O/c3_40b.json 2> $O/c3_40b.err || exit 1
echo rc=$?
