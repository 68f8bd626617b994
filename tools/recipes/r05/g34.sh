# r05 g34: two-word keys' heavy partitions through the windows only when at
# most KB_BIN_WIN_HEAVY2_MAXW windows hold their ids (0: any) -- C5 share time
# per setting, then FETCH/WRITE of the best one
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5g34; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input"
for w in 0 1 2 4; do
  KB_BIN_WIN_HEAVY2_MAXW=$w timeout -k 10 300 python -u bench.py $NOX --workload c5 --steps 2 --warmup 2 --digest > $O/c5_w$w.json 2> $O/c5_w$w.err || exit 1
done
KB_BIN_WIN_HEAVY2=0 timeout -k 10 300 python -u bench.py $NOX --workload c5 --steps 2 --warmup 2 --digest > $O/c5_off.json 2> $O/c5_off.err || exit 1
echo done
