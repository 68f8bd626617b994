# r05 g35: C5 share FETCH/WRITE with two-word heavy windows capped at one
# window per partition (KB_BIN_WIN_HEAVY2_MAXW=1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5g35; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input"
export KB_BIN_WIN_HEAVY2_MAXW=1
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c5_fetch -o pmc -- python3 bench.py $NOX --workload c5 --steps 1 --warmup 1 > $O/c5_fetch.log 2>&1 || exit 1
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/c5_write -o pmc -- python3 bench.py $NOX --workload c5 --steps 1 --warmup 1 > $O/c5_write.log 2>&1 || exit 1
echo done
