# r04 final evidence 7: C3 FETCH_SIZE / WRITE_SIZE passes with the long-list
# regime's sub-bins (the C3 tag of traffic.json is regenerated from them)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4f9; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c3_fetch -o pmc -- python3 bench.py $NOX --workload c3 --steps 1 --warmup 1 > $O/c3_fetch.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/c3_write -o pmc -- python3 bench.py $NOX --workload c3 --steps 1 --warmup 1 > $O/c3_write.log 2>&1 || exit 1
echo rc=$?
