# r05 g17: C3 FETCH_SIZE / WRITE_SIZE passes on the packed ranked stage
# (traffic.json's C3 tag regenerated from them) + C3 kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5g17; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3_kt -o kt -- python3 bench.py $NOX --workload c3 --steps 2 --warmup 1 > $O/c3_kt.log 2>&1 || exit 1
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c3_fetch -o pmc -- python3 bench.py $NOX --workload c3 --steps 1 --warmup 1 > $O/c3_fetch.log 2>&1 || exit 1
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/c3_write -o pmc -- python3 bench.py $NOX --workload c3 --steps 1 --warmup 1 > $O/c3_write.log 2>&1 || exit 1
echo done
