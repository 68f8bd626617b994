# r04 final evidence 3: FETCH_SIZE / WRITE_SIZE passes (separate) on the
# final build: C2 (the default workload), C3 (4 passes), C5 share, C4 share
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4f5; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c2_fetch -o pmc -- python3 bench.py $NOX --steps 5 --warmup 2 > $O/c2_fetch.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/c2_write -o pmc -- python3 bench.py $NOX --steps 5 --warmup 2 > $O/c2_write.log 2>&1 || exit 1
for w in c3 c5 c4; do
  timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/${w}_fetch -o pmc -- python3 bench.py $NOX --workload $w --steps 1 --warmup 1 > $O/${w}_fetch.log 2>&1 || exit 1
  timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/${w}_write -o pmc -- python3 bench.py $NOX --workload $w --steps 1 --warmup 1 > $O/${w}_write.log 2>&1 || exit 1
done
echo rc=$?
