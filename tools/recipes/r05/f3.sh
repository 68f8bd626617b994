# r05 final evidence 3: C5 share and C4 share FETCH_SIZE / WRITE_SIZE passes
# on the final build (traffic.json's C5 / C4 tags regenerated)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5f3; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input"
for w in c5 c4; do
  timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/${w}_fetch -o pmc -- python3 bench.py $NOX --workload $w --steps 1 --warmup 1 > $O/${w}_fetch.log 2>&1 || exit 1
  timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/${w}_write -o pmc -- python3 bench.py $NOX --workload $w --steps 1 --warmup 1 > $O/${w}_write.log 2>&1 || exit 1
done
echo rc=$?
