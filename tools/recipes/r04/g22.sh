# r04 g22: is the receiver conversion's write traffic cross-XCD line sharing?
# WRITE_SIZE of sk_convert_buckets_kernel with every block converting, and
# with only the blocks of one XCD group (KB_DIAG_CONVERT_GROUP=1: 1/8 of the
# records, results wrong by design)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4g22; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input"
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/all -o pmc -- python3 bench.py $NOX --workload c3 --steps 1 --warmup 1 > $O/all.log 2>&1 && \
KB_DIAG_CONVERT_GROUP=1 timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/grp -o pmc -- python3 bench.py $NOX --workload c3 --steps 1 --warmup 1 > $O/grp.log 2>&1
echo rc=$?
