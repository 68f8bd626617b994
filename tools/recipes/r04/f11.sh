# r04 final evidence 9: the default bench line and the C3 leg again, reading
# the C3 tag regenerated from f9
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4f11; mkdir -p $O
timeout -k 10 600 python -u bench.py > $O/c2_bench.json 2> $O/c2_bench.err || exit 1
timeout -k 10 400 python -u bench.py --cpu-sample 0 --workload c3 --steps 2 --warmup 2 --digest > $O/c3.json 2> $O/c3.err || exit 1
echo rc=$?
