set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3x; mkdir -p $O
BENCH_DEBUG=1 KB_DEBUG=1 timeout -k 10 300 python -u bench.py --cpu-sample 0 --no-capacity --no-host-input --workload c5 --steps 1 --warmup 1 > $O/c5.json 2> $O/c5.err || exit 1
echo rc=$?
