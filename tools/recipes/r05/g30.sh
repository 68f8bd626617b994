# r05 g30: two-word-key heavy partitions through the LDS id windows by
# default: the whole GPU suite, the C5 share and C4 share with digests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5g30; mkdir -p $O
timeout -k 10 1000 python -u -m pytest -x -q -m gpu --timeout 600 --timeout-method thread tests > $O/gpu_suite.txt 2>&1 || exit 1
timeout -k 10 500 python -u bench.py --cpu-sample 0 --workload c5 --steps 2 --warmup 2 --digest > $O/c5_share.json 2> $O/c5_share.err || exit 1
timeout -k 10 400 python -u bench.py --cpu-sample 0 --workload c4 --steps 2 --warmup 1 --digest > $O/c4_share.json 2> $O/c4_share.err || exit 1
echo done
