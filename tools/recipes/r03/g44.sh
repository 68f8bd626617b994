# round 3b: which allocations a C4-share run makes after other jobs on the box
# (KB_DEBUG: every allocation of 64 MB or more, with its time)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3c6; mkdir -p $O
timeout -k 10 300 python -u bench.py --cpu-sample 0 --no-capacity --no-host-input --workload c5 --steps 1 --warmup 1 > $O/c5_first.json 2> $O/c5_first.err || exit 1
KB_DEBUG=1 timeout -k 10 400 python -u bench.py --cpu-sample 0 --workload c4 --steps 2 --warmup 1 > $O/c4.json 2> $O/c4.err || exit 1
echo rc=$?
