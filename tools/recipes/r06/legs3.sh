# r06: C4 at 1/10 of a rank's reads, KB_DEBUG, direct split passes vs the
# routed one-rank group leg (bucket maps, largest buckets, reruns)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/legs3; mkdir -p $O
KB_DEBUG=1 timeout -k 10 300 python -u bench.py --workload c4 --reads 12500000 --steps 1 --warmup 1 --cpu-sample 0 --no-host-input > $O/direct.json 2> $O/direct.err || exit 1
KB_DEBUG=1 KB_CAPACITY_SCALE=10 timeout -k 10 400 python -u bench.py --routed --multi-legs --steps 1 --warmup 1 --cpu-sample 0 --no-host-input > $O/legs.json 2> $O/legs.err
echo rc=$?
