# r06: the C4 leg's allocations at full size (KB_DEBUG: every allocation of
# 64 MB or more, the prior map's capacity) to find the receiver's KB_ENOMEM
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/legs2; mkdir -p $O
KB_DEBUG=1 timeout -k 10 600 python -u bench.py --routed --multi-legs --steps 2 --warmup 1 --cpu-sample 0 --no-host-input > $O/legs.json 2> $O/legs.err
echo rc=$?
