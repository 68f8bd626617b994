# r06 evidence 5b (final tree): C3 / C4 share / C5 share with digests, the
# routed one-rank line, and the N > 1 run's C4 / C5 legs at full size through
# a one-rank RCCL group
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6f5b; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input"
timeout -k 10 400 python -u bench.py --cpu-sample 0 --workload c3 --steps 3 --warmup 1 --digest > $O/c3.json 2> $O/c3.err || exit 1
timeout -k 10 400 python -u bench.py --cpu-sample 0 --workload c4 --steps 2 --warmup 1 --digest > $O/c4_share.json 2> $O/c4_share.err || exit 1
timeout -k 10 500 python -u bench.py --cpu-sample 0 --workload c5 --steps 2 --warmup 2 --digest > $O/c5_share.json 2> $O/c5_share.err || exit 1
timeout -k 10 300 python -u bench.py $NOX --routed --steps 20 --warmup 3 > $O/routed.json 2> $O/routed.err || exit 1
timeout -k 10 900 python -u bench.py --routed --multi-legs --steps 10 --warmup 2 --cpu-sample 0 --no-host-input > $O/legs.json 2> $O/legs.err || exit 1
echo done
