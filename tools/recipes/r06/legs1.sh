# r06: the N > 1 run's C4 and C5 legs at full per-rank size through a
# one-rank RCCL group (bench.py --routed --multi-legs): memory and time
# rehearsal of what the driver's 8-GPU run will execute per rank
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/legs1; mkdir -p $O
timeout -k 10 1000 python -u bench.py --routed --multi-legs --steps 5 --warmup 2 --cpu-sample 0 --no-host-input > $O/legs.json 2> $O/legs.err || exit 1
echo done
