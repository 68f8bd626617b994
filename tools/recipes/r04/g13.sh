# r04 g13: static serpentine bin schedule (A/B), C5 bin distribution dump
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4g13; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input"
timeout -k 10 300 python -u bench.py $NOX --steps 20 --warmup 5 --digest > $O/c2_dyn.json 2> $O/c2_dyn.err && \
KB_BIN_SCHED=1 timeout -k 10 300 python -u bench.py $NOX --steps 20 --warmup 5 --digest > $O/c2_static.json 2> $O/c2_static.err && \
timeout -k 10 300 python -u bench.py $NOX --steps 20 --warmup 5 > $O/c2_dyn2.json 2> $O/c2_dyn2.err && \
KB_BIN_SCHED=1 timeout -k 10 300 python -u bench.py $NOX --steps 20 --warmup 5 > $O/c2_static2.json 2> $O/c2_static2.err && \
KB_DIAG_BINS=$O/c5_bins.txt timeout -k 10 500 python -u bench.py $NOX --workload c5 --steps 1 --warmup 2 > $O/c5.json 2> $O/c5.err
echo rc=$?
