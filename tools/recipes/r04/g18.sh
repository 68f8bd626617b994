# r04 g18: C4 share with ranked bins (default) and without; C2 check
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4g18; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input"
timeout -k 10 400 python -u bench.py $NOX --workload c4 --steps 2 --warmup 1 --digest > $O/c4.json 2> $O/c4.err && \
KB_BIN_RANK=0 timeout -k 10 400 python -u bench.py $NOX --workload c4 --steps 2 --warmup 1 --digest > $O/c4_r0.json 2> $O/c4_r0.err && \
timeout -k 10 300 python -u bench.py $NOX --steps 20 --warmup 5 > $O/c2.json 2> $O/c2.err
echo rc=$?
