set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3h; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input"
KB_DEBUG=1 timeout -k 10 120 python -u tools/cold.py --workload c2 --steps 3 > $O/cold_c2.txt 2>&1 && \
timeout -k 10 400 python -u bench.py $NOX --workload c4 --steps 2 --warmup 1 --digest > $O/c4.json 2> $O/c4.err && \
timeout -k 10 400 python -u bench.py $NOX --workload c5 --steps 2 --warmup 1 --digest > $O/c5.json 2> $O/c5.err
echo rc=$?
