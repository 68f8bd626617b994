# round 3b: prior maps packed by one serpentine sweep (default) vs sorted LPT
# (KB_BIN_PRIOR_LPT=1): the cold C2 step, alternating fresh processes; the
# prior-map parity cases
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3c5; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "balanced or edge_inputs or partitioned or speculative or deferred" > $O/test_prior.txt 2>&1 || exit 1
for i in 1 2 3; do
  KB_DEBUG=1 timeout -k 10 120 python -u tools/cold.py --workload c2 --steps 2 > $O/serp$i.txt 2> $O/serp$i.err || exit 1
  KB_DEBUG=1 KB_BIN_PRIOR_LPT=1 timeout -k 10 120 python -u tools/cold.py --workload c2 --steps 2 > $O/lpt$i.txt 2> $O/lpt$i.err || exit 1
done
NOX="--cpu-sample 0 --no-capacity --no-host-input --steps 10 --warmup 2"
timeout -k 10 200 python -u bench.py $NOX > $O/bench_serp.json 2> $O/bench_serp.err || exit 1
KB_BIN_PRIOR_LPT=1 timeout -k 10 200 python -u bench.py $NOX > $O/bench_lpt.json 2> $O/bench_lpt.err || exit 1
echo rc=$?
