# r04 g6: ranked-bin variant kernel (compact ranking, plain bin_kernel
# untouched): parity, C3 rank on/off with path counters, C2 line, C5 share
# with larger sub-bin budgets (light pre-filtered bins)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4g6; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  -k "ranked_bins or large_lists or clustered_long or light_prefilter or random_vs_oracle or known_answer" -m gpu > $O/tests.txt 2>&1 || exit 1
NOX="--cpu-sample 0 --no-capacity --no-host-input"
timeout -k 10 200 python -u bench.py $NOX --steps 20 --warmup 3 > $O/c2.json 2> $O/c2.err || exit 1
timeout -k 10 400 python -u bench.py $NOX --workload c3 --steps 2 --warmup 1 --digest > $O/c3.json 2> $O/c3.err || exit 1
KB_BIN_RANK=0 timeout -k 10 400 python -u bench.py $NOX --workload c3 --steps 2 --warmup 1 > $O/c3_norank.json 2> $O/c3_norank.err || exit 1
KB_BIN_SUB_EXTRA=120 timeout -k 10 400 python -u bench.py $NOX --workload c5 --steps 2 --warmup 1 --digest > $O/c5_x120.json 2> $O/c5_x120.err || exit 1
KB_BIN_SUB_EXTRA=240 timeout -k 10 400 python -u bench.py $NOX --workload c5 --steps 2 --warmup 1 --digest > $O/c5_x240.json 2> $O/c5_x240.err || exit 1
echo rc=$?
