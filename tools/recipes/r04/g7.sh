# r04 g7: ranked bins with stage loads in flight and a popcount duplicate check
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4g7; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  -k "ranked_bins or large_lists or clustered_long" -m gpu > $O/tests.txt 2>&1 || exit 1
NOX="--cpu-sample 0 --no-capacity --no-host-input"
timeout -k 10 400 python -u bench.py $NOX --workload c3 --steps 2 --warmup 1 --digest > $O/c3.json 2> $O/c3.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_c3 -o kt \
  -- python3 bench.py $NOX --workload c3 --steps 2 --warmup 1 > $O/kt_c3.log 2>&1 || exit 1
echo rc=$?
