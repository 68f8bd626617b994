# r04 g3: light pre-filtered bins (two-word keys): parity tests, C5 share A/B
# (KB_BIN_PF_LIGHT 1 vs 0, digest); ranked bins (C3's long lists from
# per-key bitmaps over record ranks): parity tests, C3 with digest and its
# kernel trace; the C2 drop-in's phase breakdown
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4g3; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_capacity.py -k "light_prefilter or c5_singleton or ranked_bins or large_lists or clustered_long or heavy_bins_flat" \
  -m gpu > $O/tests.txt 2>&1 || exit 1
NOX="--cpu-sample 0 --no-capacity --no-host-input"
timeout -k 10 400 python -u bench.py $NOX --workload c3 --steps 2 --warmup 1 --digest > $O/c3.json 2> $O/c3.err || exit 1
timeout -k 10 400 python -u bench.py $NOX --workload c5 --steps 2 --warmup 1 --digest > $O/c5_light.json 2> $O/c5_light.err || exit 1
KB_BIN_PF_LIGHT=0 timeout -k 10 400 python -u bench.py $NOX --workload c5 --steps 2 --warmup 1 --digest > $O/c5_flat.json 2> $O/c5_flat.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_c3 -o kt \
  -- python3 bench.py $NOX --workload c3 --steps 2 --warmup 1 > $O/kt_c3.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/unitig_time.py --reads 1000000 --full-max 0 --timeout 280 > $O/unitig_c2.jsonl 2> $O/unitig_c2.err || exit 1
echo rc=$?
