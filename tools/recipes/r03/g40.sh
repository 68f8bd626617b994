# round 3b: the split stage on the flat lists and split partitions too (heavy
# bins: C4 / C5 shares) vs KB_BIN_STAGE6=0; heavy-bin parity first
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3c3; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_capacity.py tests/test_gpu_scale.py -k "heavy or prefilter or split or offset or capacity or c3 or c4 or c5 or deferred" > $O/test_heavy.txt 2>&1 || exit 1
for w in c5 c4; do
  timeout -k 10 400 python -u bench.py --cpu-sample 0 --workload $w --steps 2 --warmup 1 --digest > $O/${w}_s6.json 2> $O/${w}_s6.err || exit 1
  KB_BIN_STAGE6=0 timeout -k 10 400 python -u bench.py --cpu-sample 0 --workload $w --steps 2 --warmup 1 --digest > $O/${w}_s8.json 2> $O/${w}_s8.err || exit 1
done
echo rc=$?
