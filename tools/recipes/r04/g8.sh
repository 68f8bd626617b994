# r04 g8: C5 share with sub-bins sized for the light pre-filter's sketch
# (digest), C5 parity at default knobs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4g8; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input"
timeout -k 10 500 python -u bench.py $NOX --workload c5 --steps 2 --warmup 2 --digest > $O/c5.json 2> $O/c5.err || exit 1
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_gpu_capacity.py \
  -k "c5" -m gpu > $O/tests.txt 2>&1 || exit 1
echo rc=$?
