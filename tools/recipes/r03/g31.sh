# round 3b: speculative record pass (no mid-finalize sync) -- its test, the
# binned parity suite, A/B against KB_BIN_SPEC=0, a kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3b4; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v -m gpu --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "speculative or deferred or timing" > $O/test_spec.txt 2>&1 || exit 1
NOX="--cpu-sample 0 --no-capacity --no-host-input --steps 30 --warmup 5"
for i in 1 2; do
  timeout -k 10 200 python -u bench.py $NOX > $O/spec$i.json 2> $O/spec$i.err || exit 1
  KB_BIN_SPEC=0 timeout -k 10 200 python -u bench.py $NOX > $O/nospec$i.json 2> $O/nospec$i.err || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 bench.py --cpu-sample 0 --no-capacity --no-host-input --steps 10 --warmup 3 > $O/kt.log 2>&1 || exit 1
timeout -k 10 1500 python -u -m pytest -x -q -m gpu --timeout 900 --timeout-method thread tests > $O/gpu_tests.txt 2>&1 || exit 1
echo rc=$?
