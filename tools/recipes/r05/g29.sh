# r05 g29: LDS id windows in the heavy partitions of two-word-key bins too
# (KB_BIN_WIN_HEAVY2=1): C5 share parity (digest) and time, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5g29; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input"
T="python -u -m pytest -x -q -m gpu --timeout 900 --timeout-method thread"
KB_BIN_WIN_HEAVY2=1 timeout -k 10 800 $T tests/test_gpu_scale.py tests/test_gpu_capacity.py tests/test_gpu_parity.py -k "c5 or prefilter" > $O/c5_tests.txt 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 300 python -u bench.py $NOX --workload c5 --steps 2 --warmup 2 --digest > $O/c5_off_$i.json 2> $O/c5_off_$i.err || exit 1
  KB_BIN_WIN_HEAVY2=1 timeout -k 10 300 python -u bench.py $NOX --workload c5 --steps 2 --warmup 2 --digest > $O/c5_on_$i.json 2> $O/c5_on_$i.err || exit 1
done
echo done
