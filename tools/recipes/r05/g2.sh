# r05 g2: race stress (fixed / round-4 builds), generator twin, C2 oracle
# digest, the repeated default-knob C3 regime test, parity suite, default bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5g2; mkdir -p $O
T="python -u -m pytest -x -v -m gpu --timeout 900 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_race.py > $O/race.txt 2>&1 || exit 1
timeout -k 10 600 $T tests/test_gpu_scale.py -k "generator_twin or oracle_digest" > $O/twin.txt 2>&1 || exit 1
timeout -k 10 900 $T tests/test_gpu_capacity.py -k repeated > $O/c3rep.txt 2>&1 || exit 1
timeout -k 10 900 $T tests/test_gpu_parity.py > $O/parity.txt 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > $O/c2_bench.json 2> $O/c2_bench.err || exit 1
echo done
