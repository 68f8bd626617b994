# round 3b: the light bins' stage as 4-B ordinals + 2-B slots (KB_BIN_STAGE6,
# default) vs the 8-B entries (KB_BIN_STAGE6=0), alternating; FETCH/WRITE
# passes of the new default; parity suite
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3c1; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "random or cutoffs or large or offset or edge or ids or deferred or timing or scale" > $O/test_quick.txt 2>&1 || exit 1
NOX="--cpu-sample 0 --no-capacity --no-host-input --steps 30 --warmup 5"
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py $NOX > $O/s6_$i.json 2> $O/s6_$i.err || exit 1
  KB_BIN_STAGE6=0 timeout -k 10 200 python -u bench.py $NOX > $O/s8_$i.json 2> $O/s8_$i.err || exit 1
done
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o pmc -- python3 bench.py --cpu-sample 0 --no-capacity --no-host-input --steps 5 --warmup 2 > $O/pmc_fetch.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o pmc -- python3 bench.py --cpu-sample 0 --no-capacity --no-host-input --steps 5 --warmup 2 > $O/pmc_write.log 2>&1 || exit 1
timeout -k 10 1500 python -u -m pytest -x -q -m gpu --timeout 900 --timeout-method thread tests > $O/gpu_tests.txt 2>&1 || exit 1
echo rc=$?
