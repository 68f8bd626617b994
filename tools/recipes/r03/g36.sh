# round 3b evidence: e_hi left zero for one-word keys + the bench's Python
# bookkeeping after the timed steps, vs HEAD bfe7876; GPU suite; smoke; the
# default bench line (capacity + host-input legs); kernel trace + stats;
# FETCH_SIZE / WRITE_SIZE passes (separate) for the C2 traffic
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3b9; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input --steps 30 --warmup 5"
for i in 1 2; do
  timeout -k 10 200 python -u bench.py $NOX > $O/new$i.json 2> $O/new$i.err || exit 1
  KB_LIB_PATH=genome-assembly_amd/lib/ab_old/libkbin.so timeout -k 10 200 python -u bench.py $NOX > $O/old$i.json 2> $O/old$i.err || exit 1
done
timeout -k 10 1500 python -u -m pytest -x -q -m gpu --timeout 900 --timeout-method thread tests > $O/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > $O/c2_bench.json 2> $O/c2_bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 bench.py --cpu-sample 0 --no-capacity --no-host-input --steps 20 --warmup 3 > $O/kt.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o pmc -- python3 bench.py --cpu-sample 0 --no-capacity --no-host-input --steps 5 --warmup 2 > $O/pmc_fetch.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o pmc -- python3 bench.py --cpu-sample 0 --no-capacity --no-host-input --steps 5 --warmup 2 > $O/pmc_write.log 2>&1 || exit 1
echo rc=$?
