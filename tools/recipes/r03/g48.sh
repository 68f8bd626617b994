# round 3b final evidence (the id-window fix): GPU suite; smoke; default bench
# line; 6-B vs 8-B stage A/B; C2 kernel trace + stats; FETCH/WRITE; SQ; C4 / C5
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3z3; mkdir -p $O
timeout -k 10 1500 python -u -m pytest -x -v -m gpu --timeout 900 --timeout-method thread tests > $O/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > $O/c2_bench.json 2> $O/c2_bench.err || exit 1
NOX="--cpu-sample 0 --no-capacity --no-host-input --steps 30 --warmup 5"
for i in 1 2; do
  timeout -k 10 200 python -u bench.py $NOX > $O/s6_$i.json 2> $O/s6_$i.err || exit 1
  KB_BIN_STAGE6=0 timeout -k 10 200 python -u bench.py $NOX > $O/s8_$i.json 2> $O/s8_$i.err || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 bench.py --cpu-sample 0 --no-capacity --no-host-input --steps 20 --warmup 3 > $O/kt.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o pmc -- python3 bench.py --cpu-sample 0 --no-capacity --no-host-input --steps 5 --warmup 2 > $O/pmc_fetch.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o pmc -- python3 bench.py --cpu-sample 0 --no-capacity --no-host-input --steps 5 --warmup 2 > $O/pmc_write.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $O/sq -o sq -- python3 bench.py --cpu-sample 0 --no-capacity --no-host-input --steps 5 --warmup 2 > $O/sq.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --cpu-sample 0 --workload c5 --steps 2 --warmup 1 --digest > $O/c5_share.json 2> $O/c5_share.err || exit 1
timeout -k 10 400 python -u bench.py --cpu-sample 0 --workload c4 --steps 2 --warmup 1 --digest > $O/c4_share.json 2> $O/c4_share.err || exit 1
echo rc=$?
