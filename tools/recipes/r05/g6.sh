# r05 g6: profiles of the fixed build at C2 -- kernel trace + stats, the SQ
# counter pass (once, on the fixed build, to completion),
# FETCH_SIZE and WRITE_SIZE passes for traffic.json
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5g6; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 bench.py $NOX --steps 20 --warmup 3 > $O/kt.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $O/sq -o sq -- python3 bench.py $NOX --steps 5 --warmup 2 > $O/sq.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o pmc -- python3 bench.py $NOX --steps 5 --warmup 2 > $O/pmc_fetch.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o pmc -- python3 bench.py $NOX --steps 5 --warmup 2 > $O/pmc_write.log 2>&1 || exit 1
echo done
