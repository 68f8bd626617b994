# r06 evidence 1 (tree after the unitig replay, K < 2M widening, group cap
# fix): the default bench line; C2 kernel trace + stats and FETCH_SIZE /
# WRITE_SIZE passes; C3 / C4 share / C5 share with digests; the routed
# one-rank line; the drop-in at the reference's shipped M = 4 on C2's reads
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6f1; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input"
timeout -k 10 600 python -u bench.py > $O/c2_bench.json 2> $O/c2_bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 bench.py $NOX --steps 20 --warmup 3 > $O/kt.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o pmc -- python3 bench.py $NOX --steps 5 --warmup 2 > $O/pmc_fetch.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o pmc -- python3 bench.py $NOX --steps 5 --warmup 2 > $O/pmc_write.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --cpu-sample 0 --workload c4 --steps 2 --warmup 1 --digest > $O/c4_share.json 2> $O/c4_share.err || exit 1
timeout -k 10 500 python -u bench.py --cpu-sample 0 --workload c5 --steps 2 --warmup 2 --digest > $O/c5_share.json 2> $O/c5_share.err || exit 1
timeout -k 10 300 python -u bench.py $NOX --routed --steps 20 --warmup 3 > $O/routed.json 2> $O/routed.err || exit 1
timeout -k 10 600 python -u tools/unitig_time.py --reads 20000 1000000 --M 4 --full-max 0 --timeout 500 > $O/unitig_m4.jsonl 2> $O/unitig_m4.err || exit 1
echo rc=$?
