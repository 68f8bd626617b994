# r04 final evidence 5: the default bench line (reads the regenerated
# traffic.json), C3 / C4 share / C5 share benches (digests), routed
# C2, C3 kernel trace, the drop-in's C2 wall time
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4f7; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input"
timeout -k 10 600 python -u bench.py > $O/c2_bench.json 2> $O/c2_bench.err || exit 1
timeout -k 10 400 python -u bench.py --cpu-sample 0 --workload c3 --steps 2 --warmup 1 --digest > $O/c3.json 2> $O/c3.err || exit 1
timeout -k 10 400 python -u bench.py --cpu-sample 0 --workload c4 --steps 2 --warmup 1 --digest > $O/c4_share.json 2> $O/c4_share.err || exit 1
timeout -k 10 500 python -u bench.py --cpu-sample 0 --workload c5 --steps 2 --warmup 2 --digest > $O/c5_share.json 2> $O/c5_share.err || exit 1
timeout -k 10 300 python -u bench.py $NOX --routed --steps 20 --warmup 3 > $O/routed.json 2> $O/routed.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_c3 -o kt -- python3 bench.py $NOX --workload c3 --steps 2 --warmup 1 > $O/kt_c3.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/unitig_time.py --reads 1000000 --full-max 0 --timeout 280 > $O/unitig_c2.jsonl 2> $O/unitig_c2.err || exit 1
echo rc=$?
