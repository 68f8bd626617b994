# round 3b: cold-pass breakdown (KB_DEBUG host timings + phase events), and a
# kernel trace of the first C2 finalizes of a fresh context
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3c2; mkdir -p $O
KB_DEBUG=1 timeout -k 10 200 python -u tools/cold.py --workload c2 --steps 3 > $O/cold.txt 2> $O/cold_dbg.txt || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o kt -- python3 tools/cold.py --workload c2 --steps 2 > $O/kt.log 2>&1 || exit 1
echo rc=$?
