set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3q; mkdir -p $O
timeout -k 10 100 python -u tools/cold.py --workload c2 --steps 3 > $O/cold_c2.txt 2>&1 || exit 1
KB_BIN_HLL=0 timeout -k 10 100 python -u tools/cold.py --workload c2 --steps 3 > $O/cold_c2_nohll.txt 2>&1 || exit 1
KB_DEBUG=1 timeout -k 10 100 python -u tools/cold.py --workload c2 --steps 2 > $O/cold_c2_dbg.txt 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --cpu-sample 0 --no-capacity --no-host-input --steps 20 --warmup 5 > $O/c2.json 2> $O/c2.err || exit 1
echo rc=$?
