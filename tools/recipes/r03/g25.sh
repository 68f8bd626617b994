set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3w; mkdir -p $O
KB_DEBUG=1 timeout -k 10 300 python -u tools/cold.py --workload c5 --steps 1 > $O/cold_c5_dbg.txt 2>&1 || exit 1
KB_DEBUG=1 timeout -k 10 300 python -u tools/cold.py --workload c4 --steps 1 > $O/cold_c4_dbg.txt 2>&1 || exit 1
echo rc=$?
