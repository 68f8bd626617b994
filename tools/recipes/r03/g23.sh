set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3t; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_parity.py -k "dropin or host_cli" > $O/t.log 2>&1 || exit 1
timeout -k 10 1100 python -u tools/unitig_time.py --reads 20000 100000 1000000 --timeout 500 > $O/unitig.jsonl 2> $O/unitig.err || exit 1
echo rc=$?
