set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3u; mkdir -p $O
timeout -k 10 1100 python -u tools/unitig_time.py --reads 300000 1000000 --full-max 300000 --timeout 900 > $O/unitig.jsonl 2> $O/unitig.err || exit 1
echo rc=$?
