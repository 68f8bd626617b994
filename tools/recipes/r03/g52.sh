# round 3b closing check on the committed tree (traffic.json capacity tags
# regenerated): smoke and the default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3z4; mkdir -p $O
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > $O/c2_bench.json 2> $O/c2_bench.err || exit 1
echo rc=$?
