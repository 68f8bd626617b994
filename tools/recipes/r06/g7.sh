# r06 g7: the whole GPU suite on the tree after the unitig replay, the K < 2M
# widening (complement flag, long reads) and the group capacity fix; smoke
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6g7; mkdir -p $O
timeout -k 10 1100 python -u -m pytest -x -v -m gpu --timeout 600 --timeout-method thread tests > $O/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 1
echo done
