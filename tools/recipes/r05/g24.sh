# r05 g24: the edge split by its b - 1 bases before the mmer: the whole GPU suite
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5g24; mkdir -p $O
timeout -k 10 1100 python -u -m pytest -x -q -m gpu --timeout 900 --timeout-method thread tests > $O/gpu_suite.txt 2>&1 || exit 1
echo done
