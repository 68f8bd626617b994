# r06 g4: K < 2M routed (complement flag in routed records): split passes,
# scatter, plan/pack, groups; the routing tests whose record bytes changed
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6g4; mkdir -p $O
timeout -k 10 900 python -u -m pytest -v -m gpu --timeout 300 --timeout-method thread tests/test_gpu_dist.py \
    > $O/dist.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    -k "k_below_2m" > $O/parity.txt 2>&1 || exit 1
echo done
