set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3m; mkdir -p $O
timeout -k 10 1000 python -u -m pytest -x -v --timeout 900 --timeout-method thread tests/test_gpu_capacity.py tests/test_gpu_scale.py::test_c2_full_vs_oracle > $O/t.log 2>&1 || exit 1
echo rc=$?
