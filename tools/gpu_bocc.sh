set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > gpurun_out/t_all.log 2>&1 || exit 1
for i in 1 2; do timeout -k 10 300 python bench.py --cpu-sample 0 --steps 20 > gpurun_out/b_bo$i.log 2>&1 || exit 1; done
KB_LIB_PATH=genome-assembly_amd/lib/prof/libkbin.so timeout -k 10 200 python bench.py --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/lprof.log 2>&1
echo rc=$?
