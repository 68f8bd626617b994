# quick check: binned parity first (stops at the first failure), then prof counters + bench
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -m pytest tests -x -q -m gpu -k "parity and binned" > gpurun_out/t_par.log 2>&1 && \
KB_LIB_PATH=genome-assembly_amd/lib/prof/libkbin.so timeout -k 10 200 python bench.py --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/prof0.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 10 --warmup 3 --cpu-sample 0 > gpurun_out/b_v2.log 2>&1
echo rc=$?
