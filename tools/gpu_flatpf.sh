set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread -k "heavy or split or partition or full_scale or two_word" tests > gpurun_out/t_fp.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --workload c3 --steps 2 --warmup 1 --digest --cpu-sample 0 > gpurun_out/b_fp3.log 2>&1 && \
timeout -k 10 300 python bench.py --reads 8000000 --genome 40000000 --parts 8 --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/b_fp8.log 2>&1 && \
timeout -k 10 300 python bench.py --cpu-sample 0 > gpurun_out/b_fp2.log 2>&1
echo rc=$?
