set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread -k "list or digest or random_vs or full_scale or heavy or edge or known" tests > gpurun_out/t_q.log 2>&1 || exit 1
KB_LIB_PATH=genome-assembly_amd/lib/prof/libkbin.so timeout -k 10 200 python bench.py --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/lprof.log 2>&1 || exit 1
bash tools/gpu_c2emu.sh
