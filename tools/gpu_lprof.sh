set -o pipefail
cd $GRAFT_REPO_ROOT
KB_LIB_PATH=genome-assembly_amd/lib/prof/libkbin.so timeout -k 10 200 python bench.py --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/lprof.log 2>&1
echo rc=$?
