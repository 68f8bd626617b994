# diagnostic: bin-kernel phase counters, C5 share at 32M reads in two passes
set -o pipefail
cd $GRAFT_REPO_ROOT
KB_LIB_PATH=genome-assembly_amd/lib/prof/libkbin.so timeout -k 10 400 python -u bench.py --workload c5 --reads 32000000 --parts 2 --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/c5diag2.log 2>&1
echo rc=$?
