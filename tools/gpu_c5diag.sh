# diagnostic: bin-kernel phase counters on a reduced C5 (8M x 250 bp, K63, 1 % errors, one pass)
set -o pipefail
cd $GRAFT_REPO_ROOT
KB_LIB_PATH=genome-assembly_amd/lib/prof/libkbin.so timeout -k 10 300 python -u bench.py --workload c5 --reads 8000000 --parts 1 --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/c5diag.log 2>&1 && \
KB_BIN_FLAT_L=0 timeout -k 10 300 python -u bench.py --workload c5 --reads 8000000 --parts 1 --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/c5diag_noflat.log 2>&1
echo rc=$?
