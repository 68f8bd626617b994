# the C5 per-GPU share (62.5M x 250 bp, K63, 1 % errors, 4 passes), phase counters per pass
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 170 python -u bench.py --workload c5 --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/b_c5.log 2>&1 && \
KB_LIB_PATH=genome-assembly_amd/lib/prof/libkbin.so timeout -k 10 170 python -u bench.py --workload c5 --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/b_c5_prof.log 2>&1
echo rc=$?
