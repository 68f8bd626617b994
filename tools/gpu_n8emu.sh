# per-GPU receiver load at N ranks, emulated on one GPU: N M reads of the same
# genome in N mmer-partitioned passes (each pass ~ one rank's owned share)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python bench.py --reads 2000000 --parts 2 --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/b_emu2.log 2>&1 && \
timeout -k 10 200 python bench.py --reads 8000000 --parts 8 --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/b_emu8.log 2>&1
echo rc=$?
