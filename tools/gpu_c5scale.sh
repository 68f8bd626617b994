# C5 per-GPU share: where does the time go at scale (per-pass size vs passes)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u bench.py --workload c5 --reads 16000000 --parts 1 --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/c5_16m_p1.log 2>&1 && \
timeout -k 10 300 python -u bench.py --workload c5 --reads 32000000 --parts 2 --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/c5_32m_p2.log 2>&1 && \
timeout -k 10 300 python -u bench.py --workload c5 --parts 8 --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/c5_p8.log 2>&1
echo rc=$?
