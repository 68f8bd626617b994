# SQ counters of the binned engine's kernels (two separate --pmc passes, no tracing)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
KB_ENGINE=binned timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT -d gpurun_out/pmc1 -o pmc -- python3 bench.py --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/pmc1.log 2>&1 && \
KB_ENGINE=binned timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_BRANCH SQ_INSTS_SMEM -d gpurun_out/pmc2 -o pmc -- python3 bench.py --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/pmc2.log 2>&1
echo rc=$?
