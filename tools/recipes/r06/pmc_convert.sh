# r06: SQ and TCC counters of C3's kernels (one step): where the received-
# record conversion (sk_convert_buckets_kernel) spends its wave cycles
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/pmc_convert; mkdir -p $O
B="python3 bench.py --workload c3 --steps 1 --warmup 0 --cpu-sample 0"
timeout -s KILL 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES --output-format csv -d $O/sq -o sq -- $B > $O/sq.log 2>&1 || exit 1
timeout -s KILL 400 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d $O/tcc -o tcc -- $B > $O/tcc.log 2>&1 || exit 1
timeout -s KILL 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- $B > $O/kt.log 2>&1 || exit 1
echo done
