# per-kernel durations of the C3 bench (rocprofv3 --kernel-trace --stats)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/kt3 -o kt3 --output-format csv -- python3 bench.py --workload c3 --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/kt3.log 2>&1
echo rc=$?
