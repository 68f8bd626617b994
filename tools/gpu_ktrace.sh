# per-kernel durations of the bench (rocprofv3 --kernel-trace --stats), engine from $KB_ENGINE
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt -o kt --output-format csv -- python3 bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/kt.log 2>&1
echo rc=$?
