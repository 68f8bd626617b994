set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c3k -o kt -- python3 bench.py --workload c3 --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/c3k.log 2>&1
echo rc=$?
