set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pfk -o kt -- python3 bench.py --reads 8000000 --genome 40000000 --parts 8 --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/pfk.log 2>&1
echo rc=$?
