set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3o
bash tools/gpu.sh ktrace c5n --workload c5 --steps 1 --warmup 1 --no-capacity --no-host-input || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3o/coldkt -o kt -- python3 tools/cold.py --workload c2 --steps 3 --prewarm 2000 > gpurun_out/r3o/coldkt.log 2>&1 || exit 1
echo rc=$?
