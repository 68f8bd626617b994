set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c2k -o kt -- python3 bench.py --steps 5 --warmup 1 --cpu-sample 0 > gpurun_out/c2k.log 2>&1 || exit 1
KB_LIB_PATH=genome-assembly_amd/lib/prof/libkbin.so timeout -k 10 200 python bench.py --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/c2bp.log 2>&1
echo rc=$?
