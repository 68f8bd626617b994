# round 3b: the deferred-tail surprise test; C2 kernel trace (gaps between a step's kernels)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3b2; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v -m gpu --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "deferred_tail" > $O/test_tail.txt 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 bench.py --cpu-sample 0 --no-capacity --no-host-input --steps 10 --warmup 3 > $O/kt.log 2>&1 || exit 1

KB_LIB_PATH=genome-assembly_amd/lib/prof/libkbin.so timeout -k 10 200 python -u bench.py --cpu-sample 0 --no-capacity --no-host-input --steps 5 --warmup 2 > $O/prof.json 2> $O/prof.err || exit 1

echo rc=$?
