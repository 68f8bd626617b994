# r06 closing check on the final tree (product code as in f5a/f5b; the prof
# build's accumulators moved to LDS): GPU suite, smoke, then C5 share phase
# counters with the LDS-accumulator prof build (prices the heavy windows)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/f6; mkdir -p $O
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || exit 1
KB_LIB_PATH=genome-assembly_amd/lib/prof/libkbin.so timeout -k 10 500 python -u bench.py --cpu-sample 0 --workload c5 --steps 1 --warmup 1 > $O/c5_prof.json 2> $O/c5_prof.err || exit 1
echo done
