# r05 g4: C5 share with context sub-bins to depth 5 (1025) in the light
# pre-filtered regime: C5 parity tests, then the C5 share bench (digest)
# new vs lib/ab_old, and the C4 share (digest) on the new build
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5g4; mkdir -p $O
T="python -u -m pytest -x -v -m gpu --timeout 900 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_capacity.py -k "c5" > $O/c5tests.txt 2>&1 || exit 1
timeout -k 10 500 python -u bench.py --cpu-sample 0 --workload c5 --steps 2 --warmup 2 --digest > $O/c5_new.json 2> $O/c5_new.err || exit 1
KB_LIB_PATH=genome-assembly_amd/lib/ab_old/libkbin.so timeout -k 10 500 python -u bench.py --cpu-sample 0 --workload c5 --steps 2 --warmup 2 --digest > $O/c5_old.json 2> $O/c5_old.err || exit 1
timeout -k 10 400 python -u bench.py --cpu-sample 0 --workload c4 --steps 2 --warmup 1 --digest > $O/c4_new.json 2> $O/c4_new.err || exit 1
echo done
