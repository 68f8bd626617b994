# r04 g10: no table zeroing on the empty partition stack (C2 bench + parity
# subset), bitmap set/emit cycles on C3 (prof build)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4g10; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input"
timeout -k 10 300 python -u bench.py $NOX --steps 20 --warmup 5 > $O/c2.json 2> $O/c2.err && \
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu > $O/tests.txt 2>&1 && \
KB_LIB_PATH=genome-assembly_amd/lib/prof/libkbin.so KB_BIN_RANK=2 timeout -k 10 300 python -u bench.py $NOX --workload c3 --steps 1 --warmup 1 > $O/c3_r2.json 2> $O/c3_r2.err
echo rc=$?
