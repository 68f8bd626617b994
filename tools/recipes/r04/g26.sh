# r04 g26: bank-conflict-free emission tile (lane l at 33 l): parity, C3, prof C3
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4g26; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input"
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "ranked or large_lists or clustered_long" > $O/tests.txt 2>&1 && \
timeout -k 10 300 python -u bench.py $NOX --workload c3 --steps 2 --warmup 1 --digest > $O/c3.json 2> $O/c3.err && \
KB_LIB_PATH=genome-assembly_amd/lib/prof/libkbin.so KB_BIN_RANK=2 timeout -k 10 300 python -u bench.py $NOX --workload c3 --steps 1 --warmup 1 > $O/c3_r2.json 2> $O/c3_r2.err
echo rc=$?
