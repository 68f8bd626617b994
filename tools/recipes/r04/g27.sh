# r04 g27: the long-list regime sizes context sub-bins at 40 % of a table (more
# bins ranked): ranked + capacity parity, C3 with digest (default knobs), C2
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4g27; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input"
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_capacity.py -m gpu > $O/tests.txt 2>&1 && \
timeout -k 10 300 python -u bench.py $NOX --workload c3 --steps 2 --warmup 2 --digest > $O/c3.json 2> $O/c3.err && \
timeout -k 10 300 python -u bench.py $NOX --steps 20 --warmup 5 > $O/c2.json 2> $O/c2.err
echo rc=$?
