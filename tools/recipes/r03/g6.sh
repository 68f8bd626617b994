set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3e; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input"
timeout -k 10 1200 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log
[ $rc -eq 0 ] || exit $rc
KB_DEBUG=1 timeout -k 10 120 python -u tools/cold.py --workload c2 --steps 4 > $O/cold_c2.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --cpu-sample 0 --steps 20 --warmup 5 > $O/c2.json 2> $O/c2.err && \
timeout -k 10 300 python -u bench.py $NOX --reads 8000000 --genome 40000000 --parts 8 --steps 4 --warmup 2 > $O/zs8.json 2> $O/zs8.err && \
timeout -k 10 300 python -u bench.py $NOX --reads 2000000 --genome 10000000 --parts 2 --steps 4 --warmup 2 > $O/zs2.json 2> $O/zs2.err && \
timeout -k 10 300 python -u bench.py $NOX --reads 4000000 --genome 20000000 --parts 4 --steps 4 --warmup 2 > $O/zs4.json 2> $O/zs4.err
echo rc=$?
