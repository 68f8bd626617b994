# r06 evidence 5a (final tree: bucket ordering 8 records in flight, record-pass row loads batched):
# pieces): full GPU suite and smoke, the default bench line, C2 kernel trace
# + stats and FETCH_SIZE / WRITE_SIZE passes, C3 / C4 share / C5 share with
# digests, the routed one-rank line, the N > 1 legs through a one-rank group
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6f5a; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input"
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > $O/c2_bench.json 2> $O/c2_bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 bench.py $NOX --steps 20 --warmup 3 > $O/kt.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o pmc -- python3 bench.py $NOX --steps 5 --warmup 2 > $O/pmc_fetch.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o pmc -- python3 bench.py $NOX --steps 5 --warmup 2 > $O/pmc_write.log 2>&1 || exit 1
echo done
