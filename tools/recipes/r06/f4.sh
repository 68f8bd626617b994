# r06 evidence 4 (after kb_owner_table): the full GPU suite and smoke, the
# default bench line, the routed one-rank line and the full-size legs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6f4; mkdir -p $O
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > $O/c2_bench.json 2> $O/c2_bench.err || exit 1
timeout -k 10 300 python -u bench.py --cpu-sample 0 --no-capacity --no-host-input --routed --steps 20 --warmup 3 > $O/routed.json 2> $O/routed.err || exit 1
echo done
