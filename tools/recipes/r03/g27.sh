# round-3 state: the full GPU suite, smoke, the default bench line (capacity and
# host-input legs on), the N-receiver emulations
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3y; mkdir -p $O
timeout -k 10 1500 python -u -m pytest -x -v -m gpu --timeout 900 --timeout-method thread tests > $O/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > $O/c2_bench.json 2> $O/c2_bench.err || exit 1
NOX="--cpu-sample 0 --no-capacity --no-host-input --steps 5 --warmup 2"
for n in 2 4 8; do
  timeout -k 10 300 python -u bench.py $NOX --reads ${n}000000 --genome $((5 * n))000000 --parts $n > $O/zs$n.json 2> $O/zs$n.err || exit 1
done
echo rc=$?
# A/B: 512-thread bins with 4096-slot tables (two workgroups per CU), sub-bins sized for them
NOX="--cpu-sample 0 --no-capacity --no-host-input --steps 20 --warmup 5"
timeout -k 10 200 python -u bench.py $NOX > $O/ab_base.json 2> $O/ab_base.err || exit 1
for f in 40 30 60; do
  KB_LIB_PATH=genome-assembly_amd/lib/t512/libkbin.so KB_BIN_TS_LOG2=12 KB_BIN_SUB_FILL_PCT=$f timeout -k 10 200 python -u bench.py $NOX > $O/ab_t512_f$f.json 2> $O/ab_t512_f$f.err || exit 1
done
echo rc=$?
