# round 3b: edge/timing/tail tests first; current build vs the tail-deferral
# commit (lib/ab_old); bucket_kernel ablations (lib/abl, replay input); suite
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3b5; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v -m gpu --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "edge_inputs or timing or deferred" > $O/test_edge.txt 2>&1 || exit 1
NOX="--cpu-sample 0 --no-capacity --no-host-input --steps 30 --warmup 5"
for i in 1 2; do
  timeout -k 10 200 python -u bench.py $NOX > $O/new$i.json 2> $O/new$i.err || exit 1
  KB_LIB_PATH=genome-assembly_amd/lib/ab_old/libkbin.so timeout -k 10 200 python -u bench.py $NOX > $O/old$i.json 2> $O/old$i.err || exit 1
done
for m in 0 1 2; do
  KB_LIB_PATH=genome-assembly_amd/lib/abl/libkbin.so KB_BK_ABLATE=$m timeout -k 10 200 python -u bench.py $NOX --input replay > $O/bk$m.json 2> $O/bk$m.err || exit 1
done
timeout -k 10 1500 python -u -m pytest -x -q -m gpu --timeout 900 --timeout-method thread tests > $O/gpu_tests.txt 2>&1 || exit 1
echo rc=$?
