# round 3b: record-pass plan cache + kernel-only timing in the timed steps (new),
# the same with every phase event (new --timing-all), the tail-deferral build
# (lib/ab_old); the -m gpu suite; the prof build's phase counters
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3b3; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input --steps 30 --warmup 5"
for i in 1 2; do
  timeout -k 10 200 python -u bench.py $NOX > $O/new$i.json 2> $O/new$i.err || exit 1
  timeout -k 10 200 python -u bench.py $NOX --timing-all > $O/newall$i.json 2> $O/newall$i.err || exit 1
  KB_LIB_PATH=genome-assembly_amd/lib/ab_old/libkbin.so timeout -k 10 200 python -u bench.py $NOX > $O/old$i.json 2> $O/old$i.err || exit 1
done
KB_LIB_PATH=genome-assembly_amd/lib/prof/libkbin.so timeout -k 10 200 python -u bench.py --cpu-sample 0 --no-capacity --no-host-input --steps 5 --warmup 2 > $O/prof.json 2> $O/prof.err || exit 1
timeout -k 10 1500 python -u -m pytest -x -v -m gpu --timeout 900 --timeout-method thread tests > $O/gpu_tests.txt 2>&1 || exit 1
echo rc=$?
