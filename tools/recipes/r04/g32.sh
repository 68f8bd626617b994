# r04 g32: ranked bins' long-list threshold A/B (lists above it take the
# bitmaps): 256 (product) vs 128 / 64 (lib/ab128, lib/ab64); parity on the
# A/B builds, C3 alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4g32; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input"
for v in 128 64; do
  KB_LIB_PATH=genome-assembly_amd/lib/ab$v/libkbin.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "ranked or large_lists or clustered_long" > $O/tests_$v.txt 2>&1 || exit 1
done
timeout -k 10 300 python -u bench.py $NOX --workload c3 --steps 2 --warmup 2 --digest > $O/c3_256.json 2> $O/c3_256.err || exit 1
for v in 128 64; do
  KB_LIB_PATH=genome-assembly_amd/lib/ab$v/libkbin.so timeout -k 10 300 python -u bench.py $NOX --workload c3 --steps 2 --warmup 2 --digest > $O/c3_$v.json 2> $O/c3_$v.err || exit 1
done
timeout -k 10 300 python -u bench.py $NOX --workload c3 --steps 2 --warmup 2 > $O/c3_256b.json 2> $O/c3_256b.err || exit 1
echo rc=$?
