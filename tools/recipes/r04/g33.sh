# r04 g33: ranked bins A/B -- long lists over 32 ids (lib/abL32) and ranking
# from 256 records (lib/abM256) against the product (64, 512): parity on the
# A/B builds, C3 alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4g33; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input"
for v in L32 M256; do
  KB_LIB_PATH=genome-assembly_amd/lib/ab$v/libkbin.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "ranked or large_lists or clustered_long" > $O/tests_$v.txt 2>&1 || exit 1
done
for r in 1 2; do
  timeout -k 10 300 python -u bench.py $NOX --workload c3 --steps 2 --warmup 2 --digest > $O/c3_prod_$r.json 2> $O/c3_prod_$r.err || exit 1
  for v in L32 M256; do
    KB_LIB_PATH=genome-assembly_amd/lib/ab$v/libkbin.so timeout -k 10 300 python -u bench.py $NOX --workload c3 --steps 2 --warmup 2 --digest > $O/c3_${v}_$r.json 2> $O/c3_${v}_$r.err || exit 1
  done
done
echo rc=$?
