# round 3b: the id windows' stage loads, 8 in flight (product build) vs 4 in
# flight (lib/wl4, same code) vs HEAD (lib/ab_old), alternating; window parity
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3c8; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "random or large or offset or edge or ids or heavy or prefilter" > $O/test_quick.txt 2>&1 || exit 1
NOX="--cpu-sample 0 --no-capacity --no-host-input --steps 30 --warmup 5"
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py $NOX > $O/wl8_$i.json 2> $O/wl8_$i.err || exit 1
  KB_LIB_PATH=genome-assembly_amd/lib/wl4/libkbin.so timeout -k 10 200 python -u bench.py $NOX > $O/wl4_$i.json 2> $O/wl4_$i.err || exit 1
  KB_LIB_PATH=genome-assembly_amd/lib/ab_old/libkbin.so timeout -k 10 200 python -u bench.py $NOX > $O/old_$i.json 2> $O/old_$i.err || exit 1
done
echo rc=$?
