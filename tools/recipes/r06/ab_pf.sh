# r06 A/B: (pf) bin_kernel claims two bins ahead and loads the next bin's
# descriptor during this one; (both) + the record walk's argmax in 32-bit
# halves (bit-field extracts, both orientations in one max3); against the
# round's tree (base).  C2 bench alternating on one box, then the parity suite
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/ab_pf; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input --steps 20 --warmup 3"
L=genome-assembly_amd/lib
for i in 1 2 3; do
  KB_LIB_PATH=$L/base/libkbin.so timeout -k 10 300 python -u bench.py $NOX > $O/base$i.json 2>> $O/err.txt || exit 1
  KB_LIB_PATH=$L/pf/libkbin.so timeout -k 10 300 python -u bench.py $NOX > $O/pf$i.json 2>> $O/err.txt || exit 1
  timeout -k 10 300 python -u bench.py $NOX > $O/both$i.json 2>> $O/err.txt || exit 1
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py > $O/parity.txt 2>&1 || exit 1
echo done
