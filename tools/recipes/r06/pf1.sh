# r06 A/B: bin descriptors prefetched a bin ahead (KB_DESC_PF=1, default) vs
# loaded after the claim (lib/nopf, -DKB_DESC_PF=0): parity suites, C3 digest, C2
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/pf1; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input --steps 20 --warmup 3"
L=genome-assembly_amd/lib
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_scale.py tests/test_gpu_parity.py tests/test_gpu_race.py > $O/tests.txt 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --cpu-sample 0 --workload c3 --steps 3 --warmup 1 --digest > $O/c3_pf.json 2>> $O/err.txt || exit 1
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py $NOX > $O/pf_$i.json 2>> $O/err.txt || exit 1
  KB_LIB_PATH=$L/nopf/libkbin.so timeout -k 10 300 python -u bench.py $NOX > $O/nopf_$i.json 2>> $O/err.txt || exit 1
done
echo done
