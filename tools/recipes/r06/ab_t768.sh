# r06 A/B: bin_kernel with 768-thread workgroups (12 waves: 145 VGPRs, no
# spills) and the same 8192-slot tables, against 1024 threads (128 VGPRs, 13
# spilled); C2 bench alternating, then the parity suite on the 768 build
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/ab_t768; mkdir -p $O
NOX="--cpu-sample 0 --no-capacity --no-host-input --steps 20 --warmup 3"
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py $NOX > $O/a$i.json 2>> $O/err.txt || exit 1
  KB_LIB_PATH=genome-assembly_amd/lib/t768/libkbin.so timeout -k 10 300 python -u bench.py $NOX > $O/b$i.json 2>> $O/err.txt || exit 1
done
KB_LIB_PATH=genome-assembly_amd/lib/t768/libkbin.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py > $O/parity_t768.txt 2>&1
echo "parity rc=$?"
echo done
