# in-kernel phase counters of the bin kernel: C2 vs the N=2 / N=8 receiver emulation
set -o pipefail
cd $GRAFT_REPO_ROOT
for w in "--reads 1000000 --parts 1" "--reads 2000000 --parts 2" "--reads 8000000 --parts 8"; do
  echo "== $w" >> gpurun_out/binprof2.txt
  KB_LIB_PATH=genome-assembly_amd/lib/prof/libkbin.so timeout -k 10 200 python bench.py $w --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/bp.log 2>&1 || exit 1
  grep bin_prof gpurun_out/bp.log | tail -3 >> gpurun_out/binprof2.txt
done
echo rc=$?
