# diagnostic: bin-kernel phase counters (prof build), ablations 0/1/2
set -o pipefail
cd $GRAFT_REPO_ROOT
for a in 0 1 2; do
KB_BIN_ABLATE=$a KB_LIB_PATH=genome-assembly_amd/lib/prof/libkbin.so timeout -k 10 200 python bench.py --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/prof_a$a.log 2>&1 || exit 1
done
echo done
