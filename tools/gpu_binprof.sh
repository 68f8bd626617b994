# diagnostic: bin-kernel phase counters + LDS table size sweep (stderr/stdout -> gpurun_out)
set -o pipefail
cd $GRAFT_REPO_ROOT
KB_ENGINE=binned KB_LIB_PATH=genome-assembly_amd/lib/prof/libkbin.so timeout -k 10 200 python bench.py --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/prof.log 2>&1 && \
for t in 12 13; do KB_ENGINE=binned KB_BIN_TS_LOG2=$t timeout -k 10 200 python bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/ts$t.log 2>&1 || exit 1; done
echo done
