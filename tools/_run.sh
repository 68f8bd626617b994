# scratch recipe for the current gpurun call (see tools/gpu.sh)
for ab in 0 1 2; do
KB_BIN_ABLATE=$ab KB_LIB_PATH=genome-assembly_amd/lib/prof/libkbin.so timeout -k 10 300 python bench.py --steps 5 --warmup 2 --cpu-sample 0 --input replay > gpurun_out/prof_ab$ab.json 2> gpurun_out/prof_ab$ab.err || exit 1
done
