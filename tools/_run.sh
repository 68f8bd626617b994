# scratch recipe for the current gpurun call (see tools/gpu.sh)
bash tools/gpu.sh sq c2 --steps 3 --warmup 1 && \
KB_BIN_LDS_LISTS=1 bash tools/gpu.sh sq c2lds --steps 3 --warmup 1 && \
bash tools/gpu.sh pmc c2 --steps 4 --warmup 1 && \
bash tools/gpu.sh ktrace c2 --steps 10 --warmup 3 && \
bash tools/gpu.sh bench c2 && \
for w in 100 80; do KB_BIN_LDS_LISTS=1 KB_BIN_WIN_PCT=$w KB_LIB_PATH=genome-assembly_amd/lib/prof/libkbin.so timeout -k 10 300 python bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/prof_lds$w.json 2> gpurun_out/prof_lds$w.err || exit 1; done
