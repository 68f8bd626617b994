# scratch recipe for the current gpurun call (see tools/gpu.sh)
bash tools/gpu.sh bench c2 --host-input --dropin && \
bash tools/gpu.sh ktrace c2 --steps 10 --warmup 3 && \
bash tools/gpu.sh pmc c2 --steps 4 --warmup 1 && \
KB_BIN_PF=0 bash tools/gpu.sh bench c5nopf --workload c5 --steps 1 --warmup 1 --digest --cpu-sample 0
