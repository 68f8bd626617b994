# scratch recipe for the current gpurun call (see tools/gpu.sh)
bash tools/gpu.sh bench c5 --workload c5 --steps 3 --warmup 2 --cpu-sample 0 && \
bash tools/gpu.sh ktrace c5 --workload c5 --steps 2 --warmup 2
