# scratch recipe for the current gpurun call (see tools/gpu.sh)
bash tools/gpu.sh test tests/test_gpu_parity.py tests/test_gpu_dist.py && \
timeout -k 10 600 python3 tools/cold.py --workload c5 --steps 2 > gpurun_out/cold_c5.txt 2>&1 && \
timeout -k 10 600 python3 tools/cold.py --workload c3 --steps 2 > gpurun_out/cold_c3.txt 2>&1 && \
timeout -k 10 300 python3 tools/cold.py --workload c2 --steps 3 > gpurun_out/cold_c2.txt 2>&1 && \
bash tools/gpu.sh bench c2 --cpu-sample 0 --steps 20
