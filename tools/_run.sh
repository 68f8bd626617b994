# scratch recipe for the current gpurun call (see tools/gpu.sh)
bash tools/gpu.sh bench base --cpu-sample 0 --steps 20 && \
KB_BIN_LDS_LISTS=1 bash tools/gpu.sh bench lds100 --cpu-sample 0 --steps 20 && \
KB_BIN_LDS_LISTS=1 KB_BIN_WIN_PCT=80 bash tools/gpu.sh bench lds80 --cpu-sample 0 --steps 20 && \
KB_BIN_LDS_LISTS=1 KB_BIN_WIN_PCT=60 bash tools/gpu.sh bench lds60 --cpu-sample 0 --steps 20 && \
KB_BIN_LDS_LISTS=1 bash tools/gpu.sh test tests/test_gpu_parity.py -k "not dropin" && \
bash tools/gpu.sh bench cpu --steps 5
