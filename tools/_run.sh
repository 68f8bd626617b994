# scratch recipe for the current gpurun call (see tools/gpu.sh)
bash tools/gpu.sh test tests/test_gpu_parity.py -k "alphabet or streaming or dropin or host_cli or generator" && \
bash tools/gpu.sh bench host --cpu-sample 0 --steps 10 --host-input --dropin
