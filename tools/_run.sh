# scratch recipe for the current gpurun call (see tools/gpu.sh)
for i in 1 2; do
KB_LIB_PATH=genome-assembly_amd/lib/ab/libkbin.so bash tools/gpu.sh bench old$i --cpu-sample 0 --steps 20 --input replay && \
KB_BIN_DESC=0 bash tools/gpu.sh bench nodesc$i --cpu-sample 0 --steps 20 --input replay && \
bash tools/gpu.sh bench new$i --cpu-sample 0 --steps 20 --input replay || exit 1
done
bash tools/gpu.sh test tests/test_gpu_parity.py tests/test_gpu_dist.py
