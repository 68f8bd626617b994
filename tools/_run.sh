# scratch recipe for the current gpurun call (see tools/gpu.sh)
for i in 1 2; do
KB_LIB_PATH=genome-assembly_amd/lib/ab/libkbin.so bash tools/gpu.sh bench old$i --cpu-sample 0 --steps 20 --input replay && \
bash tools/gpu.sh bench new$i --cpu-sample 0 --steps 20 --input replay || exit 1
done
bash tools/gpu.sh test tests/test_gpu_parity.py -k "prefilter or heavy or split or c2 or golden"
