# heavy-bin changes: parity (heavy/split/partition), C2 + N-rank emulation benches, bin phase counters at N=8
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread -k "heavy or split or partition or full_scale" tests > gpurun_out/t_h.log 2>&1 || exit 1
bash tools/gpu_c2emu.sh || exit 1
KB_LIB_PATH=genome-assembly_amd/lib/prof/libkbin.so timeout -k 10 200 python bench.py --reads 8000000 --parts 8 --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/bp8.log 2>&1
echo rc=$?
