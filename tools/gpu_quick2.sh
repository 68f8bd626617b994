# list/parity tests, then C2 and the N-rank emulation
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread -k "list or digest or random_vs or full_scale or heavy or edge" tests > gpurun_out/t_q.log 2>&1 || exit 1
bash tools/gpu_c2emu.sh
