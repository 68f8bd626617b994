# A/B on the GPU box: parity on both engines, then the C2 bench per engine
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -m pytest tests -x -q -m gpu -k "parity" > gpurun_out/t_par.log 2>&1 && \
KB_ENGINE=binned timeout -k 10 200 python bench.py --steps 10 --warmup 3 --cpu-sample 0 > gpurun_out/b_v2.log 2>&1 && \
KB_ENGINE=table timeout -k 10 200 python bench.py --steps 10 --warmup 3 --cpu-sample 0 > gpurun_out/b_v1.log 2>&1
echo rc=$?
