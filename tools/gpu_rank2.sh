# bench.py's N>1 path (pipelined units) rehearsed with 2 ranks on one GPU (gloo exchange)
set -o pipefail
cd $GRAFT_REPO_ROOT
KB_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 2 > gpurun_out/b_rank2.log 2>&1 && \
KB_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 3 --warmup 2 --no-pipeline > gpurun_out/b_rank2np.log 2>&1
echo rc=$?
