# round 3b: the N-rank bench path rehearsed as two gloo ranks on one GPU
# (bench.py under torch.distributed.run: the timing decision all-reduced, the
# phase step, replay and the one JSON line), then the -m gpu suite
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3c7; mkdir -p $O
KB_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 2 > $O/ranks2.json 2> $O/ranks2.err || exit 1
timeout -k 10 1500 python -u -m pytest -x -q -m gpu --timeout 900 --timeout-method thread tests > $O/gpu_tests.txt 2>&1 || exit 1
echo rc=$?
