# r06: the N > 1 run's C4 / C5 legs over two gloo ranks on one GPU through the
# C group (host transport), at 1/40 of their reads: per-pass owner tables at
# G = 2 through the partitioned legs, at a scale past the test's 1/400
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/legs_gloo40; mkdir -p $O
KB_DIST_BACKEND=gloo KB_CAPACITY_SCALE=40 KB_ROUTED_TRANSPORT=c timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 2 > $O/line.json 2> $O/err.txt || exit 1
echo done
