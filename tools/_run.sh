# scratch recipe for the current gpurun call (see tools/gpu.sh)
KB_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/bench_n2gloo.json 2> gpurun_out/bench_n2gloo.err && \
timeout -k 10 600 python bench.py --routed --steps 10 --warmup 2 --cpu-sample 0 > gpurun_out/bench_routed.json 2> gpurun_out/bench_routed.err
