set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/b_ref.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --K 63 --read-len 250 --err-ppm 10000 --cpu-sample 0 > gpurun_out/b_k63.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --K 31 --read-len 250 --err-ppm 10000 --cpu-sample 0 > gpurun_out/b_k31e.log 2>&1
echo rc=$?
