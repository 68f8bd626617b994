# two-word binned engine: new tests first, then the whole GPU suite and benches
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "two_word or heavy" > gpurun_out/t_kw2.log 2>&1 && \
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/t_all.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-sample 0 > gpurun_out/b_c2.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --K 63 --read-len 250 --err-ppm 10000 --cpu-sample 0 > gpurun_out/b_k63.log 2>&1
echo rc=$?
