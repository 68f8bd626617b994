# r04 g21: drop-in with the list-node arena: byte-identity tests (every
# drop-in binary, multi-GPU), the C2-shape wall time with its phase split
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4g21; mkdir -p $O
NCCL_DEBUG=WARN timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_dist.py \
  -k "dropin or host_cli" -m gpu > $O/dropin_tests.txt 2>&1 && \
timeout -k 10 400 python -u tools/unitig_time.py --reads 1000000 --full-max 0 --timeout 380 > $O/unitig_c2.jsonl 2> $O/unitig_c2.err
echo rc=$?
