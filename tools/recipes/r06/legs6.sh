# r06: after the exchange fix (self records by device copy, peer messages in
# 256-MB pieces) and GroupBinner.rec_words: the distributed GPU suite, then
# the N > 1 run's C4 and C5 legs at full per-rank size through a one-rank
# RCCL group (bench.py --routed --multi-legs), the driver's leg settings
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/legs6; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_dist.py > $O/dist_tests.txt 2>&1 || exit 1
timeout -k 10 900 python -u bench.py --routed --multi-legs --steps 10 --warmup 2 --cpu-sample 0 --no-host-input > $O/legs.json 2> $O/legs.err || exit 1
echo done
