# r06 g2: the group-discard case (fixed oracle comparison); the drop-in at the
# reference's shipped M = 4 on C2's 20 K and 1 M reads, traced
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6g2; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v -m gpu --timeout 200 --timeout-method thread tests/test_gpu_dist.py \
    -k "discard" > $O/dist.txt 2>&1 || exit 1
timeout -k 10 900 python -u tools/unitig_time.py --reads 20000 1000000 --M 4 --full-max 0 --timeout 800 \
    > $O/unitig_m4.jsonl 2> $O/unitig_m4.err || exit 1
echo done
