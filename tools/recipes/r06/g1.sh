# r06 g1: the unitig replay on the GPU box -- kbin_main --unitigs and the
# drop-in (find_kmer_extensions replaced) against every unitigs.json golden;
# the new group-discard and K < 2M cases; then the drop-in at the reference's
# shipped M = 4 on C2's 20 K and 1 M reads (the extension live), traced
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6g1; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    -k "unitigs or dropin or k_below_2m or host_cli" > $O/parity.txt 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -x -v -m gpu --timeout 200 --timeout-method thread tests/test_gpu_dist.py \
    -k "discard" > $O/dist.txt 2>&1 || exit 1
timeout -k 10 900 python -u tools/unitig_time.py --reads 20000 1000000 --M 4 --full-max 0 --timeout 800 \
    > $O/unitig_m4.jsonl 2> $O/unitig_m4.err || exit 1
echo done
