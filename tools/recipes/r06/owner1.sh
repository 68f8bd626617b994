# r06: owner(mmer) from kb_owner_table (LPT over the prior, per pass): the
# distributed and capacity GPU suites, the C4 scale tests, then one rank's
# share at N = 1..8 (records per rank, the heaviest rank binned alone)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/owner1; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_dist.py tests/test_gpu_capacity.py > $O/tests.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_scale.py -k "c4" > $O/scale_tests.txt 2>&1 || exit 1
timeout -k 10 600 python -u tools/sim_rank_share.py --ranks 1 2 4 8 --steps 4 > $O/share.jsonl 2> $O/share.err || exit 1
echo done
