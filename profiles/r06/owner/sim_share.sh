# r06: one rank's share of the N-GPU C2 weak-scaling run (1/N of the mmers of
# N x 1 M reads of an N x 5 Mbp genome), binned per rank on one GPU through a
# virtual-shard group: the per-rank compute the driver's 2/4/8-GPU runs time
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/sim_share; mkdir -p $O
timeout -k 10 600 python -u tools/sim_rank_share.py --ranks 1 2 4 8 --steps 3 > $O/share.jsonl 2> $O/share.err || exit 1
echo done
