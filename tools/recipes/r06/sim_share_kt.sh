# r06: kernel trace of one rank's share at N = 1 and N = 8 (tools/sim_rank_share.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/sim_share_kt; mkdir -p $O
for g in 1 8; do
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/kt$g -o kt -- python3 tools/sim_rank_share.py --ranks $g --steps 3 > $O/share$g.jsonl 2> $O/share$g.err || exit 1
done
echo done
